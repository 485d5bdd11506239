"""Linear layers of the detector head (fusion, PN-BiMamba, pooling, classifier) with their weight gradients
accumulated in fp32 straight into .grad.

Under autocast an nn.Linear's backward computes the input gradient, the bf16 weight gradient (a long-K GEMM
with a tiny output: [144 x 576] over the 1608 / 6432 token rows), its fp32 cast, the bias reduction and its
cast, and then the trainer adds both into the flat fp32 gradient buffer. Here the weight gradient is ONE GEMM
with bf16 operands and an fp32 output accumulated in place (beta = 1, torch's addmm out_dtype form) and the
bias gradient one fp32 reduction added in place: no bf16 rounding of the weight gradient, no casts, no separate
accumulation (RADHIP_SIDE_LINEAR=1 puts these on a side stream joined at the end of the backward: a parallel
branch of the captured graphs, measured 3 % slower per step than the main stream on ROCm 7; =0: F.linear).

Same math as F.linear under autocast (src/models/DualStreamSEMamba.py:445-531,537-637,700-770): the input
and weight are cast to the autocast dtype, y = x W^T + b. The direct accumulation needs .grad to exist (the
trainers' FlatGrads buffers); without it the gradients are returned to autograd as usual.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops

_SIDE = {}
_JOIN_QUEUED = [False]


def _side(device):
    d = device.index if device.index is not None else torch.cuda.current_device()
    if d not in _SIDE:
        _SIDE[d] = torch.cuda.Stream(device=d)
    return _SIDE[d]


def _join(device):
    def cb():
        _JOIN_QUEUED[0] = False
        torch.cuda.current_stream(device).wait_stream(_side(device))
    return cb


def _cast(t, dt):
    """t in dtype dt; fp32 parameters go through the window's weight-cast cache (radhip/window.py: the
    clean pass casts, the window's adversarial passes reuse; the parameters do not change within a window)."""
    if t is None or t.dtype == dt:
        return t
    cache = ops.SCONV_WCACHE
    if cache is not None and isinstance(t, nn.Parameter):
        hit = cache.get(("lin", id(t), dt))
        if hit is not None and hit[0] is t and hit[1].dtype == dt:
            return hit[1]
        c = t.to(dt)
        cache[("lin", id(t), dt)] = (t, c)
        return c
    return t.to(dt)


def _cast_t(weight, wc):
    """wc^T contiguous ([in, out]: the input-gradient GEMM's weight operand), through the window's cast cache like
    _cast (the parameters do not change within a window)."""
    cache = ops.SCONV_WCACHE
    if cache is not None and isinstance(weight, nn.Parameter):
        key = ("linT", id(weight), wc.dtype)
        hit = cache.get(key)
        if hit is not None and hit[0] is weight and hit[1].dtype == wc.dtype:
            return hit[1]
        c = wc.t().contiguous()
        cache[key] = (weight, c)
        return c
    return wc.t().contiguous()


LG_MAX_K = 320     # csrc/lgemm.hip stages K <= 320 in one LDS chunk; its per-CU operand ingest loses to hipBLASLt above


def _lg_ok(t, K):
    """csrc/lgemm.hip for a plain (unfused) head GEMM with contraction length K."""
    return _LGEMM and t.is_cuda and t.dtype in ops.HALF and K <= LG_MAX_K


def _rows(t):
    """t as a 2-D [rows, last] view (no copy when the leading dimensions collapse), unit inner stride."""
    t2 = t.reshape(-1, t.shape[-1])
    M, K = t2.shape
    if (K > 1 and t2.stride(-1) != 1) or (M > 1 and t2.stride(0) < K):   # e.g. an expanded [M, 1] gradient
        t2 = t2.clone(memory_format=torch.contiguous_format)
    return t2


def direct_grad(p):
    """True for parameters whose gradient SideLinear accumulates into .grad itself (window.py keeps their
    .grad bound during a pass instead of handing it over through autograd)."""
    return getattr(p, "_radhip_direct_grad", False)


class SideLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dt):
        xc, wc, bc = x.to(dt), _cast(weight, dt), _cast(bias, dt)
        if _lg_ok(xc, wc.shape[1]):
            # csrc/lgemm.hip at K <= 320 (3.5-5 us in a graph vs hipBLASLt's 4.4-6.5; longer K stays on hipBLASLt:
            # tools/bench_lgemm.py, profiles/r05_bench_lgemm.jsonl)
            y = torch.empty(*xc.shape[:-1], wc.shape[0], device=xc.device, dtype=dt)   # not a view: in-place
            ops.lgemm(_rows(xc), wc, bc, out=y.view(-1, wc.shape[0]))                  # consumers (SE's ReLU)
        else:
            y = F.linear(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.x_dtype = x.dtype
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        weight, bias = ctx.params
        dy = dy.to(wc.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            if _lg_ok(dy, wc.shape[0]):
                dx = ops.lgemm(_rows(dy), _cast_t(weight, wc),
                               out_dtype=torch.float32 if ctx.x_dtype == torch.float32 else None)
                dx = dx.to(ctx.x_dtype).view(*dy.shape[:-1], wc.shape[1])
            else:
                dx = torch.matmul(dy, wc).to(ctx.x_dtype)
        need_w, need_b = ctx.needs_input_grad[1], bias is not None and ctx.needs_input_grad[2]
        gw, gb = _weight_grads(dy.reshape(-1, dy.shape[-1]), xc.reshape(-1, xc.shape[-1]), weight, bias, need_w, need_b)
        return dx, gw, gb, None


def _weight_grads(dy2, x2, weight, bias, need_w, need_b):
    """The linear's weight / bias gradients from dy2 [M, N] and x2 [M, K]: accumulated in fp32 straight into .grad
    when it is bound (returns None, None), else returned for autograd."""
    direct = (dy2.is_cuda and need_w and weight.grad is not None and weight.grad.dtype == torch.float32
              and (not need_b or (bias.grad is not None and bias.grad.dtype == torch.float32)))
    if not direct:
        gw = torch.matmul(dy2.t(), x2).to(weight.dtype) if need_w else None
        gb = dy2.sum(0, dtype=torch.float32).to(bias.dtype) if need_b else None
        return gw, gb
    dev = dy2.device
    cur = torch.cuda.current_stream(dev)
    side = _side(dev) if _MODE != "2" else cur
    if side is not cur:
        side.wait_stream(cur)
    fast = (_WGRAD and dy2.dtype in ops.HALF and x2.dtype == dy2.dtype and dy2.stride(-1) == 1
            and x2.stride(-1) == 1 and weight.grad.is_contiguous())
    with torch.cuda.stream(side):
        if fast:
            # one split-over-tokens MFMA pass + a fixed-order reduce into .grad (csrc/wgrad.hip): hipBLASLt
            # ran these long-K, tiny-output GEMMs on 5-27 workgroups
            ops.wgrad_acc(dy2, x2, weight.grad, bias.grad if need_b else None)
        elif dy2.dtype == torch.float32:
            weight.grad.addmm_(dy2.t(), x2)
        else:
            torch.ops.aten.addmm.dtype_out(weight.grad, dy2.t(), x2, torch.float32, beta=1, alpha=1,
                                           out=weight.grad)
        if need_b and not fast:
            bias.grad.add_(dy2.sum(0, dtype=torch.float32))
    if side is not cur:
        dy2.record_stream(side)
        x2.record_stream(side)
        if not _JOIN_QUEUED[0]:
            _JOIN_QUEUED[0] = True
            torch.autograd.Variable._execution_engine.queue_callback(_join(dev))
    return None, None


class FFNResidualFn(torch.autograd.Function):
    """x + Linear2(GELU(Linear1(n))).to(x.dtype) (PN_BiMambas_Encoder's feed-forward and residual,
    src/models/DualStreamSEMamba.py:467-486) in two csrc/lgemm.hip launches each way: FFN1's bias + GELU in its
    epilogue (u kept for the backward), FFN2's bias, widening and residual add in its epilogue; backward: FFN2's
    input gradient times gelu'(u) in one launch, FFN1's input gradient, the weight gradients as SideLinear's.
    The roundings are autocast's: u, gelu(u), the FFN output and d u in the 16-bit dtype."""

    @staticmethod
    def forward(ctx, x, n, w1, b1, w2, b2, dt):
        n2 = _rows(n.to(dt))
        w1c, b1c, w2c, b2c = _cast(w1, dt), _cast(b1, dt), _cast(w2, dt), _cast(b2, dt)
        u, h = ops.lgemm(n2, w1c, b1c, epilogue=_lib.EPI_BIAS_GELU)
        if x.dtype == torch.float32:
            y = torch.empty(x.shape, device=x.device, dtype=torch.float32)
            ops.lgemm(h, w2c, b2c, out_dtype=torch.float32, residual=_rows(x), out=y.view(-1, x.shape[-1]))
        else:
            y = x + ops.lgemm(h, w2c, b2c).to(x.dtype).view(x.shape)
        ctx.save_for_backward(n2, u, h, w1c, w2c)
        ctx.params = (w1, b1, w2, b2)
        ctx.n_dtype = n.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        n2, u, h, w1c, w2c = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        dy2 = _rows(dy.to(w2c.dtype))
        du = ops.lgemm(dy2, _cast_t(w2, w2c), epilogue=_lib.EPI_GELU_BWD, aux=u)
        dn = None
        if ctx.needs_input_grad[1]:   # K = 4 d_model: hipBLASLt (see LG_MAX_K)
            dn = (ops.lgemm(du, _cast_t(w1, w1c)) if _lg_ok(du, w1c.shape[0]) else torch.mm(du, w1c))
            dn = dn.to(ctx.n_dtype).view(*dy.shape[:-1], w1c.shape[1])
        gw2, gb2 = _weight_grads(dy2, h, w2, b2, ctx.needs_input_grad[4], b2 is not None and ctx.needs_input_grad[5])
        gw1, gb1 = _weight_grads(du, n2, w1, b1, ctx.needs_input_grad[2], b1 is not None and ctx.needs_input_grad[3])
        return dy, dn, gw1, gb1, gw2, gb2, None


def ffn_residual(x, n, lin1, lin2):
    """x + lin2(gelu(lin1(n))).to(x.dtype) with FFNResidualFn on the GPU under 16-bit autocast (lgemm on), else the
    module path."""
    if (_LGEMM and _ON and n.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") in ops.HALF and x.dtype in (torch.float32, *ops.HALF)):
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return FFNResidualFn.apply(x, n, lin1.weight, lin1.bias, lin2.weight, lin2.bias, dt)
    return x + lin2(F.gelu(lin1(n))).to(x.dtype)


_WGRAD = os.environ.get("RADHIP_WGRAD", "1") != "0"     # csrc/wgrad.hip for the 16-bit weight gradients
_LGEMM = os.environ.get("RADHIP_LGEMM", "1") != "0"     # csrc/lgemm.hip for the forward / input-gradient GEMMs
_MODE = os.environ.get("RADHIP_SIDE_LINEAR", "2")   # "2": main stream; "1": side stream; "0": F.linear
_ON = _MODE != "0"


def side_linear(x, weight, bias=None):
    """F.linear(x, weight, bias) with the weight / bias gradients on the side stream (CUDA, autocast on or
    off); anything else is F.linear (and everything with RADHIP_SIDE_LINEAR=0)."""
    if not (_ON and x.is_cuda and torch.is_grad_enabled() and (weight.requires_grad or (bias is not None and bias.requires_grad))):
        return F.linear(x, weight, bias)
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    with torch.autocast("cuda", enabled=False):
        return SideLinearFn.apply(x, weight, bias, dt)


class SideLinear(nn.Linear):
    """nn.Linear (same parameters and state_dict keys) whose forward is side_linear."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.weight._radhip_direct_grad = True
        if self.bias is not None:
            self.bias._radhip_direct_grad = True

    def forward(self, x):
        return side_linear(x, self.weight, self.bias)


_ROWLN = os.environ.get("RADHIP_ROW_LN", "1") != "0"


class RowLNFn(torch.autograd.Function):
    """LayerNorm over the last dimension on csrc/rowln.hip; output in `out_dtype`."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_dtype):
        from ._lib import check
        C = x.shape[-1]
        xc = x.contiguous()
        M = xc.numel() // C
        y = torch.empty(x.shape, device=x.device, dtype=out_dtype)
        mean = torch.empty(M, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        w, b = weight.detach().float().contiguous(), bias.detach().float().contiguous()
        check(ops._L(xc, y).rdx_row_ln_fwd(ops._dtype_code(xc), ops._p(xc), ops._p(w), ops._p(b), float(eps),
                                   ops._dtype_code(y), ops._p(y), ops._p(mean), ops._p(rstd), M, C, ops._stream(xc)),
              "row_ln_fwd")
        ctx.save_for_backward(xc, mean, rstd, w)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ._lib import check
        xc, mean, rstd, w = ctx.saved_tensors
        weight, bias = ctx.params
        C = xc.shape[-1]
        M = xc.numel() // C
        dy = dy.contiguous()
        if dy.dtype not in (torch.float32, *ops.HALF) or (xc.dtype in ops.HALF
                                                           and dy.dtype not in (torch.float32, xc.dtype)):
            dy = dy.float()
        dx = torch.empty_like(xc)
        direct = all(p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
                     for p in (weight, bias))
        if direct:
            dgw, dgb = weight.grad, bias.grad
        else:
            dgw, dgb = torch.zeros(C, device=xc.device), torch.zeros(C, device=xc.device)
        check(ops._L(dy, xc).rdx_row_ln_bwd(ops._dtype_code(dy), ops._p(dy), ops._dtype_code(xc), ops._p(xc), ops._p(mean),
                                   ops._p(rstd), ops._p(w), ops._p(dx), ops._p(dgw), ops._p(dgb), M, C,
                                   ops._stream(xc)), "row_ln_bwd")
        if direct:
            return dx, None, None, None, None
        return dx, dgw.to(weight.dtype), dgb.to(bias.dtype), None, None


class RowLayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters and state_dict keys) on csrc/rowln.hip for C <= 1024 on the GPU: one kernel
    each way instead of torch's layer_norm forward, its three backward kernels and the casts around them. Its
    gamma / beta gradients are accumulated in fp32 straight into .grad (like SideLinear). `to_linear`: the only
    consumers are linears, so under bf16 / fp16 autocast the output is written in that dtype — the value the
    linear's input cast would produce from torch's fp32 output."""

    def __init__(self, *args, to_linear=False, **kw):
        super().__init__(*args, **kw)
        self.to_linear = to_linear
        if self.elementwise_affine:
            self.weight._radhip_direct_grad = True
            if self.bias is not None:
                self.bias._radhip_direct_grad = True

    def forward(self, x):
        if not (_ROWLN and x.is_cuda and len(self.normalized_shape) == 1 and x.shape[-1] <= 1024 and self.elementwise_affine
                and self.bias is not None and x.dtype in (torch.float32, *ops.HALF)):
            return super().forward(x)
        ac = torch.is_autocast_enabled("cuda")
        if ac:
            adt = torch.get_autocast_dtype("cuda")
            out = adt if (self.to_linear and adt in ops.HALF) else torch.float32
        else:
            out = x.dtype
        if x.dtype in ops.HALF and out in ops.HALF and out != x.dtype:
            return super().forward(x)
        with torch.autocast("cuda", enabled=False):
            return RowLNFn.apply(x, self.weight, self.bias, self.eps, out)
