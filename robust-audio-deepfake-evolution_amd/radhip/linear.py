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

from . import ops

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


def direct_grad(p):
    """True for parameters whose gradient SideLinear accumulates into .grad itself (window.py keeps their
    .grad bound during a pass instead of handing it over through autograd)."""
    return getattr(p, "_radhip_direct_grad", False)


class SideLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dt):
        xc, wc, bc = x.to(dt), _cast(weight, dt), _cast(bias, dt)
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
            dx = torch.matmul(dy, wc).to(ctx.x_dtype)
        need_w, need_b = ctx.needs_input_grad[1], bias is not None and ctx.needs_input_grad[2]
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = xc.reshape(-1, xc.shape[-1])
        direct = (dy.is_cuda and need_w and weight.grad is not None and weight.grad.dtype == torch.float32
                  and (not need_b or (bias.grad is not None and bias.grad.dtype == torch.float32)))
        if not direct:
            gw = torch.matmul(dy2.t(), x2).to(weight.dtype) if need_w else None
            gb = dy2.sum(0, dtype=torch.float32).to(bias.dtype) if need_b else None
            return dx, gw, gb, None
        dev = dy.device
        cur = torch.cuda.current_stream(dev)
        side = _side(dev) if _MODE != "2" else cur
        if side is not cur:
            side.wait_stream(cur)
        with torch.cuda.stream(side):
            if (_WGRAD and dy2.dtype in ops.HALF and x2.dtype == dy2.dtype and dy2.stride(-1) == 1
                    and x2.stride(-1) == 1 and weight.grad.is_contiguous()):
                # one split-over-tokens MFMA pass + a fixed-order reduce into .grad (csrc/wgrad.hip): hipBLASLt
                # ran these long-K, tiny-output GEMMs on 5-27 workgroups
                ops.wgrad_acc(dy2, x2, weight.grad, bias.grad if need_b else None)
            elif dy2.dtype == torch.float32:
                weight.grad.addmm_(dy2.t(), x2)
            else:
                torch.ops.aten.addmm.dtype_out(weight.grad, dy2.t(), x2, torch.float32, beta=1, alpha=1,
                                               out=weight.grad)
            if need_b and not (_WGRAD and dy2.dtype in ops.HALF and x2.dtype == dy2.dtype
                               and dy2.stride(-1) == 1 and x2.stride(-1) == 1 and weight.grad.is_contiguous()):
                bias.grad.add_(dy2.sum(0, dtype=torch.float32))
        if side is cur:
            return dx, None, None, None
        dy2.record_stream(side)
        x2.record_stream(side)
        if not _JOIN_QUEUED[0]:
            _JOIN_QUEUED[0] = True
            torch.autograd.Variable._execution_engine.queue_callback(_join(dev))
        return dx, None, None, None


_WGRAD = os.environ.get("RADHIP_WGRAD", "1") != "0"     # csrc/wgrad.hip for the 16-bit weight gradients
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
