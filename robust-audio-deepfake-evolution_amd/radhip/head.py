"""Fused pieces of the detector head on csrc/head.hip (training and 16-bit scoring passes under autocast).

Attention pooling (Model.forward's tail, src/models/DualStreamSEMamba.py:700-770): attn = softmax_t(attention_pool(f))
and features = attn^T f under autocast are a 1-output linear, the fp32 softmax, the cast of the weights back to 16
bits and a batched GEMM forward, and their six backward kernels plus the add of f's two gradients; here one launch
forward (rdx_attn_pool_fwd) and two backward (rdx_attn_pool_bwd), with the same 16-bit roundings.

DualStreamFusion's time alignment (src/models/DualStreamSEMamba.py:537-637): the SincNet features F.interpolate'd
('nearest', run in fp32 under autocast) to the WavLM frame rate and concatenated with the WavLM features: casts, the
upsample and the cat forward, the casts and the upsample backward (with its zero fill) backward. Here one gather
launch each way (rdx_upcat_fwd / _bwd); the WavLM half's gradient is a view of the concat's.

Reference: SELayer (src/models/DualStreamSEMamba.py:492-531) inside DualStreamFusion (:537-637): squeeze-excitation
over time, y = x * sigmoid(fc2(relu(fc1(mean_t x)))), fc1 / fc2 bias-free linears. Under autocast the module path is
a mean kernel, two small GEMMs, relu, sigmoid and the product forward, and about a dozen kernels backward (the product's
two gradients, the broadcast sum and its cast, sigmoid / relu backward, the GEMMs' input gradients, the mean's
expansion, the add of the two branches' gradients). Here: one launch forward (rdx_se_fwd), two backward (rdx_se_bwd:
the utterance-parallel pass and the fixed-order reduction of the fc weight gradients, added in fp32 straight into
.grad when it is bound, as radhip.linear.SideLinear does).
"""
import torch

from . import _lib, ops
from .linear import _cast


def _direct(p):
    return p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous()


def se_eligible(x, w1, w2):
    """The fused SE: CUDA, 16-bit autocast on, [B, T, C] with C % 8 == 0, C <= 256, a squeeze width <= 16."""
    if not (x.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") in ops.HALF
            and x.dim() == 3):
        return False
    C = x.shape[-1]
    R = w1.shape[0]
    return (C % 8 == 0 and C <= 256 and 0 < R <= 16 and tuple(w1.shape) == (R, C) and tuple(w2.shape) == (C, R)
            and x.shape[1] * C * 2 <= 64 * 1024     # one utterance's rows fit the kernels' LDS image
            and x.dtype == torch.get_autocast_dtype("cuda"))   # the module path's output dtype then is x's


class SEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, w2, dt):
        xc = x.to(dt).contiguous()
        if xc.data_ptr() % 16:
            xc = xc.clone()
        w1c, w2c = _cast(w1, dt).contiguous(), _cast(w2, dt).contiguous()
        B, T, C = xc.shape
        R = w1.shape[0]
        y = torch.empty_like(xc)
        m = torch.empty(B, C, device=xc.device, dtype=dt)
        h = torch.empty(B, R, device=xc.device, dtype=dt)
        s = torch.empty(B, C, device=xc.device, dtype=dt)
        _lib.check(ops._L(dt).rdx_se_fwd(ops._p(xc), ops._p(w1c), ops._p(w2c), ops._p(y), ops._p(m), ops._p(h), ops._p(s),
                                          B, T, C, R, ops._stream(xc)), "se_fwd")
        ctx.save_for_backward(xc, w1c, w2c, m, h, s)
        ctx.params = (w1, w2)
        ctx.x_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w1c, w2c, m, h, s = ctx.saved_tensors
        w1, w2 = ctx.params
        B, T, C = xc.shape
        R = w1c.shape[0]
        dt = xc.dtype
        dyc = dy.to(dt).contiguous()
        if dyc.data_ptr() % 16:
            dyc = dyc.clone()
        dx = torch.empty_like(xc)
        part = torch.empty(int(_lib.lib().rdx_se_bwd_part_floats(B, C, R)), device=xc.device, dtype=torch.float32)
        need = ctx.needs_input_grad
        direct = need[1] and need[2] and _direct(w1) and _direct(w2)
        g1, g2 = (w1.grad, w2.grad) if direct else (torch.zeros(R, C, device=xc.device),
                                                    torch.zeros(C, R, device=xc.device))
        _lib.check(ops._L(dt).rdx_se_bwd(ops._p(dyc), ops._p(xc), ops._p(w1c), ops._p(w2c), ops._p(m), ops._p(h),
                                          ops._p(s), ops._p(dx), ops._p(part), ops._p(g1), ops._p(g2), B, T, C, R,
                                          ops._stream(xc)), "se_bwd")
        gw1 = None if direct or not need[1] else g1.to(w1.dtype)
        gw2 = None if direct or not need[2] else g2.to(w2.dtype)
        return (dx.to(ctx.x_dtype) if need[0] else None), gw1, gw2, None


def se_layer(x, w1, w2):
    """x * sigmoid(w2 relu(w1 mean_t x)) on the fused kernels (x [B, T, C]; call under 16-bit autocast)."""
    dt = torch.get_autocast_dtype("cuda")
    with torch.autocast("cuda", enabled=False):
        return SEFn.apply(x, w1, w2, dt)


def pool_eligible(f, lin):
    """The fused attention pooling: CUDA, 16-bit autocast, f [B, T, C] in that dtype, a 1-output linear."""
    return (f.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") in ops.HALF
            and f.dim() == 3 and f.dtype == torch.get_autocast_dtype("cuda") and lin.weight.shape[0] == 1
            and f.shape[1] <= 1024 and f.shape[2] <= 1024 and f.shape[2] % 8 == 0
            and f.shape[1] * f.shape[2] * 2 <= 128 * 1024)   # one utterance's rows fit the kernels' LDS image


class AttnPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, w, bias, dt):
        fc = f.contiguous()
        if fc.data_ptr() % 16:
            fc = fc.clone()
        wc = _cast(w, dt).reshape(-1).contiguous()
        bc = _cast(bias, dt).reshape(-1).contiguous() if bias is not None else None
        B, T, C = fc.shape
        feat = torch.empty(B, C, device=fc.device, dtype=dt)
        a = torch.empty(B, T, device=fc.device, dtype=torch.float32)
        _lib.check(ops._L(dt).rdx_attn_pool_fwd(ops._p(fc), ops._p(wc), ops._p(bc) if bc is not None else None,
                                                 ops._p(feat), ops._p(a), B, T, C, ops._stream(fc)), "attn_pool_fwd")
        ctx.save_for_backward(fc, wc, a)
        ctx.params = (w, bias)
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        fc, wc, a = ctx.saved_tensors
        w, bias = ctx.params
        B, T, C = fc.shape
        dfc = dfeat.to(fc.dtype).contiguous()
        df = torch.empty_like(fc)
        part = torch.empty(B * (C + 1), device=fc.device, dtype=torch.float32)
        need = ctx.needs_input_grad
        has_b = bias is not None
        direct = need[1] and _direct(w) and (not has_b or (need[2] and _direct(bias)))
        if direct:
            gw, gb = w.grad.view(-1), (bias.grad.view(-1) if has_b else None)
        else:
            gw, gb = torch.zeros(C, device=fc.device), torch.zeros(1, device=fc.device)
        _lib.check(ops._L(fc).rdx_attn_pool_bwd(ops._p(fc), ops._p(wc), ops._p(a), ops._p(dfc), ops._p(df), ops._p(part),
                                                 ops._p(gw), ops._p(gb) if gb is not None else None, B, T, C,
                                                 ops._stream(fc)), "attn_pool_bwd")
        rw = None if direct or not need[1] else gw.view_as(w).to(w.dtype)
        rb = None if direct or not has_b or not need[2] else gb.view_as(bias).to(bias.dtype)
        return (df if need[0] else None), rw, rb, None


def attn_pool(f, w, bias):
    """softmax_t(f w^T + bias)^T f -> [B, C] on the fused kernels (call under 16-bit autocast)."""
    dt = torch.get_autocast_dtype("cuda")
    with torch.autocast("cuda", enabled=False):
        return AttnPoolFn.apply(f, w, bias, dt)


def upcat_eligible(fw, fs):
    """The fused alignment + concat: CUDA, 16-bit autocast, both [B, T, C] in that dtype, 'nearest' (T1 > 4 T2)."""
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else None
    return (fw.is_cuda and dt in ops.HALF and fw.dtype == dt and fs.dtype == dt and fw.dim() == 3 and fs.dim() == 3
            and fw.shape[0] == fs.shape[0] and fw.shape[2] == fs.shape[2] and fw.shape[2] % 8 == 0
            and fw.shape[1] / fs.shape[1] > 4.0)


class UpcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fw, fs):
        fwc, fsc = fw.contiguous(), fs.contiguous()
        B, T1, C = fwc.shape
        T2 = fsc.shape[1]
        out = torch.empty(B, T1, 2 * C, device=fwc.device, dtype=fwc.dtype)
        _lib.check(ops._L(fwc).rdx_upcat_fwd(ops._p(fwc), ops._p(fsc), ops._p(out), B, T1, T2, C, ops._stream(fwc)),
                   "upcat_fwd")
        ctx.dims = (B, T1, T2, C)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, T1, T2, C = ctx.dims
        dout = dout.contiguous()
        dfs = None
        if ctx.needs_input_grad[1]:
            dfs = torch.empty(B, T2, C, device=dout.device, dtype=dout.dtype)
            _lib.check(ops._L(dout).rdx_upcat_bwd(ops._p(dout), ops._p(dfs), B, T1, T2, C, ops._stream(dout)),
                       "upcat_bwd")
        dfw = dout[..., :C] if ctx.needs_input_grad[0] else None
        return dfw, dfs


def upcat(fw, fs):
    """cat([fw, nearest-upsampled fs], -1) on the fused gather (call under 16-bit autocast)."""
    with torch.autocast("cuda", enabled=False):
        return UpcatFn.apply(fw, fs)
