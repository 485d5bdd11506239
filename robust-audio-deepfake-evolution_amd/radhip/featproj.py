"""WavLM feature_projection (LayerNorm(512) -> Linear(512, 1024)) of the training passes on radhip kernels.

Reference: HF WavLMFeatureProjection (transformers modeling_wavlm.py) inside WavLMFrontend
(src/models/DualStreamSEMamba.py:292-336), trained as the FGM target (src/main.py:74-100, 540-544) under autocast
(src/main.py:1049). Autocast runs the LayerNorm in fp32 on the widened CNN features and casts its output, the
projection weight and bias to the 16-bit dtype for the GEMM; its backward computes the 16-bit weight gradient,
widens it, and accumulates. Here, per group of rows with its own parameters (the window's clean pass: one group
per micro-batch, radhip/window.py; every other pass: one group):
  forward   x16 = LN(x) rounded once to 16 bits (csrc/rowln.hip: the value autocast's cast produces from the fp32
            LayerNorm output), the projection weight / bias cast to 16 bits in one launch for every group
            (ops.cast_many, each call: FGM perturbs these parameters between passes), y = x16 W^T + b on
            csrc/hgemm.hip (fp32 accumulation, bias added before the one rounding, as addmm);
  backward  dx16 = dy W on csrc/hgemm.hip; dW += dy^T x16 and db += sum dy in fp32 straight into .grad
            (csrc/wgrad.hip, batched with the pass's other weight gradients; the reference rounds dW to 16 bits
            before widening it); LN's d gamma / d beta accumulated into .grad by csrc/rowln.hip's backward.
Six torch ops forward and ten backward per group (the casts, layer_norm, addmm, its three backward products and
the gradient casts / accumulations) become three launches each way, and the GEMMs leave hipBLASLt.
"""
import os

import torch

from . import _lib, ops

_ON = os.environ.get("RADHIP_FEATPROJ", "1") != "0"     # 0: the autocast module path (A/B)

TILE = (6, 1, 4)    # hgemm 64 x 128 tiles, no split-K, 4-row-tile groups: the M = 1608 rows of one micro-batch


def eligible(fp, x, groups=None):
    """The fused path: a CUDA training pass under 16-bit autocast, LN over 512 = 8 K steps of 64, 1024 outputs, some
    parameter (fp's own, or the groups' when given) trained."""
    if not (_ON and x.is_cuda and torch.is_grad_enabled() and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") in ops.HALF and x.dim() == 3):
        return False
    ln, pr = fp.layer_norm, fp.projection
    C, E = x.shape[-1], pr.weight.shape[0]
    return (ln.elementwise_affine and ln.bias is not None and pr.bias is not None and C == pr.weight.shape[1]
            and C % 64 == 0 and E % 64 == 0 and C <= 1024 and x.dtype in (torch.float32, *ops.HALF)
            and any(p.requires_grad for g in (groups or [(ln.weight, ln.bias, pr.weight, pr.bias)]) for p in g))


def _direct(p):
    return p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous()


class FeatProjFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps, dt, *params):
        K = len(params) // 4
        N, T, C = x.shape
        M = N * T
        if M % K:
            raise ValueError(f"radhip feature_projection: {M} rows do not split into {K} groups")
        R = M // K
        E = params[2].shape[0]
        xc = x.contiguous().view(M, C)
        dev = x.device
        x16 = torch.empty(M, C, device=dev, dtype=dt)
        mean = torch.empty(M, device=dev, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        src = [t.detach() for k in range(K) for t in (params[4 * k + 2], params[4 * k + 3])]
        dst = [torch.empty_like(t, dtype=dt) for t in src]
        ops.cast_many(src, dst)
        y = torch.empty(N, T, E, device=dev, dtype=dt)
        y2 = y.view(M, E)
        lib = ops._L(dt)
        for k in range(K):
            sl = slice(k * R, (k + 1) * R)
            lw, lb = params[4 * k].detach(), params[4 * k + 1].detach()
            _lib.check(lib.rdx_row_ln_fwd(ops._dtype_code(xc), ops._p(xc[sl]), ops._p(lw), ops._p(lb), float(eps),
                                          ops._dtype_code(x16), ops._p(x16[sl]), ops._p(mean[sl]), ops._p(rstd[sl]),
                                          R, C, ops._stream(xc)), "row_ln_fwd")
            ops.hgemm(x16[sl], dst[2 * k], dst[2 * k + 1], out=y2[sl], tile=TILE[0], splits=TILE[1],
                      group_m=TILE[2])
        ctx.save_for_backward(xc, x16, mean, rstd, *dst[0::2])
        ctx.params = params
        ctx.shape = (N, T, C, K, R, E)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, x16, mean, rstd, *wc = ctx.saved_tensors
        params = ctx.params
        N, T, C, K, R, E = ctx.shape
        M = N * T
        dt = x16.dtype
        dy2 = dy.to(dt).contiguous().view(M, E)
        lib = ops._L(dt)
        dx = torch.empty(M, C, device=xc.device, dtype=xc.dtype)
        grads = [None] * len(params)
        need = ctx.needs_input_grad[3:]
        for k in range(K):
            sl = slice(k * R, (k + 1) * R)
            lw, lb, pw, pb = params[4 * k:4 * k + 4]
            dx16 = ops.hgemm(dy2[sl], wc[k].t().contiguous(), tile=TILE[0], splits=TILE[1], group_m=TILE[2])
            if need[4 * k + 2] and need[4 * k + 3] and _direct(pw) and _direct(pb):
                ops.wgrad_acc(dy2[sl], x16[sl], pw.grad, pb.grad)
            else:
                if need[4 * k + 2]:
                    grads[4 * k + 2] = (dy2[sl].t().float() @ x16[sl].float()).to(pw.dtype)
                if need[4 * k + 3]:
                    grads[4 * k + 3] = dy2[sl].float().sum(0).to(pb.dtype)
            direct = need[4 * k] and need[4 * k + 1] and _direct(lw) and _direct(lb)
            dgw, dgb = (lw.grad, lb.grad) if direct else (torch.zeros(C, device=xc.device),
                                                          torch.zeros(C, device=xc.device))
            _lib.check(lib.rdx_row_ln_bwd(ops._dtype_code(dx16), ops._p(dx16), ops._dtype_code(xc), ops._p(xc[sl]),
                                          ops._p(mean[sl]), ops._p(rstd[sl]), ops._p(lw.detach()), ops._p(dx[sl]),
                                          ops._p(dgw), ops._p(dgb), R, C, ops._stream(xc)), "row_ln_bwd")
            if not direct:
                grads[4 * k] = dgw.to(lw.dtype) if need[4 * k] else None
                grads[4 * k + 1] = dgb.to(lb.dtype) if need[4 * k + 1] else None
        dxo = dx.view(N, T, C) if ctx.needs_input_grad[0] else None
        return (dxo, None, None, *grads)


def feature_projection(fp, x, groups=None):
    """fp(x) (dropout included) on the fused path; `groups`: K tuples (ln_w, ln_b, proj_w, proj_b) applied to K equal
    row blocks of x (the window's per-micro-batch leaf copies), else fp's own parameters."""
    ps = groups if groups is not None else [(fp.layer_norm.weight, fp.layer_norm.bias, fp.projection.weight,
                                             fp.projection.bias)]
    dt = torch.get_autocast_dtype("cuda")
    flat = [t for g in ps for t in g]
    with torch.autocast("cuda", enabled=False):
        y = FeatProjFn.apply(x, fp.layer_norm.eps, dt, *flat)
    return fp.dropout(y)
