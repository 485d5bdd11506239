"""Drop-in `Mamba` module backed by the radhip HIP kernels.

Replaces `mamba_ssm.modules.mamba_simple.Mamba(d_model, d_state)` as imported by the reference at
src/models/DualStreamSEMamba.py:43 and built per PN_BiMambas_Encoder at :455. Parameter names and
shapes are identical (in_proj.weight, conv1d.{weight,bias}, x_proj.weight, dt_proj.{weight,bias},
A_log, D, out_proj.weight), so reference checkpoints load unchanged. Arithmetic follows the
reference-owned MambaBlock (src/models/modules/mamba_block.py:41-122) == mamba_ssm semantics:
    xz = in_proj(x); x, z = split; u = silu(causal_dwconv4(x)); (dt, B, C) = x_proj(u)
    delta = softplus(dt_proj(dt)); h_t = exp(delta A) h_{t-1} + delta B u; y = C.h + D u
    out = out_proj(y * silu(z))
`bidirectional(x)` computes mamba(x) + flip(mamba(flip(x))) (DualStreamSEMamba.py:472-481) in one
pass: in_proj is shared (it is per-position), both scan directions run in every kernel launch, and
because the gate z and out_proj are per-position the two directions share ONE gate and ONE out_proj
GEMM: out = out_proj((y_fwd + y_bwd) * silu(z)).
"""
import ctypes
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from ._lib import check, lib
from .linear import LG_MAX_K, SideLinear, _LGEMM, _ON, _cast, _cast_t, _lg_ok, _rows, _weight_grads, side_linear
from .ops import BiGate, DWConvBidir, SelectiveScan, SplitLast


class Mamba(nn.Module):
    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto", dt_min=0.001, dt_max=0.1,
                 dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, conv_bias=True, bias=False, device=None,
                 dtype=None, **_ignored):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model = d_model
        self.d_state = d_state
        self.d_conv = d_conv
        self.expand = expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.in_proj = SideLinear(d_model, self.d_inner * 2, bias=bias, **fk)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, bias=conv_bias, kernel_size=d_conv,
                                groups=self.d_inner, padding=d_conv - 1, **fk)
        self.x_proj = SideLinear(self.d_inner, self.dt_rank + 2 * d_state, bias=False, **fk)
        self.dt_proj = SideLinear(self.dt_rank, self.d_inner, bias=True, **fk)
        # mamba_ssm initialisation of dt_proj (keeps softplus(bias) in [dt_min, dt_max])
        std = self.dt_rank ** -0.5 * dt_scale
        with torch.no_grad():
            if dt_init == "constant":
                nn.init.constant_(self.dt_proj.weight, std)
            else:
                nn.init.uniform_(self.dt_proj.weight, -std, std)
            dt = torch.exp(torch.rand(self.d_inner, **fk) * (math.log(dt_max) - math.log(dt_min))
                           + math.log(dt_min)).clamp(min=dt_init_floor)
            self.dt_proj.bias.copy_(dt + torch.log(-torch.expm1(-dt)))
        self.dt_proj.bias._no_reinit = True
        A = torch.arange(1, d_state + 1, dtype=torch.float32, device=device).repeat(self.d_inner, 1)
        self.A_log = nn.Parameter(torch.log(A))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_inner, device=device))
        self.D._no_weight_decay = True
        self.out_proj = SideLinear(self.d_inner, d_model, bias=bias, **fk)

    def _run(self, x, dirs):
        Di, R, N = self.d_inner, self.dt_rank, self.d_state
        xz = self.in_proj(x)                                    # [B, L, 2*Di]
        xi, z = SplitLast.apply(xz, Di, Di)                     # views; backward is one concatenation
        u = DWConvBidir.apply(xi, self.conv1d.weight, self.conv1d.bias, dirs)  # [dirs, B, L, Di]
        x_dbl = side_linear(u, self.x_proj.weight)                # [dirs, B, L, R + 2N]
        dt, Bm, Cm = SplitLast.apply(x_dbl, R, N, N)
        delta = side_linear(dt, self.dt_proj.weight)              # bias + softplus are fused in the scan
        y = SelectiveScan.apply(u, delta, self.A_log, Bm, Cm, self.D, self.dt_proj.bias)  # [dirs, B, L, Di] fp32
        g = BiGate.apply(y, z)                                  # (sum_dir y) * silu(z)
        return self.out_proj(g)

    def forward(self, hidden_states, inference_params=None):
        return self._run(hidden_states, 1)

    def bidirectional(self, hidden_states):
        """mamba(x) + flip(mamba(flip(x), dims=[1]), dims=[1]) with shared weights, one pass."""
        x = hidden_states
        if (_FUSED and _LGEMM and _ON and x.is_cuda and x.dim() == 3 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") in ops.HALF and ops.scan2_enabled() and self.d_state == 16
                and self.in_proj.bias is None and self.x_proj.bias is None and self.out_proj.bias is None
                and self.conv1d.bias is not None
                # every GEMM of the node runs on csrc/lgemm.hip with K = d_model, d_inner or dt_rank: within the K
                # its single-chunk LDS staging is built for (radhip/linear.py LG_MAX_K; larger widths take the
                # module path, whose linears fall back to hipBLASLt)
                and max(x.shape[-1], self.in_proj.weight.shape[0] // 2, self.dt_proj.weight.shape[1]) <= LG_MAX_K):
            dt = torch.get_autocast_dtype("cuda")
            with torch.autocast("cuda", enabled=False):
                return MambaBiFn.apply(x, self.in_proj.weight, self.conv1d.weight, self.conv1d.bias,
                                       self.x_proj.weight, self.dt_proj.weight, self.dt_proj.bias, self.A_log,
                                       self.D, self.out_proj.weight, dt)
        return self._run(hidden_states, 2)


_FUSED = os.environ.get("RADHIP_MAMBA_FUSED", "1") != "0"


class MambaBiFn(torch.autograd.Function):
    """Mamba.bidirectional as one autograd node over its HIP launches: in_proj, x_proj, dt_proj and out_proj on
    csrc/lgemm.hip, the causal depthwise conv + SiLU and the gate on csrc/bimamba.hip, the chunked scan on
    csrc/scan2.hip. The autograd graph of the module path (src/models/modules/mamba_block.py:41-122, both
    directions) is the same arithmetic with more launches around it: the split views' concatenating backwards,
    the dB / dC cast, the sum of the two input gradients of u. Here the backward writes d(x_dbl) and d(xz) in place
    (d dt by the dt_proj input-gradient GEMM into its columns, dB | dC copied beside it, dz by the gate's backward
    and d xi by the conv's backward into the halves of d xz) and x_proj's input gradient is added to the scan's
    d u in its GEMM epilogue (the same 16-bit rounding as autograd's add)."""

    @staticmethod
    def forward(ctx, x, w_in, conv_w, conv_b, w_x, w_dt, dt_bias, A_log, Dp, w_out, dt):
        B, L, Dm = x.shape
        M = B * L
        n2 = _rows(x.to(dt))
        wi, wx, wdt, wo = _cast(w_in, dt), _cast(w_x, dt), _cast(w_dt, dt), _cast(w_out, dt)
        Di, R, N = wi.shape[0] // 2, wdt.shape[1], A_log.shape[1]
        dev = x.device
        st = ops._stream(n2)
        Lb = ops._L(wi)
        code = ops._dtype_code(wi)
        xz = ops.lgemm(n2, wi)                                        # [M, 2 Di]
        cw = conv_w.detach().reshape(Di, -1).float().contiguous()
        cb = conv_b.detach().float().contiguous()
        K = cw.shape[1]
        u = torch.empty(2, B, L, Di, device=dev, dtype=dt)
        check(Lb.rdx_dwconv_bidir_fwd(code, ops._p(xz), 2 * Di, ops._p(cw), ops._p(cb), ops._p(u), B, L, Di, K, 2,
                                      st), "dwconv_bidir_fwd")
        x_dbl = ops.lgemm(u.view(2 * M, Di), wx)                      # [2M, R + 2N]
        delta = ops.lgemm(x_dbl[:, :R], wdt)                          # [2M, Di] (bias + softplus in the scan)
        Af = A_log.detach().float().contiguous()
        Df = Dp.detach().float().contiguous()
        bf = dt_bias.detach().float().contiguous()
        y = torch.empty(2, B, L, Di, device=dev, dtype=torch.float32)
        ck = torch.empty(lib().rdx_scan_ckpt_elems(B, L, Di, N, 2), device=dev, dtype=torch.float32)
        nrec = int(lib().rdx_scan2_rec_elems(B, L, Di, N, 2))
        P = torch.empty(nrec, device=dev, dtype=torch.float32)
        hloc = torch.empty(nrec, device=dev, dtype=torch.float32)
        ldbc = R + 2 * N
        es = u.element_size()
        with ops._timed("selective_scan_fwd", u, 2 * M * (Di * (2 * es + 4) + 2 * N * es)):
            check(Lb.rdx_scan2_fwd(code, ops._p(u), ops._p(delta), ops._p(Af), ops._p(x_dbl[:, R:]),
                                   ops._p(x_dbl[:, R + N:]), ldbc, ops._p(Df), ops._p(bf), ops._p(y), ops._p(ck),
                                   ops._p(P), ops._p(hloc), B, L, Di, N, 2, st), "scan2_fwd")
        g = torch.empty(M, Di, device=dev, dtype=dt)
        ysum = torch.empty(M, Di, device=dev, dtype=torch.float32)
        check(Lb.rdx_bigate_fwd(code, ops._p(y), 2, ops._p(xz[:, Di:]), 2 * Di, ops._p(g), ops._p(ysum), B, L, Di, st),
              "bigate_fwd")
        out = torch.empty(B, L, Dm, device=dev, dtype=dt)
        ops.lgemm(g, wo, out=out.view(M, Dm))
        ctx.save_for_backward(n2, xz, u, x_dbl, delta, ck, P, g, ysum, wi, wx, wdt, wo, cw, cb, Af, Df, bf)
        ctx.params = (w_in, conv_w, w_x, w_dt, w_out)
        ctx.x_dtype = x.dtype
        ctx.dims = (B, L, Dm, Di, R, N, K)
        return out

    @staticmethod
    def backward(ctx, dout):
        n2, xz, u, x_dbl, delta, ck, P, g, ysum, wi, wx, wdt, wo, cw, cb, Af, Df, bf = ctx.saved_tensors
        w_in, conv_w, w_x, w_dt, w_out = ctx.params
        B, L, Dm, Di, R, N, K = ctx.dims
        M = B * L
        dt = wi.dtype
        dev = dout.device
        need = ctx.needs_input_grad
        Lb = ops._L(wi)
        code = ops._dtype_code(wi)
        do2 = _rows(dout.to(dt))
        st = ops._stream(do2)
        dg = ops.lgemm(do2, _cast_t(w_out, wo))                        # [M, Di]
        gw_out, _ = _weight_grads(do2, g, w_out, None, need[9], False)
        dxz = torch.empty(M, 2 * Di, device=dev, dtype=dt)
        dy = torch.empty(M, Di, device=dev, dtype=torch.float32)
        check(Lb.rdx_bigate_bwd(code, ops._p(dg), ops._p(xz[:, Di:]), 2 * Di, ops._p(ysum), ops._p(dy),
                                ops._p(dxz[:, Di:]), 2 * Di, B, L, Di, st), "bigate_bwd")
        du = torch.empty(2 * M, Di, device=dev, dtype=dt)
        ddelta = torch.empty(2 * M, Di, device=dev, dtype=dt)
        dBC = torch.empty(2 * M, 2 * N, device=dev, dtype=torch.float32)
        parts = 2 * B * int(lib().rdx_scan2_chunks(L))
        part = torch.empty(parts, Di * N + 2 * Di, device=dev, dtype=torch.float32)
        base = part.data_ptr()
        gloc = torch.empty(int(lib().rdx_scan2_rec_elems(B, L, Di, N, 2)), device=dev, dtype=torch.float32)
        ldbc = R + 2 * N
        es = u.element_size()
        with ops._timed("selective_scan_bwd", u, 2 * M * (Di * (4 * es + 4) + 2 * N * es)):
            check(Lb.rdx_scan2_bwd(code, ops._p(u), ops._p(delta), ops._p(Af), ops._p(x_dbl[:, R:]),
                                   ops._p(x_dbl[:, R + N:]), ldbc, ops._p(Df), ops._p(bf), ops._p(ck), ops._p(P),
                                   ops._p(dy), 0, ops._p(du), ops._p(ddelta), ops._p(dBC), ctypes.c_void_p(base),
                                   ctypes.c_void_p(base + 4 * Di * N), ctypes.c_void_p(base + 4 * (Di * N + Di)),
                                   Di * N + 2 * Di, ops._p(gloc), B, L, Di, N, 2, st), "scan2_bwd")
        dxdbl = torch.empty(2 * M, ldbc, device=dev, dtype=dt)
        dxdbl[:, R:].copy_(dBC)
        ops.lgemm(ddelta, _cast_t(w_dt, wdt), out=dxdbl[:, :R])       # d dt
        gw_dt, _ = _weight_grads(ddelta, x_dbl[:, :R], w_dt, None, need[5], False)
        gw_x, _ = _weight_grads(dxdbl, u.view(2 * M, Di), w_x, None, need[4], False)
        ops.lgemm(dxdbl, _cast_t(w_x, wx), residual=du, out=du)       # d u += x_proj's input gradient
        partc = torch.empty(int(lib().rdx_dwconv_bidir_bwd_parts(L)) * B, Di * K + Di, device=dev,
                            dtype=torch.float32)
        check(Lb.rdx_dwconv_bidir_bwd(code, ops._p(xz), 2 * Di, ops._p(cw), ops._p(cb), ops._p(du), ops._p(dxz),
                                      2 * Di, ops._p(partc), ctypes.c_void_p(partc.data_ptr() + 4 * Di * K),
                                      Di * K + Di, B, L, Di, K, 2, st), "dwconv_bidir_bwd")
        tot = torch.empty(part.shape[1], device=dev, dtype=torch.float32)
        totc = torch.empty(partc.shape[1], device=dev, dtype=torch.float32)
        ops.colsum_many([(part, tot), (partc, totc)])     # the scan's and the conv's parameter-gradient partials
        gw_in, _ = _weight_grads(dxz, n2, w_in, None, need[1], False)
        dx = None
        if need[0]:
            dx = ops.lgemm(dxz, _cast_t(w_in, wi)) if _lg_ok(dxz, 2 * Di) else torch.mm(dxz, wi)   # K = 2 Di
            dx = dx.to(ctx.x_dtype).view(B, L, Dm)
        return (dx, gw_in, totc[:Di * K].view(conv_w.shape), totc[Di * K:], gw_x, gw_dt, tot[Di * N + Di:],
                tot[:Di * N].view(Di, N), tot[Di * N:Di * N + Di], gw_out, None)
