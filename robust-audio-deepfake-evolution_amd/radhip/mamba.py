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
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .linear import SideLinear, side_linear
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
        return self._run(hidden_states, 2)
