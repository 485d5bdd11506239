"""Sequential (per-time-step) restatement of the Mamba block and the Pre-Norm Bi-Mamba layer.

Restates the reference-owned pure-torch MambaBlock (src/models/modules/mamba_block.py:6-122), which
the reference itself documents as param-compatible with mamba_ssm's Mamba (the CUDA kernel parity of
mamba_ssm is unpinned: it is absent from the image), and PN_BiMambas_Encoder
(src/models/DualStreamSEMamba.py:445-486). Runs on CPU, any float dtype (tests use float64).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class MambaRef(nn.Module):
    """Same parameter names/shapes as mamba_ssm.Mamba / the product radhip.mamba.Mamba."""

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2):
        super().__init__()
        self.d_model, self.d_state, self.d_conv = d_model, d_state, d_conv
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16)
        self.in_proj = nn.Linear(d_model, 2 * self.d_inner, bias=False)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, d_conv, groups=self.d_inner, padding=d_conv - 1,
                                bias=True)
        self.x_proj = nn.Linear(self.d_inner, self.dt_rank + 2 * d_state, bias=False)
        self.dt_proj = nn.Linear(self.dt_rank, self.d_inner, bias=True)
        self.A_log = nn.Parameter(torch.log(torch.arange(1, d_state + 1, dtype=torch.float32)
                                            .repeat(self.d_inner, 1)))
        self.D = nn.Parameter(torch.ones(self.d_inner))
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=False)

    def forward(self, x):
        # mamba_block.py:41-63
        L = x.shape[1]
        xz = self.in_proj(x)
        xi, z = xz.chunk(2, dim=-1)
        xi = self.conv1d(xi.transpose(1, 2))[:, :, :L].transpose(1, 2)
        xi = F.silu(xi)
        y = self.scan(xi)
        return self.out_proj(y * F.silu(z))

    def scan(self, u):
        # mamba_block.py:65-122 — explicit loop over time
        Bsz, L, Di = u.shape
        xd = self.x_proj(u)
        dt, Bm, Cm = torch.split(xd, [self.dt_rank, self.d_state, self.d_state], dim=-1)
        dt = F.softplus(self.dt_proj(dt))
        A = -torch.exp(self.A_log)
        h = u.new_zeros(Bsz, Di, self.d_state)
        out = []
        for t in range(L):
            d_t = dt[:, t, :, None]
            h = torch.exp(A * d_t) * h + (Bm[:, t, None, :] * d_t) * u[:, t, :, None]
            out.append((h * Cm[:, t, None, :]).sum(-1))
        return torch.stack(out, 1) + u * self.D


def bimamba_ref(mamba, x):
    """mamba(x) + flip(mamba(flip(x))) with shared weights (DualStreamSEMamba.py:472-481)."""
    return mamba(x) + torch.flip(mamba(torch.flip(x, dims=[1])), dims=[1])


class PNBiMambaRef(nn.Module):
    """PN_BiMambas_Encoder (DualStreamSEMamba.py:445-486)."""

    def __init__(self, d_model, n_state):
        super().__init__()
        self.d_model = d_model
        self.mamba = MambaRef(d_model, n_state)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.feed_forward = nn.Sequential(nn.Linear(d_model, 4 * d_model), nn.GELU(), nn.Linear(4 * d_model, d_model))

    def forward(self, x):
        n = self.norm1(x)
        m = self.norm2(bimamba_ref(self.mamba, n))
        return self.feed_forward(m) + x
