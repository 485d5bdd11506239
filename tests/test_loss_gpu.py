"""Mixup focal loss on csrc/loss.hip (radhip.ops.mixup_focal) against the module criterion.

Reference: kornia FocalLoss(alpha 0.9, gamma 2.5, reduction 'mean') (src/main.py:297-305) inside the mixup
loss lam * crit(out, y_a) + (1 - lam) * crit(out, y_b), divided by the accumulation steps (:1040-1050).
The module path is radhip.train.FocalLoss (pinned by tests/test_train_cpu.py's hand-computed values) in
fp32 autograd on the same logits. Both alpha modes, fp32 and bf16 logits, one micro-batch (adversarial
pass) and K micro-batches with their own lam (the window's batched clean pass). Tolerance: fp32
transcendental rounding, 1e-5 relative on the loss and 1e-5 of the gradient scale."""
import numpy as np
import pytest
import torch

from seeded import seeded_array

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _module_loss(focal, logits, ya, yb, lam, B, accum):
    tot = 0.0
    for k in range(logits.shape[0] // B):
        sl = slice(k * B, (k + 1) * B)
        tot = tot + lam[k] * focal(logits[sl], ya[sl]) + (1 - lam[k]) * focal(logits[sl], yb[sl])
    return tot / accum


@pytest.mark.parametrize("mode", ["per_class", "scalar"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("K", [1, 4])
def test_mixup_focal_matches_module(mode, dtype, K):
    from radhip.ops import mixup_focal
    from radhip.train import FocalLoss
    B, accum = 8, 4
    focal = FocalLoss(0.9, 2.5, mode)
    z = torch.from_numpy(seeded_array(f"fl{K}", (K * B, 2), scale=3.0)).to(dtype).to(DEV)
    ya = torch.from_numpy((seeded_array(f"fla{K}", (K * B,), scale=1.0) > 0.8).astype(np.int64)).to(DEV)
    yb = ya.flip(0).contiguous()
    lam = torch.from_numpy(np.abs(seeded_array(f"fll{K}", (K,), scale=0.5)).clip(0, 1)).float().to(DEV)
    zr = z.float().clone().requires_grad_(True)
    ref = _module_loss(focal, zr, ya, yb, lam, B, accum)
    ref.backward()
    zg = z.clone().requires_grad_(True)
    got = mixup_focal(zg, ya, yb, lam, B, focal, accum)
    got.backward()
    assert got.dtype == torch.float32 and zg.grad.dtype == dtype
    np.testing.assert_allclose(float(got), float(ref), rtol=1e-5)
    g, r = zg.grad.float().cpu().numpy(), zr.grad.cpu().numpy()
    tol = 1e-5 if dtype == torch.float32 else 1e-2       # bf16: the gradient is written in bf16
    np.testing.assert_allclose(g, r, rtol=tol, atol=tol * float(np.abs(r).max()))


@pytest.mark.parametrize("gamma", [2.5, 0.0])
def test_mixup_focal_upstream_scale_and_confident_rows(gamma):
    """p -> 1 rows give (1 - p)^gamma = 0 (no NaN), also at gamma = 0 where the (1 - p)^(gamma - 1) term is
    0 * inf in fp32; and the backward scales by the upstream gradient."""
    from radhip.ops import mixup_focal
    from radhip.train import FocalLoss
    focal = FocalLoss(0.9, gamma)
    z = torch.tensor([[40.0, -40.0], [-40.0, 40.0], [0.3, -0.2], [1.0, 1.0]], device=DEV)
    ya = torch.tensor([0, 1, 1, 0], device=DEV)
    lam = torch.ones(1, device=DEV)
    zr = z.clone().requires_grad_(True)
    (3.0 * _module_loss(focal, zr, ya, ya, lam, 4, 1)).backward()
    zg = z.clone().requires_grad_(True)
    got = mixup_focal(zg, ya, ya, lam, 4, focal, 1)
    (3.0 * got).backward()
    assert torch.isfinite(got) and torch.isfinite(zg.grad).all()
    np.testing.assert_allclose(zg.grad.cpu().numpy(), zr.grad.cpu().numpy(), rtol=1e-5, atol=1e-7)
