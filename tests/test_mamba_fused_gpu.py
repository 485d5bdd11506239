"""The fused Bi-Mamba autograd node (radhip/mamba.py MambaBiFn: the PN-BiMamba layer's Mamba.bidirectional,
src/models/DualStreamSEMamba.py:467-481, src/models/modules/mamba_block.py:41-122) against the module path it
replaces (the same HIP kernels as separate autograd nodes: SideLinear, DWConvBidir, SelectiveScan, BiGate,
SplitLast). Both run the same launches on the same operands, so the output is bitwise equal; the gradients agree to
the run-to-run spread of the scan backward's dB / dC (fp32 atomic adds over its channel groups, whose order varies:
in fp16 a rounding of dB | dC can flip between runs and moves every gradient below it by a few ulps). Tolerance:
max-norm relative 1e-2 (bf16) / 2e-3 (fp16). At the bench's B = 8 and B = 32 pass shapes and a ragged one."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


def _run(m, x, dout, fused, dt, monkeypatch):
    import radhip.mamba as rm
    monkeypatch.setattr(rm, "_FUSED", fused)
    for p in m.parameters():
        p.grad = None
    xi = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        y = m.bidirectional(xi)
    y.backward(dout)
    return y.detach(), xi.grad, {k: p.grad.clone() for k, p in m.named_parameters()}


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,L", [(8, 201), (32, 201), (3, 37)])
def test_mamba_fused_bitwise_equals_module_path(B, L, dt, monkeypatch):
    from radhip.mamba import Mamba
    torch.manual_seed(0)
    m = Mamba(144, 16).to(DEV)
    x = torch.randn(B, L, 144, device=DEV).to(dt)          # norm1's output (to_linear: 16-bit)
    dout = (0.1 * torch.randn(B, L, 144, device=DEV)).to(dt)
    y0, dx0, g0 = _run(m, x, dout, False, dt, monkeypatch)
    y1, dx1, g1 = _run(m, x, dout, True, dt, monkeypatch)
    assert y1.dtype == y0.dtype and torch.equal(y1, y0)
    tol = {torch.bfloat16: 1e-2, torch.float16: 2e-3}[dt]
    assert _rel(dx1, dx0) < tol
    for k in g0:
        assert _rel(g1[k], g0[k]) < tol, k
    assert all(torch.isfinite(v).all() for v in g1.values())


def test_colsum_many_matches_torch_sum():
    """ops.colsum_many (csrc/layersum.hip): the fused node's partial-row reductions, against torch's sum in fp64,
    ragged row / column counts, a strided part, two launches bitwise equal (fixed order)."""
    from radhip.ops import colsum_many
    g = torch.Generator(device="cpu").manual_seed(7)
    parts = [torch.randn(208, 5184, generator=g).to(DEV), torch.randn(56, 1440, generator=g).to(DEV),
             torch.randn(7, 33, generator=g).to(DEV), torch.randn(301, 100, generator=g).to(DEV)[:, 3:70]]
    outs = [torch.empty(p.shape[1], device=DEV) for p in parts]
    colsum_many(list(zip(parts, outs)))
    for p, o in zip(parts, outs):
        ref = p.double().sum(0)
        assert float((o.double() - ref).abs().max()) <= 1e-5 * float(p.abs().sum(0).max())
    again = [torch.empty_like(o) for o in outs]
    colsum_many(list(zip(parts, again)))
    assert all(torch.equal(a, b) for a, b in zip(outs, again))
