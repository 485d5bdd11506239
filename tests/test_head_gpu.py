"""Fused head pieces (radhip/head.py, csrc/head.hip) against the autocast module path they replace.

Reference: SELayer (src/models/DualStreamSEMamba.py:492-531) and Model.forward's attention pooling (:700-770) under
autocast (src/main.py:1049). The fused kernels
round every intermediate to 16 bits where autocast's ops would, so output and input gradient agree to 16-bit
rounding of a few elements (relative L2 <= 2e-3 fp16, 1e-2 bf16); the fc weight gradients are fp32 sums of the same
products in a different order (relative L2 <= 1e-2).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B", [8, 32])
@pytest.mark.parametrize("direct", [True, False])
def test_se_layer_matches_autocast_module(dt, B, direct, monkeypatch):
    import models.DualStreamSEMamba as M
    torch.manual_seed(B)
    se = M.SELayer(144, 16).cuda()
    x = (torch.randn(B, 201, 144, device="cuda") * 2).to(dt).requires_grad_(True)
    dy = torch.randn(B, 201, 144, device="cuda").to(dt)
    params = [se.fc[0].weight, se.fc[2].weight]
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(M, "_SE_FUSED", fused)
        for p in params:
            p.grad = torch.zeros_like(p) if (direct or not fused) else None
        x.grad = None
        with torch.autocast("cuda", dtype=dt):
            y = se(x)
        assert y.dtype == dt
        y.backward(dy)
        res[fused] = (y.detach().clone(), x.grad.clone(), [p.grad.clone() for p in params])
    torch.cuda.synchronize()
    tol = 2e-3 if dt == torch.float16 else 1e-2
    (y0, dx0, g0), (y1, dx1, g1) = res[False], res[True]
    assert _rel(y1, y0) < tol, _rel(y1, y0)
    assert _rel(dx1, dx0) < tol, _rel(dx1, dx0)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-2, _rel(a, b)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B", [8, 32])
@pytest.mark.parametrize("direct", [True, False])
def test_attention_pooling_matches_autocast_module(dt, B, direct):
    """radhip.head.attn_pool against Model.forward's tail (softmax over time of the 1-output linear, then the
    weighted sum) under autocast: features, the gradient of f and the linear's weight / bias gradients."""
    import torch.nn.functional as F
    from radhip import head
    from radhip.linear import SideLinear
    torch.manual_seed(B + 1)
    lin = SideLinear(144, 1).cuda()
    f = (torch.randn(B, 201, 144, device="cuda")).to(dt).requires_grad_(True)
    dfe = torch.randn(B, 144, device="cuda").to(dt)
    res = {}
    for fused in (False, True):
        for p in (lin.weight, lin.bias):
            p.grad = torch.zeros_like(p) if (direct or not fused) else None
        f.grad = None
        with torch.autocast("cuda", dtype=dt):
            if fused:
                assert head.pool_eligible(f, lin)
                feat = head.attn_pool(f, lin.weight, lin.bias)
            else:
                attn = F.softmax(lin(f), dim=1)
                feat = torch.matmul(attn.transpose(1, 2), f).squeeze(1)
        assert feat.dtype == dt and feat.shape == (B, 144)
        feat.backward(dfe)
        res[fused] = (feat.detach().clone(), f.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone())
    torch.cuda.synchronize()
    tol = 2e-3 if dt == torch.float16 else 1e-2
    for a, b in zip(res[True][:2], res[False][:2]):
        assert _rel(a, b) < tol, _rel(a, b)
    assert _rel(res[True][2], res[False][2]) < 1e-2, _rel(res[True][2], res[False][2])
    # d bias = sum over (b, t) of the softmax gradient, which sums to zero per utterance in exact arithmetic: both
    # sides are rounding residue, so it is held to an absolute bound at the scale of the weight gradient
    dbias = float((res[True][3] - res[False][3]).abs().max())
    assert dbias <= tol * float(res[False][2].abs().max()), (dbias, float(res[False][2].abs().max()))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 201, 29, 144), (32, 201, 29, 144), (3, 100, 13, 16)])
def test_upcat_matches_interpolate_cat(dt, shape):
    """radhip.head.upcat against DualStreamFusion's alignment (F.interpolate 'nearest' of the SincNet features to
    the WavLM frame count, then cat) under autocast: the forward is a gather (bit-exact); the SincNet half's gradient
    is the upsample backward's per-frame fp32 sums rounded once (relative L2 <= 1e-3), the WavLM half's a view."""
    import torch.nn.functional as F
    from radhip import head
    B, T1, T2, C = shape
    torch.manual_seed(T1 + T2)
    fw = torch.randn(B, T1, C, device="cuda").to(dt).requires_grad_(True)
    fs = torch.randn(B, T2, C, device="cuda").to(dt).requires_grad_(True)
    dout = torch.randn(B, T1, 2 * C, device="cuda").to(dt)
    res = {}
    for fused in (False, True):
        fw.grad = fs.grad = None
        with torch.autocast("cuda", dtype=dt):
            if fused:
                assert head.upcat_eligible(fw, fs)
                out = head.upcat(fw, fs)
            else:
                up = F.interpolate(fs.permute(0, 2, 1), size=T1, mode="nearest").permute(0, 2, 1)
                out = torch.cat([fw, up.to(fw.dtype)], dim=-1)
        assert out.dtype == dt and out.shape == (B, T1, 2 * C)
        out.backward(dout)
        res[fused] = (out.detach().clone(), fw.grad.clone(), fs.grad.clone())
    torch.cuda.synchronize()
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    assert _rel(res[True][2], res[False][2]) < 1e-3, _rel(res[True][2], res[False][2])
