"""feature_projection on radhip kernels (radhip/featproj.py) against the autocast module path it replaces.

Reference: HF WavLMFeatureProjection (LayerNorm(512) -> Linear(512, 1024)) as trained under autocast by
src/main.py:1049 (FGM target, src/main.py:74-100). Both paths round the LayerNorm output and the GEMM output once to
the 16-bit dtype; the fused weight gradient is accumulated in fp32 (autocast rounds it to 16 bits first), so the
tolerances are those of 16-bit GEMM outputs: output and input gradient within 2 ulp-scale relative L2 (1e-2 bf16,
2e-3 fp16), parameter gradients within 1e-2 relative L2.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _setup(dt, K, seed=0):
    from radhip.wavlm import FeatureProjection, WavLMConfigLite
    torch.manual_seed(seed)
    cfg = WavLMConfigLite(feat_proj_dropout=0.0)
    fp = FeatureProjection(cfg).cuda()
    with torch.no_grad():
        fp.layer_norm.weight.uniform_(0.5, 1.5)
        fp.layer_norm.bias.uniform_(-0.2, 0.2)
        fp.projection.bias.uniform_(-0.1, 0.1)
    x = (torch.randn(8 * K, 201, 512, device="cuda") * 3 + 0.5).to(dt)
    return fp, x


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("direct", [True, False])
def test_feature_projection_matches_autocast_module(dt, direct):
    from radhip import featproj
    fp, x = _setup(dt, 1)
    dy = torch.randn(8, 201, 1024, device="cuda").to(dt)
    params = list(fp.parameters())
    # reference: the module under autocast, grads accumulated by autograd into fp32 .grad
    for p in params:
        p.grad = torch.zeros_like(p)
    with torch.autocast("cuda", dtype=dt):
        y0 = fp(x)
    y0.backward(dy)
    ref = [p.grad.clone() for p in params]
    # fused: .grad bound (direct accumulation) or unset (returned to autograd)
    for p in params:
        p.grad = torch.zeros_like(p) if direct else None
    with torch.autocast("cuda", dtype=dt):
        assert featproj.eligible(fp, x)
        y1 = featproj.feature_projection(fp, x)
    assert y1.dtype == dt and y1.shape == y0.shape
    y1.backward(dy)
    torch.cuda.synchronize()
    tol = 1e-2 if dt == torch.bfloat16 else 2e-3
    assert _rel(y1, y0) < tol, _rel(y1, y0)
    for p, r in zip(params, ref):
        assert p.grad is not None and p.grad.dtype == torch.float32
        assert _rel(p.grad, r) < 1e-2, (tuple(p.shape), _rel(p.grad, r))


def test_feature_projection_groups_and_input_gradient():
    """K = 4 row groups with their own leaf parameters (the window's clean pass) equal four single-group calls; the
    input gradient (a trainable CNN) matches the module's."""
    from radhip import featproj
    dt = torch.float16
    fp, x = _setup(dt, 4, seed=1)
    x.requires_grad_(True)
    groups = []
    for k in range(4):
        g = []
        for p in fp.parameters():
            c = (p.detach() * (1 + 0.01 * k)).clone().requires_grad_(True)
            c.grad = torch.zeros_like(c)
            g.append(c)
        groups.append(tuple(g))
    dy = torch.randn(32, 201, 1024, device="cuda").to(dt)
    with torch.autocast("cuda", dtype=dt):
        y = featproj.feature_projection(fp, x, groups)
    y.backward(dy)
    dx = x.grad.clone()
    for k in range(4):
        sl = slice(8 * k, 8 * (k + 1))
        xs = x.detach()[sl].clone().requires_grad_(True)
        g = [p.detach().clone().requires_grad_(True) for p in groups[k]]
        with torch.autocast("cuda", dtype=dt):
            yr = torch.nn.functional.linear(torch.nn.functional.layer_norm(xs, (512,), g[0], g[1], 1e-5), g[2], g[3])
        yr.backward(dy[sl])
        assert _rel(y[sl], yr) < 2e-3
        assert _rel(dx[sl], xs.grad) < 1e-2
        for a, b in zip(groups[k], g):
            assert _rel(a.grad, b.grad) < 1e-2, (k, tuple(a.shape), _rel(a.grad, b.grad))
