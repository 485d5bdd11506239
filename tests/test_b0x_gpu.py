"""SincNet block 0 in one pass (csrc/b0fused.hip, radhip.ops.Block0Fused) against the unfused HIP path it
replaces (Block0Front: rdx_sincnet_b0_fwd + sconv conv2, then ResTail), which the fixture tests pin to the
reference (tests/test_fixtures_gpu.py: the SincNet encoder vs sincnet_encoder.npz; tests/test_model_gpu.py).
The fused forward keeps the unfused kernels' arithmetic and roundings, so its output and window argmax must be
bit-identical; its backward runs the same kernels on recomputed intermediates, so the gradients must be too.
Shapes: the full 64 600-sample block-0 input (H = 23, W = 21490), a ragged width (W % 3 == 2, last strip
partial), tiny widths (W = 3, 5) and one utterance (row chunks).

fp16 storage (libradhip_f16.so): bf16 operands (8-bit significands) make every product of conv1 / conv_downsample and
of conv2's MFMA exact in fp32, so the two paths' different fp32 summation orders cannot show and they agree bit for
bit; fp16 operands (11-bit significands) round those sums, so there the paths agree to one fp16 ulp on a small
fraction of the outputs (measured 0.05 %), and the gradients to fp32 summation order."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _block(seed):
    from radhip.sinc import Residual_block
    torch.manual_seed(seed)
    blk = Residual_block([1, 32], first=True).to(DEV)
    with torch.no_grad():
        for m in (blk.bn2,):
            m.running_mean.normal_(0, 0.2)
            m.running_var.uniform_(0.5, 2.0)
            m.weight.normal_(1, 0.2)
            m.bias.normal_(0, 0.2)
        blk.conv2.bias.normal_(0, 0.1)
        blk.conv_downsample.bias.normal_(0, 0.1)
    blk.eval()
    return blk


def _x(N, H, W, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, 1, H, W, generator=g).to(DEV)
    return x.as_strided((N, 1, H, W), (H * W, 1, W, 1))


def _run(blk, x, fused, monkeypatch, fused_bwd=True, dt=torch.bfloat16):
    monkeypatch.setenv("RADHIP_B0X", "1" if fused else "0")
    monkeypatch.setenv("RADHIP_B0X_BWD", "1" if fused_bwd else "0")
    for p in blk.parameters():
        p.grad = None
    xx = x.detach().clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        y = blk(xx)
    g = torch.Generator(device="cpu").manual_seed(7)
    dy = torch.randn(y.shape, generator=g).to(DEV).to(y.dtype).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    grads = {n: p.grad.clone() for n, p in blk.named_parameters() if p.grad is not None}
    return y.detach(), xx.grad.detach().clone(), grads


SHAPES = [(2, 23, 21490), (3, 23, 1001), (1, 5, 3), (2, 4, 5), (1, 23, 2000), (1, 23, 255), (1, 23, 256)]
# every shape in bf16 storage (libradhip.so), a ragged, a tiny and the full-width shape in fp16 (libradhip_f16.so)
CASES = [(*sh, torch.bfloat16) for sh in SHAPES] + [(*SHAPES[i], torch.float16) for i in (0, 1, 2)]


@pytest.mark.parametrize("N,H,W,dt", CASES)
def test_block0_fused_equals_unfused(N, H, W, dt, monkeypatch):
    """Forward bit-identical; the interim backward (unfused kernels on recomputed intermediates) gives the same dx
    and conv2 weight gradient bit for bit; the other weight / BN gradients come from kernels that reduce with
    atomics (rdx_sincnet_b0_bwd's LDS sums, rdx_sconv_dgrad_bnselu's channel sums), so they match to fp32
    summation order."""
    blk = _block(N + W)
    x = _x(N, H, W, seed=W)
    y1, dx1, g1 = _run(blk, x, True, monkeypatch, fused_bwd=False, dt=dt)
    y0, dx0, g0 = _run(blk, x, False, monkeypatch, dt=dt)
    assert y1.shape == y0.shape == (N, 32, H, W // 3) and y1.dtype == dt
    assert _same_forward(y1, y0)
    assert g1.keys() == g0.keys()
    if dt == torch.bfloat16:
        assert torch.equal(dx1, dx0)
        assert torch.equal(g1["conv2.weight"], g0["conv2.weight"])
    else:           # a window argmax can move with a one-ulp tie break: gradient entries move with it
        assert _rel(dx1, dx0) < 5e-2
    for k in g0:
        assert _rel(g1[k], g0[k]) < (1e-5 if dt == torch.bfloat16 else 5e-2), k


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _same_forward(y1, y0):
    """bf16: bit-identical. fp16: bit-identical on >= 99.8 % of the outputs, elsewhere within one fp16 ulp of the
    pre-pool terms (conv2 + conv_downsample, |.| <= ~4: 2^-9 absolute; the sum can cancel, so the bound is not
    relative to the output)."""
    if y0.dtype == torch.bfloat16:
        return torch.equal(y1, y0)
    a, b = y1.float(), y0.float()
    return bool(((a - b).abs() <= 2.0 ** -9 + 2.0 ** -10 * b.abs()).all()) and float((y1 != y0).float().mean()) < 2e-3


@pytest.mark.parametrize("N,H,W,dt", CASES)
def test_block0_fused_backward(N, H, W, dt, monkeypatch):
    """The one-pass backward (rdx_b0x_bwd) against the unfused kernels: the same bf16 dc / ds / out1 and MFMA
    order, so the only differences are the order of the fp32 sums (dx over 288 terms, the weight and BN sums over
    every position): relative L2 below 1e-5 for every gradient. A second run gives the same bits (no atomics)."""
    blk = _block(N + W + 1)
    x = _x(N, H, W, seed=W + 1)
    y1, dx1, g1 = _run(blk, x, True, monkeypatch, fused_bwd=True, dt=dt)
    y0, dx0, g0 = _run(blk, x, False, monkeypatch, dt=dt)
    assert _same_forward(y1, y0)
    tol = 1e-5 if dt == torch.bfloat16 else 5e-2
    assert _rel(dx1, dx0) < tol
    assert g1.keys() == g0.keys()
    for k in g0:
        assert _rel(g1[k], g0[k]) < tol, (k, _rel(g1[k], g0[k]))
    y2, dx2, g2 = _run(blk, x, True, monkeypatch, fused_bwd=True, dt=dt)
    assert torch.equal(dx2, dx1) and all(torch.equal(g2[k], g1[k]) for k in g1)
