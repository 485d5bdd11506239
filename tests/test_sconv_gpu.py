"""SincNet residual-stack convolutions on the hand-written MFMA kernels (csrc/sconv.hip) against torch fp32.

Every (C_in, C_out, kernel, padding) the Phase-6 SincNet stack uses (Residual_block, src/models/
DualStreamSEMamba.py:144-200: conv1 2x3 pad (1,1), conv2 2x3 pad (0,1), conv_downsample 1x3 pad (0,1), 32 and
64 channels), widths that are and are not multiples of the 128-position strip. The reference is conv2d in
fp32 on the same bf16-rounded operands (what bf16 autocast feeds MIOpen), so the only differences are fp32
summation order and the bf16 rounding of the outputs: forward and input gradient within bf16 output
rounding (rtol 1e-2 of the tensor scale), weight gradient (fp32 output, reductions over N*H*W) to 2e-3."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from seeded import seeded_array

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = [(32, 32, 2, 1, 23, 300), (32, 32, 2, 0, 24, 300), (32, 64, 2, 1, 23, 129), (64, 64, 2, 0, 24, 257),
         (32, 64, 1, 0, 23, 200), (64, 64, 2, 1, 23, 88), (32, 32, 2, 0, 24, 7163)]


def _t(tag, shape, scale):
    return torch.from_numpy(seeded_array(tag, shape, scale=scale)).float().to(torch.bfloat16).float().to(DEV)


def _close(got, ref, rtol, what):
    scale = float(ref.abs().max())
    np.testing.assert_allclose(got.detach().float().cpu().numpy(), ref.detach().float().cpu().numpy(), rtol=rtol,
                               atol=rtol * scale,
                               err_msg=what)


@pytest.mark.parametrize("ci,co,kh,ph,H,W", CASES)
def test_sconv_forward_and_gradients_match_torch(ci, co, kh, ph, H, W):
    from radhip.ops import SConv
    N = 2
    x = _t(f"sc.x{ci}{W}", (N, ci, H, W), 1.0)
    w = _t(f"sc.w{ci}{co}{kh}", (co, ci, kh, 3), 0.1)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, 1, (ph, 1))
    dy = _t(f"sc.dy{co}{W}", tuple(ref.shape), 1.0)
    (ref * dy).sum().backward()
    xg = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    y = SConv.apply(xg, wg, ph)
    assert y.shape == ref.shape and y.dtype == torch.bfloat16
    _close(y, ref, 1e-2, "y")
    (y.float() * dy).sum().backward()
    _close(xg.grad, xr.grad, 1e-2, "dx")
    _close(wg.grad, wr.grad, 2e-3, "dw")


def test_sconv_bn_selu_matches_conv_then_bnselu():
    from radhip.ops import BnSelu, SConvBnSelu
    N, ci, co, H, W = 2, 32, 64, 23, 300
    x = _t("scb.x", (N, ci, H, W), 1.0)
    w = _t("scb.w", (co, ci, 2, 3), 0.1)
    cb = _t("scb.cb", (co,), 0.1).requires_grad_(True)
    mean = _t("scb.m", (co,), 0.1)
    invstd = 1.0 / torch.sqrt(_t("scb.v", (co,), 0.1).abs() + 0.5)
    gamma = (1 + _t("scb.g", (co,), 0.1)).requires_grad_(True)
    beta = _t("scb.b", (co,), 0.1).requires_grad_(True)
    xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    # reference: torch conv2d on the bf16 operands (bf16 output, as autocast), then the fused BnSelu kernel
    c = F.conv2d(xb.float(), w, None, 1, (1, 1)).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = BnSelu.apply(c, cb, mean, invstd, gamma, beta)
    dy = _t("scb.dy", tuple(ref.shape), 1.0)
    (ref.float() * dy).sum().backward()
    ref_grads = [t.grad.clone() for t in (cb, gamma, beta)]
    for t in (cb, gamma, beta):
        t.grad = None
    got = SConvBnSelu.apply(xb, w, 1, cb, mean, invstd, gamma, beta)
    _close(got, ref, 2e-2, "y")
    (got.float() * dy).sum().backward()
    for g, r, nm in zip((cb.grad, gamma.grad, beta.grad), ref_grads, ("dcb", "dgamma", "dbeta")):
        _close(g, r, 2e-2, nm)


def _bn_params(tag, co):
    cb = _t(f"{tag}.cb", (co,), 0.1).requires_grad_(True)
    mean = _t(f"{tag}.m", (co,), 0.1)
    invstd = 1.0 / torch.sqrt(_t(f"{tag}.v", (co,), 0.1).abs() + 0.5)
    gamma = (1 + _t(f"{tag}.g", (co,), 0.1)).requires_grad_(True)
    beta = _t(f"{tag}.b", (co,), 0.1).requires_grad_(True)
    return cb, mean, invstd, gamma, beta


@pytest.mark.parametrize("ci,co,W", [(32, 32, 300), (32, 32, 7163), (32, 64, 257), (32, 64, 2387), (64, 64, 129)])
def test_sconv_pair_matches_unfused_ops(ci, co, W):
    """conv1 -> BN -> SELU -> conv2 as one op (SConvBnSeluSConv; its backward fuses conv2's input gradient with
    the BN + SELU backward for 32 and 64 channels) against SConvBnSelu followed by SConv (separate kernels): the same
    forward bits; gradients equal up to the summation order of the fp32 channel sums."""
    from radhip.ops import SConv, SConvBnSelu, SConvBnSeluSConv
    N, H = 2, 23
    x = _t(f"sp.x{ci}{W}", (N, ci, H, W), 1.0).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w1 = _t(f"sp.w1{ci}{co}", (co, ci, 2, 3), 0.1)
    w2 = _t(f"sp.w2{co}", (co, co, 2, 3), 0.1)
    prm = _bn_params(f"sp{co}", co)
    dy = _t(f"sp.dy{co}{W}", (N, co, H, W), 1.0)

    def run(fused):
        xs = x.clone().requires_grad_(True)
        a1, a2 = w1.clone().requires_grad_(True), w2.clone().requires_grad_(True)
        for t in (prm[0], prm[3], prm[4]):
            t.grad = None
        if fused:
            out = SConvBnSeluSConv.apply(xs, a1, 1, *prm, a2)
        else:
            out = SConv.apply(SConvBnSelu.apply(xs, a1, 1, *prm), a2, 0)
        (out.float() * dy).sum().backward()
        return out, [xs.grad, a1.grad, a2.grad] + [prm[i].grad.clone() for i in (0, 3, 4)]

    ref, rg = run(False)
    got, gg = run(True)
    assert torch.equal(got, ref)
    for g, r, nm in zip(gg, rg, ("dx", "dw1", "dw2", "dcb", "dgamma", "dbeta")):
        _close(g, r, 2e-3, nm)


def test_bnselu_sconv_block0_matches_unfused():
    from radhip.ops import BnSelu, BnSeluSConv, SConv
    N, C, H, W = 2, 32, 24, 1000
    c = _t("b0p.c", (N, C, H, W), 1.0).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w2 = _t("b0p.w2", (C, C, 2, 3), 0.1)
    prm = _bn_params("b0p", C)
    dy = _t("b0p.dy", (N, C, H - 1, W), 1.0)

    def run(fused):
        cs = c.clone().requires_grad_(True)
        a2 = w2.clone().requires_grad_(True)
        for t in (prm[0], prm[3], prm[4]):
            t.grad = None
        out = BnSeluSConv.apply(cs, *prm, a2) if fused else SConv.apply(BnSelu.apply(cs, *prm), a2, 0)
        (out.float() * dy).sum().backward()
        return out, [cs.grad, a2.grad] + [prm[i].grad.clone() for i in (0, 3, 4)]

    ref, rg = run(False)
    got, gg = run(True)
    assert torch.equal(got, ref)
    assert torch.equal(gg[0], rg[0])           # dc: the same arithmetic on the same bf16 dO1
    for g, r, nm in zip(gg[1:], rg[1:], ("dw2", "dcb", "dgamma", "dbeta")):
        _close(g, r, 2e-3, nm)


@pytest.mark.parametrize("C,W", [(32, 7163), (64, 795), (32, 301)])
def test_res_block_identity_matches_autograd_sum(C, W, monkeypatch):
    """A non-downsampling Residual_block as one op (radhip.ops.ResBlockIdentity: the block input's gradient = conv1's
    input gradient + the identity branch's, added in the input-gradient kernel's epilogue) against the same block
    with autograd summing the two branches (RADHIP_RES_FUSED=0): the same kernels and the same bf16 add, so the
    output, the input gradient and the weight gradients are bit-identical (the bias / BN channel sums come from fp32
    atomics in both paths: equal to their summation order)."""
    from radhip.sinc import Residual_block
    torch.manual_seed(C + W)
    blk = Residual_block([C, C]).cuda()
    with torch.no_grad():
        blk.bn2.running_mean.normal_(0, 0.2)
        blk.bn2.running_var.uniform_(0.5, 2.0)
        blk.bn2.weight.normal_(1, 0.2)
        blk.bn2.bias.normal_(0, 0.2)
        blk.conv2.bias.normal_(0, 0.1)
    blk.eval()
    N, H = 2, 23
    x0 = _t(f"rb.x{C}{W}", (N, C, H, W), 1.0).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = None

    def run(fused):
        nonlocal dy
        monkeypatch.setenv("RADHIP_RES_FUSED", "1" if fused else "0")
        for p in blk.parameters():
            p.grad = None
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
        if dy is None:
            dy = _t(f"rb.dy{C}{W}", tuple(y.shape), 1.0).to(y.dtype).contiguous(memory_format=torch.channels_last)
        y.backward(dy)
        return y.detach(), x.grad.detach().clone(), {n: p.grad.clone() for n, p in blk.named_parameters()
                                                     if p.grad is not None}

    y0, dx0, g0 = run(False)
    y1, dx1, g1 = run(True)
    assert torch.equal(y1, y0)
    assert torch.equal(dx1, dx0)
    assert g1.keys() == g0.keys()
    for k in g0:
        if k in ("conv1.bias", "bn2.weight", "bn2.bias", "conv2.bias"):   # fp32 atomic channel sums: their order
            _close(g1[k], g0[k], 1e-5, k)
        else:
            assert torch.equal(g1[k], g0[k]), k
