"""Parity of every HIP kernel (through the C ABI) with the oracle on the same seeded inputs."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from seeded import seeded_array, seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


# ------------------------------------------------------------------------------- SincConv ----
@pytest.mark.parametrize("mask", [(0, 0), (12, 31), (60, 70)])
def test_sincconv_absmaxpool_full_length(mask):
    from oracle.sinc import sinc_filterbank, sincconv_absmaxpool
    from radhip.ops import sincconv_absmaxpool as hip_sinc
    bank = sinc_filterbank()
    x = seeded_array("k.sinc", (2, 64600), scale=0.1).astype(np.float32)
    out = hip_sinc(torch.from_numpy(x).to(DEV), bank.to(DEV), *mask).cpu().numpy()
    ref = sincconv_absmaxpool(x, bank.numpy(), *mask)
    assert out.shape == ref.shape == (2, 23, 21490)
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=2e-6)


@pytest.mark.parametrize("mask", [(0, 0), (12, 31), (60, 70)])
@pytest.mark.parametrize("L", [64600, 3001])
def test_sincconv_f16_mfma_vs_oracle(mask, L):
    """The autocast form (f16 MFMA; the reference's autocast runs this conv in fp16): equal to the fp64 oracle
    on the fp16-rounded waveform and bank up to fp32 accumulation order, and to the exact fp32 conv within fp16
    input rounding. L = 3001: a partial last block (positions past the utterance read as zeros)."""
    from oracle.sinc import sinc_filterbank, sincconv_absmaxpool
    from radhip.ops import sincconv_absmaxpool as hip_sinc
    bank = sinc_filterbank()
    x = seeded_array(f"k.sinc16.{L}", (3, L), scale=0.1).astype(np.float32)
    with torch.autocast("cuda", dtype=torch.float16):
        out = hip_sinc(torch.from_numpy(x).to(DEV), bank.to(DEV), *mask).cpu().numpy()
    x16 = x.astype(np.float16).astype(np.float32)
    b16 = bank.numpy().astype(np.float16).astype(np.float32)
    ref16 = sincconv_absmaxpool(x16, b16, *mask)
    assert out.shape == ref16.shape == (3, 23, (L - 128) // 3)
    np.testing.assert_allclose(out, ref16, rtol=1e-4, atol=2e-6)
    ref = sincconv_absmaxpool(x, bank.numpy(), *mask)
    assert float(np.abs(out - ref).max()) <= 2e-3 * float(np.abs(ref).max())
    # the per-utterance device mask (the window's graph-replayable form) gives the same rows
    md = torch.tensor([list(mask)] * 3, dtype=torch.int32, device=DEV)
    with torch.autocast("cuda", dtype=torch.float16):
        out2 = hip_sinc(torch.from_numpy(x).to(DEV), bank.to(DEV), mask_dev=md).cpu().numpy()
    assert np.array_equal(out, out2)
    # bf16 autocast keeps the exact fp32 kernel
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out3 = hip_sinc(torch.from_numpy(x).to(DEV), bank.to(DEV), *mask).cpu().numpy()
    np.testing.assert_allclose(out3, ref, rtol=1e-4, atol=2e-6)


def test_sincconv_golden(golden):
    from radhip.ops import sincconv_absmaxpool as hip_sinc
    g = golden("sinc_conv.npz")
    out = hip_sinc(torch.from_numpy(g["x"][:, 0]).to(DEV), torch.from_numpy(g["band_pass"]).to(DEV),
                   int(g["mask_lo"]), int(g["mask_hi"])).cpu().numpy()
    np.testing.assert_allclose(out, g["pooled_masked"], rtol=1e-4, atol=1e-6)


# ------------------------------------------------------------------------------- Bi-Mamba -----
def _mamba_pair(d_model, seed):
    from oracle.mamba import MambaRef
    from radhip.mamba import Mamba
    ref = MambaRef(d_model, 16)
    seeded_fill_(ref, seed=seed)
    hip = Mamba(d_model, 16)
    hip.load_state_dict(ref.state_dict())
    return ref.double(), hip.to(DEV)


# L covers fewer checkpoint chunks than time segments (19, 23: the segmented forward's empty segments), chunk-
# aligned and ragged lengths, and the Phase-6 201
@pytest.mark.parametrize("scan2", ["1", "0"])     # csrc/scan2.hip (chunked, the default) and csrc/bimamba.hip
@pytest.mark.parametrize("dirs,d_model,L,B", [(1, 16, 23, 2), (2, 16, 19, 2), (2, 144, 201, 2), (1, 144, 201, 3),
                                              (2, 32, 64, 2), (2, 32, 65, 1), (2, 16, 7, 2), (2, 16, 16, 1),
                                              (2, 24, 33, 2)])
def test_mamba_fwd_bwd_fp32(dirs, d_model, L, B, scan2, monkeypatch):
    """Also L = 16 (one full chunk, no checkpoint), L = 33 (a 1-step last chunk) and Di = 48 (a partial 32-channel
    group in csrc/scan2.hip)."""
    monkeypatch.setenv("RADHIP_SCAN2", scan2)
    from oracle.mamba import bimamba_ref
    ref, hip = _mamba_pair(d_model, 100 + d_model)
    x = seeded_array(f"k.mamba.{d_model}.{L}", (B, L, d_model))
    r = seeded_array(f"k.mamba.r.{d_model}.{L}", (B, L, d_model))
    xr = torch.from_numpy(x).requires_grad_(True)
    yr = bimamba_ref(ref, xr) if dirs == 2 else ref(xr)
    (yr * torch.from_numpy(r)).sum().backward()
    xh = torch.from_numpy(x).float().to(DEV).requires_grad_(True)
    yh = hip.bidirectional(xh) if dirs == 2 else hip(xh)
    (yh * torch.from_numpy(r).float().to(DEV)).sum().backward()
    assert _rel(yh.detach().cpu(), yr.detach()) < 2e-5
    assert _rel(xh.grad.cpu(), xr.grad) < 1e-4
    for (k, pr), (k2, ph) in zip(ref.named_parameters(), hip.named_parameters()):
        assert k == k2
        assert _rel(ph.grad.cpu(), pr.grad) < 2e-4, k


def test_mamba_golden_reference_block(golden):
    """Product Mamba on the reference MambaBlock's own fixture (fp32)."""
    from radhip.mamba import Mamba
    g = golden("mamba_block.npz")
    m = Mamba(16, 16)
    seeded_fill_(m, seed=21)
    m = m.to(DEV)
    x = torch.from_numpy(g["x"]).to(DEV).requires_grad_(True)
    y = m(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["y"], rtol=1e-4, atol=1e-5)
    (y * torch.from_numpy(g["r"]).to(DEV)).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), g["dx"], rtol=1e-3, atol=1e-5)
    for k, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g[f"grad:{k}"], rtol=2e-3, atol=1e-5, err_msg=k)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_scan2_matches_segmented_scan_16bit(dt):
    """The chunked scan against csrc/bimamba.hip's segmented kernels at the Phase-6 shape in bf16 / fp16 storage
    (libradhip.so / libradhip_f16.so): the same outputs and gradients up to fp32 summation order (both chains run
    in fp32)."""
    from radhip import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    dirs, B, L, D, N, R = 2, 4, 201, 288, 16, 9
    u = torch.randn(dirs, B, L, D, device=DEV, generator=g).to(dt)
    delta = (0.5 * torch.randn(dirs, B, L, D, device=DEV, generator=g)).to(dt)
    xdbl = torch.randn(dirs, B, L, R + 2 * N, device=DEV, generator=g).to(dt)
    A_log = torch.log(torch.arange(1, N + 1, device=DEV, dtype=torch.float32)).repeat(D, 1)
    Dp = torch.randn(D, device=DEV, generator=g)
    bias = 0.1 * torch.randn(D, device=DEV, generator=g)
    dy = torch.randn(dirs, B, L, D, device=DEV, generator=g)
    outs = {}
    for kind in ("0", "1"):
        os.environ["RADHIP_SCAN2"] = kind
        try:
            leaves = [t.clone().requires_grad_() for t in (u, delta, xdbl, A_log, Dp, bias)]
            uu, dd, xx, al, dp, bb = leaves
            y = ops.SelectiveScan.apply(uu, dd, al, xx[..., R:R + N], xx[..., R + N:], dp, bb)
            y.backward(dy)
            outs[kind] = [y.detach()] + [t.grad for t in leaves]
        finally:
            os.environ.pop("RADHIP_SCAN2", None)
    for a, b in zip(outs["1"], outs["0"]):
        assert _rel(a.float().cpu(), b.float().cpu()) < 1e-2


def test_mamba_bf16_autocast():
    from oracle.mamba import bimamba_ref
    ref, hip = _mamba_pair(144, 7)
    x = seeded_array("k.mamba.bf16", (4, 201, 144))
    with torch.no_grad():
        yr = bimamba_ref(ref, torch.from_numpy(x)).numpy()
    xh = torch.from_numpy(x).float().to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yh = hip.bidirectional(xh)
    yh.float().sum().backward()
    assert torch.isfinite(xh.grad).all()
    assert _rel(yh.float().detach().cpu(), yr) < 3e-2


def test_dwconv_both_directions_vs_torch():
    from radhip.ops import DWConvBidir
    B, L, D = 3, 57, 40
    xz = torch.randn(B, L, 2 * D, device=DEV, dtype=torch.float64).float().requires_grad_(True)
    w = torch.randn(D, 1, 4, device=DEV).requires_grad_(True)
    b = torch.randn(D, device=DEV).requires_grad_(True)
    u = DWConvBidir.apply(xz[..., :D], w, b, 2)
    xt = xz[..., :D].transpose(1, 2)
    u0 = F.silu(F.conv1d(xt, w, b, padding=3, groups=D)[..., :L]).transpose(1, 2)
    u1 = torch.flip(F.silu(F.conv1d(torch.flip(xt, [2]), w, b, padding=3, groups=D)[..., :L]), [2]).transpose(1, 2)
    torch.testing.assert_close(u[0], u0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(u[1], u1, rtol=1e-5, atol=1e-6)
    r = torch.randn_like(u)
    g_h = torch.autograd.grad((u * r).sum(), (xz, w, b))
    g_t = torch.autograd.grad((torch.stack([u0, u1]) * r).sum(), (xz, w, b))
    for a, c in zip(g_h, g_t):
        torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-5)


# -------------------------------------------------------------------- layer-weighted sum -----
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_layer_weighted_sum(dtype):
    from radhip.ops import layer_weighted_sum
    hs = [torch.randn(2, 201, 1024, device=DEV).to(dtype).requires_grad_(True) for _ in range(25)]
    w = torch.randn(25, device=DEV).requires_grad_(True)
    out = layer_weighted_sum(hs, w)
    ref = (F.softmax(w, 0).view(-1, 1, 1, 1) * torch.stack([h.float() for h in hs])).sum(0)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)
    g = torch.randn_like(ref).to(dtype).float()   # the incoming gradient has the states' dtype
    gh = torch.autograd.grad((out.float() * g).sum(), [w] + hs)
    gr = torch.autograd.grad((ref * g).sum(), [w] + hs)
    torch.testing.assert_close(gh[0], gr[0], rtol=1e-3 if dtype == torch.float32 else 5e-2, atol=1e-3)
    for a, c in zip(gh[1:], gr[1:]):
        torch.testing.assert_close(a.float(), c.float(), rtol=tol, atol=tol)


# ------------------------------------------------------------------------------- RawBoost -----
def _records_from_draws(draws, lens, seed=0):
    from radhip._lib import RawboostUtt
    recs, off = [], 0
    for d, n in zip(draws, lens):
        r = RawboostUtt()
        r.offset, r.len, r.algo, r.seed = off, n, d["algo"], seed
        if "lnl" in d:
            b = np.zeros(6)
            b[:len(d["lnl"]["b"])] = d["lnl"]["b"]
            a = np.zeros(6)
            a[:len(d["lnl"]["a"])] = d["lnl"]["a"]
            r.b[:] = list(b)
            r.a[:] = list(a)
            r.n_a = len(d["lnl"]["a"]) - 1
            r.f = d["lnl"]["f"]
        if "isd" in d:
            r.beta = d["isd"]["beta"]
        if "ssi" in d:
            r.snr_db = d["ssi"]["snr"]
        recs.append(r)
        off += n
    return recs


def test_rawboost_batch_exact_with_reference_draws():
    from oracle import rawboost as orb
    from radhip.ops import rawboost_batch
    lens = [64000, 64000, 37000, 64000, 5000, 64000, 64000, 64000]
    algos = [1, 2, 3, 4, 1, 4, 0, 3]
    rng = np.random.RandomState(42)
    xs = [(0.1 * rng.randn(n)).astype(np.float32) for n in lens]
    draws, refs = [], []
    for x, a in zip(xs, algos):
        d = orb.draw_process(len(x), [a], rng) if a else {"algo": 0}
        draws.append(d)
        refs.append(orb.apply_process(x.astype(np.float64), d))
    isd = np.concatenate([d["isd"]["nm"] if "isd" in d else np.zeros(n) for d, n in zip(draws, lens)])
    ssi = np.concatenate([d["ssi"]["noise"] if "ssi" in d else np.zeros(n) for d, n in zip(draws, lens)])
    flat = torch.from_numpy(np.concatenate(xs)).to(DEV)
    out = rawboost_batch(flat, _records_from_draws(draws, lens), torch.from_numpy(isd).to(DEV),
                         torch.from_numpy(ssi).to(DEV)).cpu().numpy()
    off = 0
    for n, ref, a in zip(lens, refs, algos):
        np.testing.assert_allclose(out[off:off + n], ref.astype(np.float32), rtol=2e-6, atol=2e-7,
                                   err_msg=f"algo {a}")
        off += n


def test_rawboost_philox_statistics():
    from radhip.ops import rawboost_batch
    n = 64000
    x = torch.full((3 * n,), 0.1, device=DEV)
    draws = [{"algo": 2, "isd": {"beta": 5}}, {"algo": 2, "isd": {"beta": 9}}, {"algo": 3, "ssi": {"snr": 20.0}}]
    out = rawboost_batch(x, _records_from_draws(draws, [n] * 3, seed=1234)).cpu().numpy().astype(np.float64)
    for i, beta in enumerate([5, 9]):
        seg = out[i * n:(i + 1) * n]
        frac = np.mean(seg != np.float32(0.1))
        assert abs(frac - 1 / beta) < 0.01
        nz = (seg[seg != np.float32(0.1)] - 0.1) / 0.2      # = noise samples
        assert abs(nz.mean()) < 0.05 and abs(nz.std() - 1) < 0.05
    seg = out[2 * n:]
    noise = seg - 0.1
    snr = 10 * np.log10(np.sum(np.full(n, 0.1) ** 2) / np.sum(noise ** 2))
    assert abs(snr - 20.0) < 0.01


# ---------------------------------------------------------------------- codec resampling ----
@pytest.mark.parametrize("sr", [8000, 6000, 4000])
def test_resample_roundtrip(sr):
    from oracle.resample import resample
    from radhip._lib import ResampleJob
    from radhip.ops import resample_batch, resample_kernel
    x = seeded_array(f"k.rs.{sr}", (30011,), scale=0.1)
    kd, wd, ogd, ngd = resample_kernel(16000, sr)
    ku, wu, ogu, ngu = resample_kernel(sr, 16000)
    kern = torch.cat([kd.reshape(-1), ku.reshape(-1)]).to(DEV)
    n_down = -(-ngd * len(x) // ogd)
    n_up = -(-ngu * n_down // ogu)
    xin = torch.from_numpy(x).float().to(DEV)
    mid = torch.empty(n_down, device=DEV)
    out = torch.empty(n_up, device=DEV)
    resample_batch(xin, mid, kern, [ResampleJob(0, len(x), 0, n_down, ogd, ngd, wd, 0)])
    resample_batch(mid, out, kern, [ResampleJob(0, n_down, 0, n_up, ogu, ngu, wu, kd.numel())])
    ref_mid = resample(x.astype(np.float32).astype(np.float64), 16000, sr)
    ref = resample(ref_mid, sr, 16000)
    np.testing.assert_allclose(mid.cpu().numpy(), ref_mid, rtol=0, atol=2e-6)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=0, atol=4e-6)


# ----------------------------------------------------------------------- pad + mixup ---------
def test_pad_mixup_gather():
    from oracle.data import pad
    from radhip.ops import pad_mixup
    lens = [1000, 64600, 70000, 64000]
    sig = [seeded_array(f"k.pad.{n}", (n,)).astype(np.float32) for n in lens]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    starts = [0, 0, 3333, 0]
    flat = torch.from_numpy(np.concatenate(sig)).to(DEV)
    perm = [2, 0, 3, 1]
    lam = 0.3
    out = pad_mixup(flat, offs, lens, starts, 64600, perm, lam).cpu().numpy()
    base = [pad(s) if n < 64600 else s[st:st + 64600] for s, n, st in zip(sig, lens, starts)]
    for b in range(4):
        np.testing.assert_allclose(out[b], lam * base[b] + (1 - lam) * base[perm[b]], rtol=1e-6, atol=1e-7)
    plain = pad_mixup(flat, offs, lens, starts, 64600).cpu().numpy()
    for b in range(4):
        np.testing.assert_array_equal(plain[b], base[b])


# ------------------------------------------------------------------------------------ FGM ----
def test_fgm_attack_matches_reference_fixture(golden):
    from radhip.ops import fgm_attack
    g = golden("train_toy.npz")
    keys = [k.split(":", 1)[1] for k in g if k.startswith("fgm_before:") and "feature_projection" in k]
    ps = [torch.from_numpy(g[f"fgm_before:{k}"]).to(DEV).contiguous() for k in keys]
    gs = [torch.from_numpy(g[f"fgm_grad:{k}"]).to(DEV).contiguous() for k in keys]
    bk = [torch.empty_like(p) for p in ps]
    fgm_attack(ps, gs, bk, 0.5)
    for k, p, b in zip(keys, ps, bk):
        np.testing.assert_allclose(p.cpu().numpy(), g[f"fgm_attacked:{k}"], rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(b.cpu().numpy(), g[f"fgm_before:{k}"])
    # zero gradient: untouched
    p = torch.ones(10, device=DEV)
    fgm_attack([p], [torch.zeros(10, device=DEV)], [torch.empty(10, device=DEV)], 0.5)
    assert torch.equal(p, torch.ones(10, device=DEV))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("first", [True, False])
def test_fused_residual_block_matches_torch(dtype, first):
    """SincNet Residual_block with frozen BN: fused NHWC epilogues (bnselu, res_tail) == the torch
    conv/bn/selu/add/maxpool graph, forward and every gradient (incl. a W % 3 tail and ties)."""
    from radhip.sinc import Residual_block
    torch.manual_seed(0)
    filts = [1, 32] if first else [32, 32]
    blk = Residual_block(filts, first=first).to(DEV)
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.5, 0.5)
            m.running_var.uniform_(0.5, 2.0)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    blk.eval()                                    # frozen BN (freeze_bn)
    x = torch.randn(2, filts[0], 7, 101, device=DEV)
    x[..., :3] = 0.0                              # ties inside the first pooling windows
    x = x.contiguous(memory_format=torch.channels_last)
    bf16 = dtype != torch.float32            # a 16-bit autocast dtype (bf16 or fp16)

    def run(fused, amp):
        b = Residual_block(filts, first=first).to(DEV)
        b.load_state_dict(blk.state_dict())
        b.eval()
        if not fused:
            b._fused_ok = lambda _x: False         # torch conv/bn/selu/add/maxpool graph
        xx = x.detach().clone().requires_grad_()
        with torch.autocast("cuda", dtype=dtype if amp else torch.bfloat16, enabled=amp):
            y = b(xx)
        assert (not fused) or b._fused_ok(xx)
        y.backward(g.to(y.dtype))
        out = {"y": y.float(), "dx": xx.grad.float()}
        out.update({n: p.grad.float() for n, p in b.named_parameters() if p.grad is not None})
        return out

    torch.manual_seed(1)
    g = torch.randn(2, filts[1], 7, 101 // 3, device=DEV)
    fused = run(True, bf16)
    ref32 = run(False, False)
    if not bf16:
        for n, b in ref32.items():
            scale = b.abs().max().item() + 1e-6
            torch.testing.assert_close(fused[n] / scale, b / scale, rtol=1e-4, atol=1e-5, msg=n)
    else:
        # 16-bit rounding can flip a max-pool argmax between near-equal values, which moves whole gradient
        # entries: hold the fused path to torch's own graph's distance (same autocast dtype) from the fp32 result
        tb16 = run(False, True)
        for n, b in ref32.items():
            e_f = ((fused[n] - b).norm() / (b.norm() + 1e-12)).item()
            e_t = ((tb16[n] - b).norm() / (b.norm() + 1e-12)).item()
            assert e_f <= 1.5 * e_t + 1e-2, (n, e_f, e_t)


def _toeplitz_bias(H, T, seed=0):
    """A random relative-position bias: bias[h, i, j] = table[h, j - i + T - 1] (WavLM's bias depends on the
    key - query offset only, and the kernels take it in that form)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    tab = torch.randn(H, 2 * T - 1, generator=g).to(DEV)
    i = torch.arange(T, device=DEV)
    return tab[:, i[None, :] - i[:, None] + T - 1]


@pytest.mark.parametrize("bwd", ["fused", "fused_keysplit", "split"])
@pytest.mark.parametrize("p_drop,H", [(0.0, 4), (0.1, 4), (0.1, 16)])
def test_gated_attention_matches_torch(p_drop, H, bwd, monkeypatch):
    """Fused MFMA WavLM attention (gated rel-pos bias formed in registers, hashed dropout) vs an fp32
    torch reference fed the same bf16 inputs and the kernel's own dropout mask; forward and the q/k/v/
    gate gradients, through every backward path (the one-launch fused kernel, its two-workgroups-per-(b, h)
    key-split form with the last-arriver dQ / d gate combine, and the dQ + dK/dV pair).
    k is a strided column view of a fused q|k|v tensor (as in the model). H = 16 takes the fused
    kernel's head-per-XCD block mapping."""
    from radhip.ops import GatedAttention, attention_dropout_mask
    monkeypatch.setenv("RADHIP_ATTN_BWD", "split" if bwd == "split" else "fused")
    monkeypatch.setenv("RADHIP_ATTN_SPLIT", "1" if bwd == "fused_keysplit" else "0")
    torch.manual_seed(0)
    B, T, D = 2, 201, 64
    E = H * D
    qkv = (0.5 * torch.randn(B, T, 3 * E, device=DEV)).to(torch.bfloat16)
    q = qkv[..., :E].contiguous().requires_grad_()
    k_full = qkv.clone().requires_grad_()
    k = k_full[..., E:2 * E]
    v = qkv[..., 2 * E:].contiguous().requires_grad_()
    gate = torch.rand(B, T, H, device=DEV).mul(2).requires_grad_()
    pb = _toeplitz_bias(H, T)
    seed = torch.tensor([1234567], dtype=torch.int64, device=DEV)
    o = GatedAttention.apply(q, k, v, gate, pb, seed, p_drop, 3)
    go = torch.randn(B, T, E, device=DEV).to(torch.bfloat16)
    o.backward(go)
    # reference
    qr, kr, vr = (t.detach().float().view(B, T, H, D).transpose(1, 2).requires_grad_() for t in (q, k, v))
    gr = gate.detach().clone().requires_grad_()
    s = qr @ kr.transpose(-1, -2) * 0.125 + gr.permute(0, 2, 1).unsqueeze(-1) * pb.unsqueeze(0)
    pr = torch.softmax(s, -1)
    if p_drop > 0:
        keep = attention_dropout_mask(seed, 3, p_drop, (B, H, T, T)).float()
        assert abs(keep.mean().item() - (1 - p_drop)) < 0.01
        pr = pr * keep / (1 - p_drop)
    orf = (pr @ vr).transpose(1, 2).reshape(B, T, E)
    orf.backward(go.float())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()
    assert rel(o, orf) < 1e-2
    assert rel(q.grad, qr.grad.transpose(1, 2).reshape(B, T, E)) < 2e-2
    assert rel(k_full.grad[..., E:2 * E], kr.grad.transpose(1, 2).reshape(B, T, E)) < 2e-2
    assert k_full.grad[..., :E].abs().max().item() == 0
    assert rel(v.grad, vr.grad.transpose(1, 2).reshape(B, T, E)) < 2e-2
    assert rel(gate.grad, gr.grad) < 2e-2
    # a new seed gives a new mask; the same seed the same output
    if p_drop > 0:
        o2 = GatedAttention.apply(q, k, v, gate, pb, seed, p_drop, 3)
        assert torch.equal(o2, o)
        o3 = GatedAttention.apply(q, k, v, gate, pb, seed + 1, p_drop, 3)
        assert not torch.equal(o3, o)


@pytest.mark.parametrize("B,T,H", [(1, 33, 2), (3, 64, 1), (2, 224, 8), (1, 225, 2), (1, 256, 2), (3, 2, 16)])
def test_gated_attention_ragged_lengths(B, T, H):
    """Sequence lengths with a one-row last tile, an exact tile multiple, the fused backward's 224-row
    maximum, the first length past it (dQ + dK/dV pair), the 256-row maximum and two frames: forward
    and gradients against the fp32 torch reference (no dropout). B * H = 16 and 48 take the key-split fused
    backward (the T = 2 case gives its second workgroup no key tile)."""
    from radhip.ops import GatedAttention
    torch.manual_seed(T)
    E = H * 64
    q, k, v = ((0.5 * torch.randn(B, T, E, device=DEV)).to(torch.bfloat16).requires_grad_() for _ in range(3))
    gate = (torch.rand(B, T, H, device=DEV) * 2).requires_grad_()
    pb = _toeplitz_bias(H, T, seed=T)
    o = GatedAttention.apply(q, k, v, gate, pb, None, 0.0, 0)
    go = torch.randn(B, T, E, device=DEV).to(torch.bfloat16)
    o.backward(go)
    qr, kr, vr = (t.detach().float().view(B, T, H, 64).transpose(1, 2).requires_grad_() for t in (q, k, v))
    gr = gate.detach().clone().requires_grad_()
    s = qr @ kr.transpose(-1, -2) * 0.125 + gr.permute(0, 2, 1).unsqueeze(-1) * pb.unsqueeze(0)
    orf = (torch.softmax(s, -1) @ vr).transpose(1, 2).reshape(B, T, E)
    orf.backward(go.float())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()
    assert rel(o, orf) < 1e-2
    assert rel(q.grad, qr.grad.transpose(1, 2).reshape(B, T, E)) < 2e-2
    assert rel(k.grad, kr.grad.transpose(1, 2).reshape(B, T, E)) < 2e-2
    assert rel(v.grad, vr.grad.transpose(1, 2).reshape(B, T, E)) < 2e-2
    assert rel(gate.grad, gr.grad) < 2e-2


def test_posconv_matches_torch():
    """WavLM positional conv (grouped conv1d 16 x 64 channels, 128 taps, padding 64, last frame dropped,
    GELU; csrc/posconv.hip) vs torch fp32 on the same bf16 operands: output and input gradient. T <= 256 takes
    the one-workgroup-per-(b, g) kernel (256 = every wave with two row tiles, 193 = the last wave with one), longer
    sequences the row-block kernel (300)."""
    from radhip.ops import PosConv, posconv_weights
    torch.manual_seed(0)
    w = torch.randn(1024, 64, 128, device=DEV) * 0.01
    bias = torch.randn(1024, device=DEV) * 0.1
    wk, wkt = posconv_weights(w)
    wr = w.to(torch.bfloat16).float()
    for B, T in ((2, 201), (1, 37), (1, 129), (1, 256), (1, 193), (1, 300)):
        h = torch.randn(B, T, 1024, device=DEV).to(torch.bfloat16).requires_grad_()
        y = PosConv.apply(h, wk, wkt, bias)
        go = torch.randn(B, T, 1024, device=DEV).to(torch.bfloat16)
        y.backward(go)
        hr = h.detach().float().requires_grad_()
        yr = F.gelu(F.conv1d(hr.transpose(1, 2), wr, bias, padding=64, groups=16)[:, :, :-1]).transpose(1, 2)
        yr.backward(go.float())
        assert y.shape == yr.shape
        assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2, (B, T)
        assert ((h.grad.float() - hr.grad).norm() / hr.grad.norm()).item() < 2e-2, (B, T)


@pytest.mark.parametrize("N,H,W", [(2, 23, 301), (5, 1, 33), (1, 3, 2)])
def test_sincnet_block0_backward_kernel(N, H, W):
    """SincNet block-0 convs (one input channel) through radhip.ops.Block0Convs vs torch autograd of the same
    bf16-rounded convolutions in fp32: dx, d conv1.weight, d conv_downsample.weight. (5, 1, 33) has more
    (utterance, 32-column strip) units than blocks (the grid-stride path); (1, 3, 2) a strip of 2 columns."""
    from radhip.ops import Block0Convs
    torch.manual_seed(3)
    x = torch.randn(N, 1, H, W, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_()
    w1 = (0.3 * torch.randn(32, 1, 2, 3, device=DEV)).requires_grad_()
    wd = (0.3 * torch.randn(32, 1, 1, 3, device=DEV)).requires_grad_()
    c, idn = Block0Convs.apply(x, w1, wd)
    assert c.shape == (N, 32, H + 1, W) and idn.shape == (N, 32, H, W)
    gc = torch.randn(c.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gi = torch.randn(idn.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    torch.autograd.backward([c, idn], [gc, gi])
    xr = x.detach().to(torch.bfloat16).float().requires_grad_()
    w1r = w1.detach().to(torch.bfloat16).float().requires_grad_()
    wdr = wd.detach().to(torch.bfloat16).float().requires_grad_()
    cr = F.conv2d(xr, w1r, None, 1, (1, 1))
    ir = F.conv2d(xr, wdr, None, 1, (0, 1))
    torch.autograd.backward([cr, ir], [gc.float(), gi.float()])
    for got, ref in ((x.grad, xr.grad), (w1.grad, w1r.grad), (wd.grad, wdr.grad)):
        assert ((got.float() - ref).norm() / ref.norm()).item() < 1e-3


@pytest.mark.parametrize("N,H,W", [(2, 23, 301), (3, 1, 34), (1, 4, 2)])
def test_sincnet_block0_front(N, H, W):
    """radhip.ops.Block0Front (rdx_sincnet_b0_fwd + conv2 on sconv.hip; backward _conv2_grad_to_c +
    rdx_sincnet_b0_bwd) vs torch fp32 of the same bf16-rounded operands: conv1 / conv_downsample of the one-channel
    input, frozen BN + SELU on the bf16 conv1 output, conv2 (2 x 3, padding (0, 1)). Outputs and the gradients of
    x, the three conv weights, conv1's bias and the BN affine."""
    from radhip.ops import Block0Front
    torch.manual_seed(4)
    x = torch.randn(N, 1, H, W, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_()
    w1 = (0.3 * torch.randn(32, 1, 2, 3, device=DEV)).requires_grad_()
    wd = (0.3 * torch.randn(32, 1, 1, 3, device=DEV)).requires_grad_()
    w2 = (0.1 * torch.randn(32, 32, 2, 3, device=DEV)).requires_grad_()
    cb = (0.1 * torch.randn(32, device=DEV)).requires_grad_()
    mean, var = 0.1 * torch.randn(32, device=DEV), torch.rand(32, device=DEV) + 0.5
    invstd = torch.rsqrt(var + 1e-5)
    gamma = (torch.rand(32, device=DEV) + 0.5).requires_grad_()
    beta = (0.1 * torch.randn(32, device=DEV)).requires_grad_()
    a, idn = Block0Front.apply(x, w1, wd, cb, mean, invstd, gamma, beta, w2)
    assert a.shape == (N, 32, H, W) and idn.shape == (N, 32, H, W)
    ga = torch.randn(a.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gi = torch.randn(idn.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    torch.autograd.backward([a, idn], [ga, gi])
    bf = lambda t: t.detach().to(torch.bfloat16).float().requires_grad_()  # noqa: E731
    xr, w1r, wdr, w2r = bf(x), bf(w1), bf(wd), bf(w2)
    cbr, gr, br = (t.detach().clone().requires_grad_() for t in (cb, gamma, beta))
    cr = F.conv2d(xr, w1r, None, 1, (1, 1))
    c16 = cr + (cr.to(torch.bfloat16).float() - cr).detach()        # the bf16-rounded conv1 output, identity grad
    o1 = F.selu(((c16 + cbr[None, :, None, None]) - mean[None, :, None, None]) * invstd[None, :, None, None]
                * gr[None, :, None, None] + br[None, :, None, None])
    ar = F.conv2d(o1.to(torch.bfloat16).float(), w2r, None, 1, (0, 1))
    ir = F.conv2d(xr, wdr, None, 1, (0, 1))
    torch.autograd.backward([ar, ir], [ga.float(), gi.float()])
    assert ((a.float() - ar).norm() / ar.norm()).item() < 1e-2
    assert ((idn.float() - ir).norm() / ir.norm()).item() < 1e-2
    for got, ref in ((x.grad, xr.grad), (w1.grad, w1r.grad), (wd.grad, wdr.grad), (w2.grad, w2r.grad),
                     (cb.grad, cbr.grad), (gamma.grad, gr.grad), (beta.grad, br.grad)):
        assert ((got.float() - ref).norm() / ref.norm()).item() < 2e-2


@pytest.mark.parametrize("C,dt_in,to_linear", [(144, torch.float32, True), (144, torch.bfloat16, True),
                                               (64, torch.bfloat16, True), (1024, torch.float32, True),
                                               (144, torch.float32, False), (36, torch.float32, False)])
def test_row_layer_norm(C, dt_in, to_linear):
    """radhip.linear.RowLayerNorm (csrc/rowln.hip) under bf16 autocast vs torch fp32 layer_norm of the same input:
    output (bf16 when it feeds a linear, else fp32), input gradient, and gamma / beta gradients both accumulated
    into existing fp32 .grad buffers and returned to autograd."""
    from radhip.linear import RowLayerNorm
    torch.manual_seed(6)
    ln = RowLayerNorm(C, to_linear=to_linear).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.rand(C) + 0.5)
        ln.bias.copy_(0.1 * torch.randn(C))
    x = (torch.randn(3, 201, C, device=DEV) * 2 + 0.3).to(dt_in).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ln(x)
    assert y.dtype == (torch.bfloat16 if to_linear else torch.float32)
    gy = torch.randn(y.shape, device=DEV).to(y.dtype)
    ln.weight.grad = torch.full_like(ln.weight, 0.5)      # accumulation on top of existing values:
    ln.bias.grad = torch.zeros_like(ln.bias) if C != 36 else None   # in place (direct) / returned to autograd
    y.backward(gy)
    xr = x.detach().float().requires_grad_()
    wr, br = ln.weight.detach().clone().requires_grad_(), ln.bias.detach().clone().requires_grad_()
    yr = F.layer_norm(xr, (C,), wr, br, ln.eps)
    yr.backward(gy.float())
    tol = 1e-2 if to_linear or dt_in == torch.bfloat16 else 1e-5
    assert ((y.float() - yr).norm() / yr.norm()).item() < tol
    assert ((x.grad.float() - xr.grad).norm() / xr.grad.norm()).item() < (2e-2 if dt_in == torch.bfloat16 else 1e-4)
    assert ((ln.weight.grad - 0.5 - wr.grad).norm() / wr.grad.norm()).item() < 1e-4
    assert ((ln.bias.grad - br.grad).norm() / br.grad.norm()).item() < 1e-4


def test_attention_rejects_non_toeplitz_bias():
    """The kernels take the bias as a relative-position table; a bias that is not a function of key - query
    is refused loudly rather than silently mis-read."""
    from radhip.ops import GatedAttention
    T, H = 40, 2
    q = torch.randn(1, T, H * 64, device=DEV).to(torch.bfloat16)
    gate = torch.rand(1, T, H, device=DEV)
    with pytest.raises(ValueError, match="Toeplitz"):
        GatedAttention.apply(q, q, q, gate, torch.randn(H, T, T, device=DEV), None, 0.0, 0)
