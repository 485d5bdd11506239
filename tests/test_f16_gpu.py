"""The fp16 product path: libradhip_f16.so (the same kernel sources built with -DRDX_F16, csrc/common.h) driven by
fp16 autocast, the reference's training dtype (src/main.py:28,1049 — torch.cuda.amp.autocast() + GradScaler).

Every test runs the fp16 kernel against an fp32 torch restatement AND runs the bf16 kernel on the same inputs, and
asserts two things: the fp16 result is within the tolerance the bf16 tests use, and its error is well below the bf16
error (fp16 keeps 3 more mantissa bits: ~8x finer rounding; the bound asserted is 3x, leaving room for the fp32
accumulation and the error terms that are not rounding). That second check is what shows the fp16 library really
computes in fp16: a kernel that kept bf16 anywhere on its data path would fail it.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
GAIN = 3.0          # bf16 error / fp16 error must exceed this


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _gelu(x):
    return F.gelu(x)


# --------------------------------------------------------------------------------------- GEMMs ----
GEMMS = [("wgemm", dict(tile=5)), ("wgemm", dict(tile=6)), ("wgemm", dict(tile=12, splits=4)),
         ("pgemm", dict(tile=4, group_m=4)), ("pgemm", dict(tile=5, group_m=0)), ("gemm", {}),
         ("hgemm", dict(tile=0)), ("hgemm", dict(tile=2)), ("hgemm", dict(tile=4, splits=2))]


@pytest.mark.parametrize("kind,kw", GEMMS)
@pytest.mark.parametrize("epi", ["bias", "gelu", "gelu_bwd"])
def test_f16_gemms_bias_and_gelu_epilogues(kind, kw, epi):
    from radhip import _lib, ops
    if kind == "wgemm" and kw.get("splits", 1) > 1 and epi != "bias":
        pytest.skip("split-K runs the plain epilogue only")
    torch.manual_seed(0)
    M, N, K = 1608, 1024, 1024
    a = 0.5 * torch.randn(M, K, device=DEV)
    b = torch.randn(N, K, device=DEV) / K ** 0.5
    bias = 0.1 * torch.randn(N, device=DEV)
    aux = torch.randn(M, N, device=DEV)
    fn = getattr(ops, kind)
    epilogue = {"bias": _lib.EPI_BIAS, "gelu": _lib.EPI_BIAS_GELU, "gelu_bwd": _lib.EPI_GELU_BWD}[epi]
    errs = {}
    for dt in (torch.bfloat16, torch.float16):
        ah, bh, ch, uh = a.to(dt), b.to(dt), bias.to(dt), aux.to(dt)
        out = fn(ah, bh, ch if epi != "gelu_bwd" else None, epilogue=epilogue,
                 aux=uh if epi == "gelu_bwd" else None, **kw)
        acc = ah.float() @ bh.float().t()
        if epi == "bias":
            ref, got = acc + ch.float(), out
        elif epi == "gelu":
            ref, got = _gelu(acc + ch.float()), out[1]
        else:
            u = uh.float().requires_grad_()
            g = torch.autograd.grad(_gelu(u), u, acc)[0]
            ref, got = g, out
        assert got.dtype == dt
        errs[dt] = _rel(got.float(), ref)
        # against the exact product of the unrounded fp32 operands: the storage dtype's rounding shows here
        if epi == "bias":
            errs[(dt, "exact")] = _rel(got.float(), a @ b.t() + bias)
    assert errs[torch.float16] < 2e-3 and errs[torch.bfloat16] < 1.5e-2, errs
    if epi == "bias":
        assert errs[(torch.bfloat16, "exact")] > GAIN * errs[(torch.float16, "exact")], errs


def test_f16_wgrad_acc():
    from radhip import ops
    torch.manual_seed(1)
    M, N, K = 3216, 288, 144
    dy, x = torch.randn(M, N, device=DEV), torch.randn(M, K, device=DEV)
    exact = dy.t() @ x
    errs = {}
    for dt in (torch.bfloat16, torch.float16):
        dw = torch.zeros(N, K, device=DEV)
        db = torch.zeros(N, device=DEV)
        ops.wgrad_acc(dy.to(dt), x.to(dt), dw, db)
        errs[dt] = _rel(dw, exact)
        assert _rel(dw, dy.to(dt).float().t() @ x.to(dt).float()) < 1e-5
        assert _rel(db, dy.to(dt).float().sum(0)) < 1e-5
    assert errs[torch.bfloat16] > GAIN * errs[torch.float16], errs


# ------------------------------------------------------------------------------- attention ----
@pytest.mark.parametrize("bwd", ["fused", "split"])
def test_f16_gated_attention(bwd, monkeypatch):
    from radhip.ops import GatedAttention, attention_dropout_mask
    monkeypatch.setenv("RADHIP_ATTN_BWD", bwd)
    torch.manual_seed(0)
    B, T, H = 2, 201, 16
    E = H * 64
    q0, k0, v0 = (0.5 * torch.randn(B, T, E, device=DEV) for _ in range(3))
    gate0 = 2 * torch.rand(B, T, H, device=DEV)
    g = torch.Generator(device="cpu").manual_seed(5)
    tab = torch.randn(H, 2 * T - 1, generator=g).to(DEV)
    i = torch.arange(T, device=DEV)
    pb = tab[:, i[None, :] - i[:, None] + T - 1]
    seed = torch.tensor([777], dtype=torch.int64, device=DEV)
    go0 = torch.randn(B, T, E, device=DEV)
    p = 0.1
    keep = attention_dropout_mask(seed, 3, p, (B, H, T, T)).float() / (1 - p)

    def reference(q, k, v, gate, go):
        qr, kr, vr = (t.detach().float().view(B, T, H, 64).transpose(1, 2).requires_grad_() for t in (q, k, v))
        gr = gate.detach().clone().requires_grad_()
        s = qr @ kr.transpose(-1, -2) * 0.125 + gr.permute(0, 2, 1).unsqueeze(-1) * pb.unsqueeze(0)
        o = ((torch.softmax(s, -1) * keep) @ vr).transpose(1, 2).reshape(B, T, E)
        o.backward(go.float())
        return [o.detach()] + [t.grad.transpose(1, 2).reshape(B, T, E) for t in (qr, kr, vr)] + [gr.grad]

    exact = reference(q0, k0, v0, gate0, go0)
    errs = {}
    for dt in (torch.bfloat16, torch.float16):
        q, k, v = (t.to(dt).requires_grad_() for t in (q0, k0, v0))
        gate = gate0.clone().requires_grad_()
        o = GatedAttention.apply(q, k, v, gate, pb, seed, p, 3)
        go = go0.to(dt)
        o.backward(go)
        assert o.dtype == dt
        got = [o, q.grad, k.grad, v.grad, gate.grad]
        same = reference(q, k, v, gate, go)           # fp32 on the same rounded inputs
        tol = [1e-2, 2e-2, 2e-2, 2e-2, 2e-2] if dt == torch.bfloat16 else [3e-3, 5e-3, 5e-3, 5e-3, 5e-3]
        for x, r, t in zip(got, same, tol):
            assert _rel(x.float(), r) < t, (dt, _rel(x.float(), r))
        errs[dt] = [_rel(x.float(), r) for x, r in zip(got, exact)]
    for e16, e8 in zip(errs[torch.float16], errs[torch.bfloat16]):
        assert e8 > GAIN * e16, errs


# -------------------------------------------------------------------------------- posconv ----
def test_f16_posconv():
    from radhip.ops import PosConv, posconv_weights
    torch.manual_seed(0)
    w = torch.randn(1024, 64, 128, device=DEV) * 0.01
    bias = torch.randn(1024, device=DEV) * 0.1
    B, T = 2, 201
    h0 = torch.randn(B, T, 1024, device=DEV)
    go0 = torch.randn(B, T, 1024, device=DEV)

    def reference(h, wr, go):
        hr = h.detach().float().requires_grad_()
        yr = F.gelu(F.conv1d(hr.transpose(1, 2), wr, bias, padding=64, groups=16)[:, :, :-1]).transpose(1, 2)
        yr.backward(go.float())
        return yr.detach(), hr.grad

    exact = reference(h0, w, go0)
    errs = {}
    for dt in (torch.bfloat16, torch.float16):
        wk, wkt = posconv_weights(w, dt)
        h = h0.to(dt).requires_grad_()
        y = PosConv.apply(h, wk, wkt, bias)
        y.backward(go0.to(dt))
        assert y.dtype == dt and h.grad.dtype == dt
        yr, gr = reference(h, w.to(dt).float(), go0.to(dt))
        t = (1e-2, 2e-2) if dt == torch.bfloat16 else (2e-3, 4e-3)
        assert _rel(y.float(), yr) < t[0] and _rel(h.grad.float(), gr) < t[1], dt
        errs[dt] = (_rel(y.float(), exact[0]), _rel(h.grad.float(), exact[1]))
    assert all(a > GAIN * b for a, b in zip(errs[torch.bfloat16], errs[torch.float16])), errs


# ------------------------------------------------------------------- fused WavLM layers ----
@pytest.mark.parametrize("B,inter", [(2, 512), (8, 4096)])
def test_f16_fused_wavlm_layers(B, inter):
    """Two fused layers (LN1 + gate + LoRA-A, the q/k/v, out_proj and FFN GEMMs, gated attention, dropout +
    residual + LN2, GELU and every backward) under fp16 autocast against the fp32 restatement with the kernels'
    own dropout masks (tests/test_wavlm_fused_gpu.py), next to the same run under bf16 autocast."""
    from radhip import wavlm_fused
    from test_wavlm_fused_gpu import _encoder, _lora_params, _ref_layer
    T, E, p = 201, 1024, 0.1
    enc = _encoder(p=p, inter=inter).train()
    torch.manual_seed(1)
    h00 = 0.5 * torch.randn(B, T, E, device=DEV)
    gout = torch.randn(B, T, E, device=DEV)
    seed = torch.tensor([12345], dtype=torch.int64, device=DEV)
    runner = wavlm_fused.FusedEncoderRunner(enc)
    res = {}
    for dt in (torch.bfloat16, torch.float16):
        h0 = h00.clone().requires_grad_(True)
        for prm in _lora_params(enc):
            prm.grad = None
        with torch.autocast("cuda", dtype=dt):
            assert wavlm_fused.eligible(enc, h0)
            loras = runner.prepare(h0.device)
            assert runner.caches[0].wext.dtype == dt
            pb = runner.position_bias(T, h0.device)
            h = h0
            for i in range(len(enc.layers)):
                h = runner.layer(i, h, pb, loras, seed)
        (h * gout).sum().backward()
        res[dt] = [h.detach(), h0.grad.clone()] + [prm.grad.clone() for prm in _lora_params(enc)]
    h0 = h00.clone().requires_grad_(True)
    for prm in _lora_params(enc):
        prm.grad = None
    ii = torch.arange(T, device=DEV)
    pb_full = pb[:, ii[None, :] - ii[:, None] + T - 1]
    hr = h0
    for i, layer in enumerate(enc.layers):
        hr = _ref_layer(layer, i, hr, pb_full, seed, p)
    (hr * gout).sum().backward()
    ref = [hr.detach(), h0.grad] + [prm.grad for prm in _lora_params(enc)]
    e16 = [_rel(a, b) for a, b in zip(res[torch.float16], ref)]
    e8 = [_rel(a, b) for a, b in zip(res[torch.bfloat16], ref)]
    assert max(e16) < 1e-2, e16
    for a, b in zip(e8, e16):
        assert a > GAIN * b, (e8, e16)


# ------------------------------------------------------------------- fused CNN feature encoder ----
def test_f16_fused_feature_encoder(monkeypatch):
    from seeded import seeded_array
    from test_featconv_gpu import _encoder as fe_encoder
    fe = fe_encoder(False)
    x = torch.from_numpy(seeded_array("fe16", (2, 64600), scale=0.1)).float().to(DEV)
    with torch.no_grad():
        ref32 = fe(x)
        errs = {}
        for dt in (torch.bfloat16, torch.float16):
            with torch.autocast("cuda", dtype=dt):
                assert fe._fused_ok(x)
                got = fe(x)
                monkeypatch.setenv("RADHIP_FUSED_FE", "0")
                mod = fe(x)                                         # torch's module path under the same autocast
                monkeypatch.delenv("RADHIP_FUSED_FE")
            errs[dt] = (_rel(got, ref32), _rel(mod.float(), ref32))
    e16, m16 = errs[torch.float16]
    assert e16 <= 1.5 * m16 + 1e-4, errs
    assert errs[torch.bfloat16][0] > GAIN * e16, errs


# ------------------------------------------------------------------------ SincNet block 0 ----
def test_f16_sincnet_block0_fused_vs_fp32():
    """Block 0 in one pass each way (csrc/b0fused.hip) under fp16 autocast against the fp32 torch graph of the
    module (frozen BN): forward and every gradient, bf16 alongside."""
    from test_b0x_gpu import _block, _x
    blk = _block(11)
    x = _x(2, 23, 3001, seed=5)
    g = torch.Generator(device="cpu").manual_seed(7)

    def run(dt, fused):
        for p_ in blk.parameters():
            p_.grad = None
        xx = x.detach().clone().requires_grad_(True)
        if fused:
            with torch.autocast("cuda", dtype=dt):
                y = blk(xx)
        else:
            blk._fused_ok = lambda _x: False                # the module's torch graph, fp32
            try:
                y = blk(xx)
            finally:
                del blk._fused_ok
        dy = torch.randn(y.shape, generator=g.manual_seed(7)).to(DEV).contiguous(memory_format=torch.channels_last)
        y.backward(dy.to(y.dtype))
        out = {"y": y.detach().float(), "dx": xx.grad.detach().float()}
        out.update({n: p_.grad.detach().float().clone() for n, p_ in blk.named_parameters() if p_.grad is not None})
        return out
    ref = run(None, False)
    r16, r8 = run(torch.float16, True), run(torch.bfloat16, True)
    assert r16.keys() == ref.keys()
    e16 = {k: _rel(r16[k], ref[k]) for k in ref}
    e8 = {k: _rel(r8[k], ref[k]) for k in ref}
    assert e16["y"] < 2e-3 and max(e16.values()) < 5e-2, e16
    assert e8["y"] > GAIN * e16["y"], (e8, e16)


# ------------------------------------------------------------------------------ multi-tensor cast ----
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_cast_many_equals_to(dt):
    """rdx_cast_f32_many (the window's per-window weight cast) == tensor.to(dt) bit for bit, over more than one
    64-tensor launch and ragged sizes (including an empty tensor)."""
    from radhip import ops
    torch.manual_seed(0)
    srcs = [torch.randn(n, device=DEV) * 10 ** (k % 5 - 2) for k, n in enumerate([0, 1, 7, 255, 256, 257, 83000] * 10)]
    dsts = [torch.empty_like(s, dtype=dt) for s in srcs]
    ops.cast_many(srcs, dsts)
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.to(dt))
