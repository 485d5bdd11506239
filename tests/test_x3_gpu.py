"""The split-precision ("x3") scoring path (radhip/wavlm_x3.py, csrc/hgemm.hip rdx_hgemm_x3, csrc/x3.hip): the fp32
eval forward of the reference (src/main.py:958-995, no autocast) with its WavLM-Large stream on hand-written kernels.

Each kernel against an fp64 torch restatement of the same math, then the whole Phase-6 model through
radhip.infer._scores(amp="x3") against the fp64 oracle (oracle/model.py: transformers' WavLM + the restated
reference modules) within the north-star 1e-3 on the logits.

Bounds: an fp32 value is carried as bf16 hi + lo (|x - hi - lo| <= 2^-17 |x|) and a product drops lo.lo (<= 2^-16),
so a GEMM element is within a few 1e-5 of sum |a||b|; the asserted 5e-5 (relative to sum |a||b|) leaves room for the
fp32 accumulation at K = 12288 while any wrong tile, plane or pass (O(1) errors) fails it. The fp32 attention /
LayerNorm / conv kernels are held to 1e-5 relative to the output scale (fp32 rounding plus the planes of their
inputs)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
PROFILES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")


def _planes(t):
    from radhip.wavlm_x3 import planes
    return planes(t)


def _gemm_err(c, a64, b64, ref):
    scale = a64.abs() @ b64.abs().t()
    return float(((c.double() - ref).abs() / scale.clamp_min(1e-30)).max())


@pytest.mark.parametrize("M,N,K,pol", [(6432, 3072, 1024, "qkv"), (6432, 1024, 1024, "out"), (1608, 4096, 1024, "ffn1"),
                                       (6432, 1024, 4096, "ffn2"), (333, 260, 192, "proj"), (1, 4, 64, "out")])
def test_hgemm_x3_f32_matches_fp64(M, N, K, pol):
    from radhip import wavlm_x3
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g, dtype=torch.float64)
    w = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    bias = 0.1 * torch.randn(N, generator=g, dtype=torch.float64)
    ah, al = _planes(a.float().to(DEV))
    wp = _planes(w.float().to(DEV))
    got = wavlm_x3.gemm(ah, al, wp, bias.float().to(DEV).contiguous(), pol=pol)
    a64, w64 = a.float().double().to(DEV), w.float().double().to(DEV)       # the fp32 operands the planes carry
    ref = a64 @ w64.t() + bias.float().double().to(DEV)
    err = _gemm_err(got, a64, w64, ref)
    err32 = _gemm_err(a64.float() @ w64.float().t() + bias.float().to(DEV), a64, w64, ref)
    print(f"[x3 gemm {M}x{N}x{K}] max err / sum|a||b| {err:.2e} (torch fp32 GEMM {err32:.2e})")
    assert got.dtype == torch.float32 and got.shape == (M, N)
    assert err < 5e-5


def test_hgemm_x3_splitk_matches_unsplit():
    """Split-K 3 (the passes cut across splits) sums to the unsplit result up to fp32 reassociation."""
    from radhip import wavlm_x3
    g = torch.Generator(device="cpu").manual_seed(3)
    a = torch.randn(1608, 1024, generator=g).to(DEV)
    w = (torch.randn(1024, 1024, generator=g) / 32).to(DEV)
    ah, al = _planes(a)
    wp = _planes(w)
    one = wavlm_x3.gemm(ah, al, wp, None, pol="out")
    old = wavlm_x3.X3_POLICY["out"]
    try:
        wavlm_x3.X3_POLICY["out"] = (4, 3, 4)
        three = wavlm_x3.gemm(ah, al, wp, None, pol="out")
    finally:
        wavlm_x3.X3_POLICY["out"] = old
    assert float((one - three).abs().max()) <= 1e-5 * float(one.abs().max())


def test_hgemm_x3_gelu_split_epilogue():
    """EPI_F32_GELU_SPLIT: the planes of gelu(acc + bias) (FFN1 feeding FFN2)."""
    from radhip import _lib, wavlm_x3
    g = torch.Generator(device="cpu").manual_seed(5)
    a = torch.randn(1000, 1024, generator=g).to(DEV)
    w = (torch.randn(4096, 1024, generator=g) / 32).to(DEV)
    bias = (0.1 * torch.randn(4096, generator=g)).to(DEV)
    ah, al = _planes(a)
    wp = _planes(w)
    vh, vl = wavlm_x3.gemm(ah, al, wp, bias, epilogue=_lib.EPI_F32_GELU_SPLIT, pol="ffn1")
    assert vh.dtype == torch.bfloat16 and vl.dtype == torch.bfloat16
    ref = torch.nn.functional.gelu(a.double() @ w.double().t() + bias.double())
    got = vh.double() + vl.double()
    assert float((got - ref).abs().max()) < 5e-5 * float(ref.abs().max())
    # lo really is the residual of hi (not a second copy)
    assert float((vh.double() - ref).abs().max()) > 10 * float((got - ref).abs().max())


def test_hgemm_x3_batched_strided_conv():
    """The WavLM CNN's layers 1-6 as one batched launch: A rows overlapping at stride * C (lda < K), per-utterance
    A and C strides, against conv1d in fp64."""
    from radhip import wavlm_x3
    g = torch.Generator(device="cpu").manual_seed(7)
    B, T, C, k, s = 3, 517, 512, 3, 2
    x = torch.randn(B, T, C, generator=g).to(DEV)
    w = (torch.randn(C, C, k, generator=g) / (C * k) ** 0.5).to(DEV)
    To = (T - k) // s + 1
    xh, xl = _planes(x)
    wp = _planes(w.permute(0, 2, 1).reshape(C, k * C))
    y = torch.empty(B, To, C, device=DEV)
    wavlm_x3.gemm(xh, xl, wp, None, out=y, M=To, lda=s * C, sa=T * C, batch=B, sc=To * C, K=k * C, pol="cnn")
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.double(), stride=s).transpose(1, 2)
    assert float((y.double() - ref).abs().max()) < 5e-5 * float(ref.abs().max())


def test_x3_ln_split_and_gate():
    from radhip.wavlm_x3 import _ln
    g = torch.Generator(device="cpu").manual_seed(9)
    M, E, H = 403, 1024, 16
    a = torch.randn(M, E, generator=g).to(DEV)
    b = torch.randn(M, E, generator=g).to(DEV)
    gm = (1 + 0.1 * torch.randn(E, generator=g)).to(DEV)
    bt = (0.1 * torch.randn(E, generator=g)).to(DEV)
    wg = (0.2 * torch.randn(8, 64, generator=g)).to(DEV)
    bg = (0.1 * torch.randn(8, generator=g)).to(DEV)
    gc = (1 + 0.1 * torch.randn(H, generator=g)).to(DEV)
    s = torch.empty(M, E, device=DEV)
    gate = torch.empty(M, H, device=DEV)
    hi, lo = _ln(a, (gm, bt, 1e-5), b=b, sum_out=s, gate=(wg, bg, gc), gate_out=gate)
    x = a.double() + b.double()
    assert torch.equal(s, a + b)
    y = torch.nn.functional.layer_norm(x, (E,), gm.double(), bt.double(), 1e-5)
    assert float((hi.double() + lo.double() - y).abs().max()) < 1e-5 * float(y.abs().max())
    z = (y.view(M, H, 64) @ wg.double().t() + bg.double()).view(M, H, 2, 4).sum(-1).sigmoid()
    ref_gate = z[..., 0] * (z[..., 1] * gc.double() - 1.0) + 2.0
    assert float((gate.double() - ref_gate).abs().max()) < 1e-5
    # E = 512 (feature_projection's LayerNorm) into fp32
    a5 = a[:, :512].contiguous()
    y32 = torch.empty(M, 512, device=DEV)
    _ln(a5, (gm[:512].contiguous(), bt[:512].contiguous(), 1e-5), out_planes=False, y32=y32)
    ref5 = torch.nn.functional.layer_norm(a5.double(), (512,), gm[:512].double(), bt[:512].double(), 1e-5)
    assert float((y32.double() - ref5).abs().max()) < 1e-5 * float(ref5.abs().max())


@pytest.mark.parametrize("B,T,qsplit", [(2, 201, 1), (3, 201, 2), (2, 33, 1), (1, 256, 2), (2, 100, 3)])
def test_x3_attention_matches_fp64(B, T, qsplit):
    from radhip import _lib
    from radhip.ops import _p
    from radhip.wavlm_x3 import lib
    H, E = 16, 1024
    g = torch.Generator(device="cpu").manual_seed(T + B)
    qkv = torch.randn(B * T, 3 * E, generator=g).to(DEV)
    gate = (1 + 0.5 * torch.rand(B * T, H, generator=g)).to(DEV)
    rel = torch.randn(H, 2 * T - 1, generator=g).to(DEV)
    oh = torch.empty(B * T, E, device=DEV, dtype=torch.bfloat16)
    ol = torch.empty_like(oh)
    _lib.check(lib().rdx_x3_attn_fwd(_p(qkv), _p(qkv[:, E:]), _p(qkv[:, 2 * E:]), 3 * E, _p(gate), _p(rel), 0.125,
                                     _p(oh), _p(ol), E, B, T, H, qsplit, None), "x3_attn")
    torch.cuda.synchronize()
    q, k, v = qkv.double().view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    i = torch.arange(T, device=DEV)
    bias = rel.double()[:, (i[None, :] - i[:, None] + T - 1)]                       # [H, T(i), T(j)]
    gb = gate.double().view(B, T, H).permute(0, 2, 1)[..., None] * bias[None]       # [B, H, T, T]
    p = torch.softmax(0.125 * q @ k.transpose(-1, -2) + gb, dim=-1)
    ref = (p @ v).permute(0, 2, 1, 3).reshape(B * T, E)
    got = oh.double() + ol.double()
    assert float((got - ref).abs().max()) < 1e-5 * float(ref.abs().max())


def test_x3_posconv_matches_fp64():
    from radhip.ops import _p
    from radhip.wavlm_x3 import lib
    from radhip import _lib
    g = torch.Generator(device="cpu").manual_seed(13)
    B, T = 3, 201
    h = torch.randn(B, T, 1024, generator=g).to(DEV)
    W = (torch.randn(1024, 64, 128, generator=g) / (64 * 128) ** 0.5).to(DEV)
    bias = (0.1 * torch.randn(1024, generator=g)).to(DEV)
    wk = W.reshape(16, 64, 64, 128).permute(0, 3, 1, 2).contiguous()
    wh, wl = _planes(wk)
    out = torch.empty_like(h)
    _lib.check(lib().rdx_x3_posconv_fwd(_p(h), _p(wh), _p(wl), _p(bias), _p(out), B, T, None), "x3_posconv")
    torch.cuda.synchronize()
    y = torch.nn.functional.conv1d(h.double().transpose(1, 2), W.double(), bias.double(), padding=64, groups=16)
    ref = h.double() + torch.nn.functional.gelu(y[..., :T].transpose(1, 2))
    assert float((out.double() - ref).abs().max()) < 2e-5 * float(ref.abs().max())


def test_x3_feature_encoder_matches_fp64():
    """The whole frozen CNN (conv0 direct + 6 batched strided x3 GEMMs, LayerNorm + GELU in fp32) against the
    module path in fp64."""
    from radhip.wavlm import FeatureEncoder, WavLMConfigLite
    from radhip.wavlm_x3 import X3Weights, feature_encoder
    torch.manual_seed(0)
    cfg = WavLMConfigLite()
    fe = FeatureEncoder(cfg).to(DEV).eval()
    for p in fe.parameters():
        p.requires_grad_(False)
    x = (0.1 * torch.randn(2, 64600)).clamp(-1, 1).to(DEV)

    W = X3Weights.__new__(X3Weights)      # only the CNN's parts
    f = lambda t: t.detach().float().contiguous() if t is not None else None   # noqa: E731
    from radhip.wavlm_x3 import planes
    c0 = fe.conv_layers[0]
    W.fe0 = (f(c0.conv.weight.reshape(512, -1)), f(c0.conv.bias), f(c0.layer_norm.weight), f(c0.layer_norm.bias),
             float(c0.layer_norm.eps), 10, 5)
    W.fe = [(planes(ly.conv.weight.detach().float().permute(0, 2, 1).reshape(512, -1)), f(ly.conv.bias),
             f(ly.layer_norm.weight), f(ly.layer_norm.bias), float(ly.layer_norm.eps), ly.conv.kernel_size[0],
             ly.conv.stride[0]) for ly in fe.conv_layers[1:]]
    with torch.no_grad():
        got = feature_encoder(W, x)
        ref = fe.double()(x.double()).transpose(1, 2)
    assert got.shape == ref.shape == (2, 201, 512)
    err = float((got.double() - ref).abs().max())
    print(f"[x3 CNN] max abs err {err:.3e} (|ref| max {float(ref.abs().max()):.3f})")
    assert err < 1e-4 * float(ref.abs().max())


# ------------------------------------------------------------------------------------------ whole model ----------
def _model_and_oracle(lora_mode):
    from oracle.model import OracleModel, apply_lora, from_peft_state
    from radhip.build import apply_lora_to_wavlm, get_model, load_config
    from radhip.wavlm import WAVLM_LARGE
    cfg = load_config("Phase6_Proposed.conf")
    cfg["training_config"]["lora_mode"] = lora_mode
    w = dict(WAVLM_LARGE)
    cfg["model_config"] = dict(cfg["model_config"], wavlm_config=w)
    torch.manual_seed(1234)
    m = apply_lora_to_wavlm(get_model(cfg["model_config"], DEV), cfg["training_config"])
    with torch.no_grad():           # peft initialises lora_B to zero: give the adapters a part to play
        for n, p in m.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.02)
    m.eval()
    ocfg = dict(w)
    ocfg["conv_dim"] = tuple(ocfg["conv_dim"])
    o = OracleModel(ocfg, emb_size=144, num_encoders=4)
    apply_lora(o, merged=(lora_mode == "active"))
    o.load_state_dict(from_peft_state({k: v.detach().cpu() for k, v in m.state_dict().items()}), strict=True)
    return m, o.double().to(DEV).eval()


@pytest.mark.parametrize("lora_mode", ["reference", "active"])
def test_x3_scores_full_model_vs_fp64_oracle(lora_mode):
    """north star: per-utterance logits within 1e-3 of the reference's fp32 path, here of its fp64 restatement,
    with the full WavLM-Large Phase-6 model on the x3 path (configs 3 / 5 score at batch 32). Also: the x3 stream
    really ran (its weight planes exist), and the same bound with the classifier scaled 40x (|logits| ~ 10, the range
    of a trained detector: the x3 error grows with the logit scale, the bound does not)."""
    from radhip.infer import _scores
    m, o = _model_and_oracle(lora_mode)
    rng = np.random.default_rng(21)
    B = 8
    x = torch.from_numpy(np.clip(0.1 * rng.standard_normal((B, 64600)), -1, 1).astype(np.float32)).to(DEV)
    res = {}
    for scale in (1.0, 40.0):
        with torch.no_grad():
            if scale != 1.0:
                m.classifier.weight.mul_(scale)
                o.classifier.weight.mul_(scale)
                m.classifier.bias.mul_(scale)
                o.classifier.bias.mul_(scale)
            _, lo = o(x.double())
            s_x3 = _scores(m, x, None, "x3").double()
            s_32 = _scores(m, x, None, None).double()
        assert "_x3w" in m.wavlm_stream._core().__dict__, "the x3 stream did not run"
        ref = lo[:, 1]
        e3 = float((s_x3 - ref).abs().max())
        e32 = float((s_32 - ref).abs().max())
        res[f"scale{scale:g}"] = {"logit1_absmax": float(ref.abs().max()), "x3_max_abs_err": e3,
                                  "fp32_max_abs_err": e32}
        print(f"[x3 {lora_mode} head x{scale:g}] |logit| max {float(ref.abs().max()):.4f}: x3 max abs err {e3:.3e}, "
              f"fp32 (torch SDPA + hipBLASLt) {e32:.3e}")
        assert e3 < 1e-3, (e3, scale)
    os.makedirs(PROFILES, exist_ok=True)
    with open(os.path.join(PROFILES, f"r06_x3_logit_errors_{lora_mode}.json"), "w") as f:
        json.dump(res, f, indent=1)
