"""Fused frozen WavLM CNN feature encoder (csrc/featconv.hip + rdx_hgemm_batched; rdx_gemm_bf16_strided before round 6)
against the module path.

The WavLM-Large geometry (7 conv layers of 512 channels, kernels 10,3,3,3,3,2,2, strides 5,2,...,2,
LayerNorm-over-channels + GELU after every conv), with seeded weights, on full-length and ragged inputs.
Reference: the same modules run in fp32 (float64 accumulation is not needed at these sizes). The fused path
computes in bf16 exactly where the bf16-autocast module path does (waveform, weights, every layer's
activation), so the tolerance is bf16 rounding propagated through 7 normalised layers: per utterance, 2 %
relative L2 against fp32, and no more than 1.5x the error of the bf16-autocast module path it replaces."""
import numpy as np
import pytest
import torch

from seeded import seeded_array, seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _encoder(conv_bias):
    from radhip.wavlm import FeatureEncoder, WavLMConfigLite
    fe = FeatureEncoder(WavLMConfigLite(conv_bias=conv_bias))
    seeded_fill_(fe, seed=61)
    for p in fe.parameters():
        p.requires_grad = False
    return fe.to(DEV).eval()


def _rel(a, b):
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("conv_bias", [False, True])
@pytest.mark.parametrize("L,B", [(64600, 3), (30011, 2)])
def test_fused_feature_encoder_matches_modules(conv_bias, L, B, monkeypatch):
    fe = _encoder(conv_bias)
    x = torch.from_numpy(seeded_array(f"fe{L}", (B, L), scale=0.1)).float().to(DEV)
    with torch.no_grad():
        ref32 = fe(x)                                                   # fp32 module path (no autocast)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert fe._fused_ok(x)
            got = fe(x)
            monkeypatch.setenv("RADHIP_FUSED_FE", "0")
            ref16 = fe(x)                                               # bf16-autocast module path
            monkeypatch.delenv("RADHIP_FUSED_FE")
    T = (L - 10) // 5 + 1
    for _ in range(6):
        T = (T - 3) // 2 + 1 if _ < 4 else (T - 2) // 2 + 1
    assert got.shape == ref32.shape == (B, 512, T) and got.dtype == torch.float32
    for b in range(B):
        e_fused, e_mod = _rel(got[b], ref32[b]), _rel(ref16[b].float(), ref32[b])
        assert e_fused < 2e-2 and e_fused <= 1.5 * e_mod + 1e-3, (b, e_fused, e_mod)


@pytest.mark.parametrize("K,s,T,B", [(3, 2, 101, 3), (2, 2, 64, 2), (3, 2, 6459, 1)])
def test_strided_gemm_is_the_token_major_conv(K, s, T, B):
    from radhip import _lib
    from radhip._lib import check, lib
    from radhip.ops import _p, _stream
    C = 512
    x = torch.from_numpy(seeded_array(f"sg{K}{T}", (B, T, C), scale=0.5)).to(torch.bfloat16).to(DEV)
    w = torch.from_numpy(seeded_array(f"sgw{K}", (C, C, K), scale=0.05)).to(torch.bfloat16).to(DEV)
    bias = torch.from_numpy(seeded_array(f"sgb{K}", (C,), scale=0.1)).to(torch.bfloat16).to(DEV)
    To = (T - K) // s + 1
    wk = w.permute(0, 2, 1).reshape(C, K * C).contiguous()
    y = torch.empty(B, To, C, device=DEV, dtype=torch.bfloat16)
    check(lib().rdx_gemm_bf16_strided(_p(x), s * C, T * C, _p(wk), K * C, _p(y), C, To, B, To, C, K * C, _p(bias),
                                      _stream(x)), "gemm_bf16_strided")
    ref = torch.nn.functional.conv1d(x.float().transpose(1, 2), w.float(), bias.float(), stride=s).transpose(1, 2)
    np.testing.assert_allclose(y.float().cpu().numpy(), ref.cpu().numpy(), rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    assert _lib is not None


@pytest.mark.parametrize("tile", [0, 2, 4])
@pytest.mark.parametrize("K,s,T,B", [(3, 2, 101, 3), (2, 2, 64, 2), (3, 2, 6459, 2), (2, 2, 403, 5)])
def test_batched_hgemm_is_the_token_major_conv(K, s, T, B, tile):
    """rdx_hgemm_batched (csrc/hgemm.hip, blockIdx.y over the utterances, A rows overlapping at stride * C): the CNN
    layers' product since round 6 (radhip.ops.FE_HGEMM_TILE)."""
    from radhip._lib import check, lib
    from radhip.ops import _p, _stream
    C = 512
    x = torch.from_numpy(seeded_array(f"sg{K}{T}", (B, T, C), scale=0.5)).to(torch.bfloat16).to(DEV)
    w = torch.from_numpy(seeded_array(f"sgw{K}", (C, C, K), scale=0.05)).to(torch.bfloat16).to(DEV)
    bias = torch.from_numpy(seeded_array(f"sgb{K}", (C,), scale=0.1)).to(torch.bfloat16).to(DEV)
    To = (T - K) // s + 1
    wk = w.permute(0, 2, 1).reshape(C, K * C).contiguous()
    y = torch.full((B, To, C), float("nan"), device=DEV, dtype=torch.bfloat16)
    check(lib().rdx_hgemm_batched(_p(x), s * C, T * C, _p(wk), K * C, _p(y), C, To * C, To, C, K * C, B, _p(bias), tile,
                                  0, _stream(x)), "hgemm_batched")
    ref = torch.nn.functional.conv1d(x.float().transpose(1, 2), w.float(), bias.float(), stride=s).transpose(1, 2)
    np.testing.assert_allclose(y.float().cpu().numpy(), ref.cpu().numpy(), rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
