"""Fused WavLM layer (radhip/wavlm_fused.py, csrc/wavlm_layer.hip) against an fp32 torch restatement
of the same layer (HF WavLMEncoderLayerStableLayerNorm + peft LoRA q/v), with every dropout mask
regenerated from the kernels' counter hash (rdx_attn_dropout_mask), forward and backward.
Tolerance: bf16 operands with fp32 accumulation vs fp32 -> 3e-2 relative (max-norm) on outputs and
gradients; with all dropouts off the fused encoder must also match the module path (the one the
fp32 oracle tests pin) to the same tolerance."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _encoder(n_layers=2, inter=512, p=0.1, seed=0):
    from radhip.wavlm import Encoder, WavLMConfigLite, inject_lora
    torch.manual_seed(seed)
    cfg = WavLMConfigLite(num_hidden_layers=n_layers, intermediate_size=inter, hidden_dropout=p,
                          attention_dropout=p, layerdrop=0.0, num_conv_pos_embeddings=16)
    enc = Encoder(cfg).to(DEV)
    with torch.no_grad():
        for n, prm in enc.named_parameters():
            if "layer_norm" in n:
                prm.copy_((1.0 if n.endswith("weight") else 0.0) + 0.1 * torch.randn_like(prm))
            elif "gru_rel_pos_const" in n:
                prm.copy_(1.0 + 0.3 * torch.rand_like(prm))
            else:
                prm.copy_(torch.randn_like(prm) * (0.5 / math.sqrt(prm.shape[-1]) if prm.ndim > 1 else 0.05))
    for prm in enc.parameters():
        prm.requires_grad_(False)
    wrapped, n = inject_lora(enc, r=8, alpha=32, dropout=p)
    assert n == 2 * n_layers
    with torch.no_grad():
        for layer in enc.layers:
            for ad in (layer.attention.q_proj, layer.attention.v_proj):
                ad.lora_B["default"].weight.normal_(0, 0.05)
    return enc


def _mask(seed, salt, p, shape):
    """Scaled keep mask: attention scores [B, H, T, T] use the attention kernels' paired hash, the
    layer's [M, E] hidden / LoRA dropouts the element-wise hash."""
    from radhip.ops import attention_dropout_mask, dropout_mask
    if p == 0:
        return torch.ones(shape, device=DEV)
    fn = attention_dropout_mask if len(shape) == 4 else dropout_mask
    return fn(seed, salt, p, shape).float() / (1 - p)


def _ref_layer(layer, i, h, pb, seed, p):
    """fp32 restatement with the fused path's masks (salts: attention i, hidden 4096+8i+{1,2},
    LoRA 4096+8i+{3,4})."""
    B, T, E = h.shape
    H = E // 64
    M = B * T
    a = layer.attention
    s = 4096 + 8 * i
    x1 = F.layer_norm(h, (E,), layer.layer_norm.weight, layer.layer_norm.bias, layer.layer_norm.eps)
    g = F.linear(x1.view(B, T, H, 64), a.gru_rel_pos_linear.weight, a.gru_rel_pos_linear.bias)
    g = torch.sigmoid(g.view(B, T, H, 2, 4).sum(-1))
    gate = g[..., 0] * (g[..., 1] * a.gru_rel_pos_const.view(1, 1, H) - 1.0) + 2.0
    q, v = a.q_proj, a.v_proj
    mq = _mask(seed, s + 3, p, (M, E)).view(B, T, E)
    mv = _mask(seed, s + 4, p, (M, E)).view(B, T, E)
    qq = F.linear(x1, q.base_layer.weight, q.base_layer.bias) + q.scaling["default"] * F.linear(
        F.linear(x1 * mq, q.lora_A["default"].weight), q.lora_B["default"].weight)
    kk = F.linear(x1, a.k_proj.weight, a.k_proj.bias)
    vv = F.linear(x1, v.base_layer.weight, v.base_layer.bias) + v.scaling["default"] * F.linear(
        F.linear(x1 * mv, v.lora_A["default"].weight), v.lora_B["default"].weight)
    qh, kh, vh = (t.view(B, T, H, 64).transpose(1, 2) for t in (qq, kk, vv))
    S = qh @ kh.transpose(-1, -2) / 8.0 + gate.permute(0, 2, 1).unsqueeze(-1) * pb.unsqueeze(0)
    P = torch.softmax(S, -1) * _mask(seed, i, p, (B, H, T, T))
    o = (P @ vh).transpose(1, 2).reshape(B, T, E)
    h2 = h + F.linear(o, a.out_proj.weight, a.out_proj.bias) * _mask(seed, s + 1, p, (M, E)).view(B, T, E)
    ff = layer.feed_forward
    x2 = F.layer_norm(h2, (E,), layer.final_layer_norm.weight, layer.final_layer_norm.bias, layer.final_layer_norm.eps)
    f = F.linear(F.gelu(F.linear(x2, ff.intermediate_dense.weight, ff.intermediate_dense.bias)),
                 ff.output_dense.weight, ff.output_dense.bias)
    return h2 + f * _mask(seed, s + 2, p, (M, E)).view(B, T, E)


def _lora_params(enc):
    out = []
    for layer in enc.layers:
        for ad in (layer.attention.q_proj, layer.attention.v_proj):
            out += [ad.lora_A["default"].weight, ad.lora_B["default"].weight]
    return out


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("p,B,inter", [(0.0, 2, 512), (0.1, 2, 512), (0.1, 21, 512), (0.1, 8, 4096),
                                       (0.1, 32, 4096)])
def test_fused_layers_match_fp32_restatement(p, B, inter):
    """B = 21 (M = 4221 rows) takes the LoRA weight-grad kernel's multi-chunk path (2 chunks of 32
    rows per block, ragged last block); B = 2 the single-chunk path with a ragged last chunk.
    inter = 4096 is WavLM-Large's FFN width: B = 8 is the adversarial pass and B = 32 the batched
    clean pass the bench times."""
    from radhip import wavlm_fused
    enc = _encoder(p=p, inter=inter).train()
    T, E = 201, 1024
    torch.manual_seed(1)
    h0 = (0.5 * torch.randn(B, T, E, device=DEV)).requires_grad_(True)
    seed = torch.tensor([12345], dtype=torch.int64, device=DEV)
    runner = wavlm_fused.FusedEncoderRunner(enc)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert wavlm_fused.eligible(enc, h0)
        loras = runner.prepare(h0.device)
        pb = runner.position_bias(T, h0.device)
        h = h0
        for i in range(len(enc.layers)):
            h = runner.layer(i, h, pb, loras, seed)
    gout = torch.randn_like(h)
    (h * gout).sum().backward()
    got_h, got_g = h.detach(), h0.grad.clone()
    got_p = [prm.grad.clone() for prm in _lora_params(enc)]
    h0.grad = None
    for prm in _lora_params(enc):
        prm.grad = None
    # fp32 restatement with the same masks
    hr = h0
    ii = torch.arange(T, device=DEV)
    pb_full = pb[:, ii[None, :] - ii[:, None] + T - 1]          # relative-position table -> [H, T, T]
    for i, layer in enumerate(enc.layers):
        hr = _ref_layer(layer, i, hr, pb_full, seed, p)
    (hr * gout).sum().backward()
    assert _rel(got_h, hr.detach()) < 3e-2
    assert _rel(got_g, h0.grad) < 3e-2
    for gp, prm in zip(got_p, _lora_params(enc)):
        assert _rel(gp, prm.grad) < 5e-2, prm.shape


@pytest.mark.parametrize("B,inter", [(2, 512), (8, 4096)])
def test_fused_encoder_matches_module_path_without_dropout(monkeypatch, B, inter):
    """Encoder.forward with the fused layers (bf16) vs the module path in fp32 (dropouts off); the
    module path is the one pinned to HF WavLM by the model golden. inter 4096 = WavLM-Large width."""
    enc = _encoder(n_layers=3, p=0.0, inter=inter).train()
    torch.manual_seed(2)
    x = (0.5 * torch.randn(B, 201, 1024, device=DEV))
    outs, grads = [], []
    for fused in (True, False):
        monkeypatch.setenv("RADHIP_FUSED_WAVLM", "1" if fused else "0")
        enc.__dict__.pop("_fused_ok", None)
        for prm in _lora_params(enc):
            prm.grad = None
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=fused):
            last, states = enc(xi)
        loss = sum((s.float() * (k + 1)).mean() for k, s in enumerate(states))
        loss.backward()
        outs.append([s.detach().float() for s in states])
        grads.append([xi.grad.clone()] + [prm.grad.clone() for prm in _lora_params(enc)])
    for a, b in zip(outs[0], outs[1]):
        assert _rel(a, b) < 3e-2
    for a, b in zip(grads[0], grads[1]):
        assert _rel(a, b) < 5e-2


def test_fused_layer_eval_needs_no_seed():
    """Eval (no dropout) runs the fused layers without a seed and is deterministic."""
    from radhip import wavlm_fused
    enc = _encoder(p=0.1).eval()
    x = torch.randn(2, 201, 1024, device=DEV)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        a, _ = enc(x)
        b, _ = enc(x)
    assert torch.equal(a, b) and torch.isfinite(a).all()
    assert wavlm_fused.enabled()
