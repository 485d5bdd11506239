"""What LoRA computes in the reference (src/main.py:103-158 on transformers' WavLM), on CPU.

The reference wraps q_proj / v_proj of `WavLMModel` in peft LoRA layers. transformers' WavLMAttention never
calls those layers: it passes `q_proj.weight` (and the concatenated q/k/v biases) to
F.multi_head_attention_forward, and a peft layer's `weight` / `bias` are its base layer's (peft's
BaseTunerLayer properties; older peft layers subclass nn.Linear). peft is not installed here, so its layer is
restated (oracle/model.py::OLoraLinear, parity of peft itself unpinned); transformers' WavLM is the installed
one. With non-zero adapters the outputs stay the base model's and the adapters get no gradient, which is what
the product's default lora_mode "reference" reproduces (radhip.wavlm.LoraLinear active=False; radhip.train
leaves such weights out of the gradient buffer, as AdamW skips parameters without .grad)."""
import json

import numpy as np
import torch


def _tiny_hf(golden):
    from transformers import WavLMConfig, WavLMModel
    g = golden("model_tiny.npz")
    cfg = json.loads(str(g["wavlm_config"]))
    cfg["conv_dim"] = tuple(cfg["conv_dim"])
    cfg.update(hidden_dropout=0.0, attention_dropout=0.0, feat_proj_dropout=0.0, activation_dropout=0.0,
               layerdrop=0.0, mask_time_prob=0.0)
    torch.manual_seed(0)
    return WavLMModel(WavLMConfig(**cfg)).double().eval()


def _wrap(model, merged):
    from oracle.model import OLoraLinear
    for layer in model.encoder.layers:
        for t in ("q_proj", "v_proj"):
            lin = OLoraLinear(getattr(layer.attention, t), 8, 32, merged=merged).double()
            with torch.no_grad():
                lin.lora_B["default"].weight.normal_(0, 0.5)
            setattr(layer.attention, t, lin)
    return model


def test_peft_lora_on_hf_wavlm_is_bypassed(golden):
    x = torch.from_numpy(np.random.default_rng(0).standard_normal((2, 16000))).double()
    m = _tiny_hf(golden)
    with torch.no_grad():
        base = m(x).last_hidden_state
    _wrap(m, merged=False)
    for p in m.parameters():
        p.requires_grad_(False)
    lora = [p for n, p in m.named_parameters() if "lora_" in n]
    assert lora
    for p in lora:
        p.requires_grad_(True)
    out = m(x).last_hidden_state
    # equal to fp64 rounding (the grad-mode forward takes another MHA code path); an applied adapter with
    # B ~ N(0, 0.5) would move the outputs by O(1)
    torch.testing.assert_close(out, base, rtol=0, atol=1e-12)
    assert not out.requires_grad                                  # nothing trainable is in the graph


def test_merged_lora_changes_output_and_trains(golden):
    """The oracle of lora_mode "active": merging s * B A into q/v makes the adapters count."""
    x = torch.from_numpy(np.random.default_rng(0).standard_normal((2, 16000))).double()
    m = _tiny_hf(golden)
    with torch.no_grad():
        base = m(x).last_hidden_state
    _wrap(m, merged=True)
    for n, p in m.named_parameters():
        p.requires_grad_("lora_" in n)
    out = m(x).last_hidden_state
    assert float((out - base).abs().max()) > 1e-3
    out.square().mean().backward()
    assert all(p.grad is not None and float(p.grad.abs().max()) > 0 for n, p in m.named_parameters() if "lora_B" in n)


def test_product_reference_mode_leaves_adapters_out_of_the_step():
    """lora_mode "reference": the product's adapters are bypassed in the forward and left out of the flat
    gradient buffer and the clip / step (so weight decay never touches them, as AdamW skips them in the
    reference); "active" puts them in."""
    import torch.nn as nn
    from radhip.wavlm import LoraLinear, inert_lora_params
    torch.manual_seed(0)
    lin = nn.Linear(6, 6)
    on, off = LoraLinear(lin, 2, 4, 0.0, active=True), LoraLinear(nn.Linear(6, 6), 2, 4, 0.0, active=False)
    with torch.no_grad():
        for m in (on, off):
            m.lora_B["default"].weight.normal_()
        off.base_layer.load_state_dict(lin.state_dict())
    x = torch.randn(3, 6)
    torch.testing.assert_close(off(x), lin(x), rtol=0, atol=0)
    assert float((on(x) - lin(x)).abs().max()) > 1e-4
    ids = {id(p) for p in inert_lora_params(nn.ModuleList([on, off]))}
    assert ids == {id(p) for p in list(off.lora_A.parameters()) + list(off.lora_B.parameters())}


def test_reference_mode_bypasses_only_the_attention_projections():
    """HF WavLM skips calling only q/k/v/out_proj (it hands their tensors to
    F.multi_head_attention_forward); an adapter on the FFN's Linears is called as a module, so peft applies it.
    In lora_mode "reference" the product therefore bypasses the attention adapters and keeps the others active."""
    import torch.nn as nn
    from radhip.wavlm import Attention, LoraLinear, inject_lora

    class Layer(nn.Module):
        def __init__(self):
            super().__init__()
            self.attention = Attention.__new__(Attention)
            nn.Module.__init__(self.attention)
            self.attention.q_proj, self.attention.v_proj = nn.Linear(4, 4), nn.Linear(4, 4)
            self.feed_forward = nn.Module()
            self.feed_forward.intermediate_dense = nn.Linear(4, 8)
    targets = ("q_proj", "v_proj", "intermediate_dense")
    _, n = inject_lora(Layer(), r=2, alpha=4, dropout=0.0, targets=targets, active=False)
    wrapped, _ = inject_lora(Layer(), r=2, alpha=4, dropout=0.0, targets=targets, active=False)
    layer = wrapped.model if hasattr(wrapped, "model") else next(iter(wrapped.children()))
    assert n == 3
    assert isinstance(layer.attention.q_proj, LoraLinear) and not layer.attention.q_proj.active
    assert not layer.attention.v_proj.active
    assert isinstance(layer.feed_forward.intermediate_dense, LoraLinear)
    assert layer.feed_forward.intermediate_dense.active
    wrapped2, _ = inject_lora(Layer(), r=2, alpha=4, dropout=0.0, targets=targets, active=True)
    layer2 = wrapped2.model if hasattr(wrapped2, "model") else next(iter(wrapped2.children()))
    assert layer2.attention.q_proj.active and layer2.feed_forward.intermediate_dense.active
