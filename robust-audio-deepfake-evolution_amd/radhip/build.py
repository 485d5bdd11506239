"""Model construction shared by main.py, bench.py and the smoke test.

get_model (reference src/main.py:799-812): `models.<architecture>.Model(Args(model_config), device)`.
apply_lora_to_wavlm (reference src/main.py:103-158): freeze the WavLM base, inject LoRA (r, alpha,
dropout, q_proj/v_proj) with peft's state-dict layout, no silent fallback.
"""
import inspect
import json
import os
from importlib import import_module

import torch

from .wavlm import PeftWrapped, inject_lora

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIG_DIR = os.path.join(PKG_DIR, "config")


class Args:
    def __init__(self, d):
        self.__dict__.update(d)


def load_config(path):
    if not os.path.exists(path) and os.path.exists(os.path.join(CONFIG_DIR, os.path.basename(path))):
        path = os.path.join(CONFIG_DIR, os.path.basename(path))
    with open(path) as f:
        return json.load(f)


def legacy_plugin(cls):
    """True for the AASIST-era plugin signature Model(d_args) (models/AASIST.py:470,
    models/RawNet2Spoof.py:170): one positional argument, the model_config dict itself."""
    params = [p for p in inspect.signature(cls.__init__).parameters.values()
              if p.name != "self" and p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
    return len(params) == 1


def get_model(model_config, device, extra=None):
    """models.<architecture>.Model: the Phase-5/6 plugins take (Args(model_config), device) (src/main.py:799-812);
    the legacy AASIST / RawNet2 plugins take the model_config dict alone (their reference signature, which
    the reference's own get_model cannot call)."""
    module = import_module("models.{}".format(model_config["architecture"]))
    d = dict(model_config)
    if extra:
        d.update(extra)
    cls = getattr(module, "Model")
    model = cls(d) if legacy_plugin(cls) else cls(Args(d), device)
    return model.to(device)


LORA_MODES = ("reference", "active")


def apply_lora_to_wavlm(model, training_config):
    """training_config "lora_mode": "reference" (default) injects the adapters the way the reference's HF
    WavLM ends up using them, i.e. bypassed (radhip.wavlm.LoraLinear); "active" applies them."""
    mode = training_config.get("lora_mode", "reference")
    if mode not in LORA_MODES:
        raise ValueError(f"lora_mode must be one of {LORA_MODES}, got {mode!r}")
    if not training_config.get("use_lora", False):
        return model
    if not (hasattr(model, "wavlm_stream") and hasattr(model.wavlm_stream, "model")):
        raise RuntimeError("use_lora is set but the model has no wavlm_stream.model")
    if isinstance(model.wavlm_stream.model, PeftWrapped):
        return model        # already injected (the reference injects twice in --eval; once is enough)
    base = model.wavlm_stream.model
    for p in base.parameters():
        p.requires_grad = False
    wrapped, n = inject_lora(base, r=training_config.get("lora_r", 8), alpha=training_config.get("lora_alpha", 32),
                             dropout=training_config.get("lora_dropout", 0.1),
                             targets=tuple(training_config.get("lora_target_modules", ["q_proj", "v_proj"])),
                             active=(mode == "active"))
    if n == 0:
        raise RuntimeError("LoRA: no target modules found")
    model.wavlm_stream.model = wrapped
    dev = next(base.parameters()).device
    wrapped.to(dev)
    return model


def trainable_count(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def strip_module_prefix(sd):
    return {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}


def load_weights(model, path, device="cpu", strict=True):
    """Reference checkpoints: plain state_dict or {'model_state_dict': ...}, optional DataParallel/EMA
    'module.' prefix and EMA 'n_averaged' entry (main.py:246-268,336-359). Loaded with
    weights_only=True; strict by default (the reference's strict=False silently drops mismatches)."""
    ck = torch.load(path, map_location=device, weights_only=True)
    sd = ck["model_state_dict"] if isinstance(ck, dict) and "model_state_dict" in ck else ck
    sd = strip_module_prefix(sd)
    sd.pop("n_averaged", None)
    from .wavlm import remap_peft_keys
    sd = remap_peft_keys(sd, set(model.state_dict().keys()))
    return model.load_state_dict(sd, strict=strict)
