"""Checkpoint compatibility with the reference's files (src/main.py:246-268, :336-359, :602-664).

The reference saves `eval_model.state_dict()`, where eval_model is torch's AveragedModel EMA wrapper when
use_ema is on: every key gets the "module." prefix and an "n_averaged" counter is added; the LoRA keys are
peft's (`...q_proj.base_layer.weight` on newer peft, `...q_proj.weight` on older, plus
`...q_proj.lora_A.default.weight`). Here the file is produced by that same torch code path
(torch.optim.swa_utils.AveragedModel over the product model, as the reference constructs it), in both peft
layouts and inside {"model_state_dict": ...}, then loaded STRICTLY into a fresh model (radhip.build.load_weights,
what --eval / --eval_model_weights / --resume use): the logits must equal the EMA model's own."""
import json

import pytest
import torch
from torch.optim.swa_utils import AveragedModel, get_ema_multi_avg_fn

from seeded import seeded_array, seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(golden, seed):
    from radhip.build import apply_lora_to_wavlm, get_model, load_config
    cfg = load_config("Phase6_Proposed.conf")
    cfg["model_config"]["num_encoders"] = 2
    cfg["model_config"]["wavlm_config"] = json.loads(str(golden("model_tiny.npz")["wavlm_config"]))
    m = apply_lora_to_wavlm(get_model(cfg["model_config"], "cpu"), cfg["training_config"])
    seeded_fill_(m, seed=seed)
    return m.to(DEV), cfg


def _old_peft(sd):
    return {k.replace(".base_layer.", "."): v for k, v in sd.items()}


@pytest.mark.parametrize("layout", ["new_peft", "old_peft", "model_state_dict"])
def test_reference_ema_checkpoint_loads_strictly_and_reproduces_logits(golden, tmp_path, layout):
    from radhip.build import load_weights
    m, _ = _model(golden, seed=51)
    ema = AveragedModel(m, multi_avg_fn=get_ema_multi_avg_fn(0.999))    # the reference's EMA (main.py:495)
    for step in range(3):                                              # a few updates after moving the live model
        with torch.no_grad():
            for p in m.parameters():
                if p.requires_grad:
                    p.add_(0.01 * (step + 1))
        ema.update_parameters(m)
    sd = ema.state_dict()
    assert "n_averaged" in sd and all(k.startswith("module.") for k in sd if k != "n_averaged")
    assert any(".lora_A.default.weight" in k for k in sd) and any(".base_layer.weight" in k for k in sd)
    if layout == "old_peft":
        sd = _old_peft(sd)
    obj = {"model_state_dict": sd} if layout == "model_state_dict" else sd
    path = tmp_path / "best.pth"
    torch.save(obj, path)

    fresh, _ = _model(golden, seed=52)
    load_weights(fresh, path, DEV, strict=True)
    x = torch.from_numpy(seeded_array("ckpt.x", (2, 64600), scale=0.1)).float().to(DEV)
    ema.module.eval()
    fresh.eval()
    with torch.no_grad():
        _, want = ema.module(x)
        _, got = fresh(x)
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6)
    for k, v in ema.module.state_dict().items():
        assert torch.equal(fresh.state_dict()[k], v), k


def test_strict_load_rejects_a_mismatched_checkpoint(golden, tmp_path):
    from radhip.build import load_weights
    m, _ = _model(golden, seed=51)
    sd = {"module." + k: v for k, v in m.state_dict().items()}
    sd.pop(next(k for k in sd if "lora_B" in k))
    torch.save(sd, tmp_path / "bad.pth")
    fresh, _ = _model(golden, seed=52)
    with pytest.raises(RuntimeError, match="Missing key"):
        load_weights(fresh, tmp_path / "bad.pth", DEV, strict=True)
