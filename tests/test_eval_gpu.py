"""Scoring pass (BASELINE configs 3 and 5, main.py --eval): radhip.infer._scores in the reference's fp32 and with
--eval_amp bf16, which takes the hand-written HIP path (fused WavLM encoder layers, SincNet block 0 in one pass).
Same random-init Phase-6 weights and inputs for both. The bf16 scores must stay close to the fp32 ones: the bound
is 0.05 absolute on logits[:, 1] (tools/bench_eval.py measured 0.013 max / 0.008 mean over 192 utterances, rank
correlation 0.995; with random weights the scores spread only ~0.02, so this is a bf16 accuracy check, not an EER
parity claim: no trained checkpoint exists here). --eval_amp fp16 (libradhip_f16.so) is held to a 4x tighter bound:
fp16 keeps 3 more mantissa bits."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt,bound", [(torch.bfloat16, 0.05), (torch.float16, 0.0125)])
def test_eval_16bit_scores_track_fp32(dt, bound):
    from radhip.build import apply_lora_to_wavlm, get_model, load_config
    from radhip.infer import _scores
    dev = torch.device("cuda", 0)
    cfg = load_config("Phase6_Proposed.conf")
    torch.manual_seed(1234)
    model = apply_lora_to_wavlm(get_model(cfg["model_config"], dev), cfg["training_config"]).eval()
    rng = np.random.default_rng(3)
    x = torch.from_numpy(np.clip(0.1 * rng.standard_normal((4, 64600)), -1, 1).astype(np.float32)).to(dev)
    with torch.no_grad():
        s32 = _scores(model, x).double()
        s16 = _scores(model, x, None, dt).double()
    enc = model.wavlm_stream._core().encoder
    assert enc.__dict__.get("_fused_ok", (None, False))[1], "16-bit eval did not take the fused encoder path"
    assert torch.isfinite(s16).all()
    print(f"[eval {dt}] max |score - fp32 score| {float((s16 - s32).abs().max()):.3e}")
    assert float((s16 - s32).abs().max()) < bound, (s16, s32)
