"""Eval (scoring) throughput of the Phase-6 model (BASELINE configs 3 and 5: the ASVspoof 2019-LA / 2021-DF score
passes of main.py --eval), synthetic utterances of the scoring length (64 600 samples), batch 32 as the reference's
test loader: the reference's fp32 forward, and the bf16-autocast forward that runs the hand-written HIP path (fused
WavLM encoder layers, attention, SincNet block 0 / sconv), and x3: the fp32 forward with the WavLM stream on the
split-precision kernels (radhip/wavlm_x3.py). Random-init weights (no checkpoint); the score is
logits[:, 1] exactly as radhip.infer._scores takes it. Prints one JSON line: utt/s and ms/utt per precision, and
the bf16 scores' deviation from the fp32 scores of the same weights and inputs.

    python tools/bench_eval.py [--batch 32] [--batches 6] [--warmup 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--modes", default="fp32,x3,bf16,fp16", help="comma list of fp32 / x3 / bf16 / fp16")
    a = ap.parse_args()
    modes = {"fp32": None, "x3": "x3", "bf16": torch.bfloat16, "fp16": torch.float16}
    from radhip.build import apply_lora_to_wavlm, get_model, load_config
    from radhip.infer import _scores
    dev = torch.device("cuda", 0)
    cfg = load_config("Phase6_Proposed.conf")
    torch.manual_seed(1234)
    model = apply_lora_to_wavlm(get_model(cfg["model_config"], dev), cfg["training_config"]).eval()
    rng = np.random.default_rng(7)
    xs = [torch.from_numpy(np.clip(0.1 * rng.standard_normal((a.batch, 64600)), -1, 1).astype(np.float32)).to(dev)
          for _ in range(a.batches)]
    res = {"workload": f"Phase6_Proposed.conf scoring pass, batch {a.batch} x 64600 samples, random-init weights",
           "batches": a.batches}
    scores = {}
    with torch.no_grad():
        for name in a.modes.split(","):
            amp = modes[name]
            for i in range(a.warmup):
                _scores(model, xs[i % len(xs)], None, amp)
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = [_scores(model, x, None, amp) for x in xs]
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            n = a.batch * a.batches
            scores[name] = torch.cat(out).double()
            res[name] = {"utt_s": round(n / dt, 2), "ms_per_utt": round(dt / n * 1e3, 3),
                         "ms_per_batch": round(dt / a.batches * 1e3, 2)}
    for name in scores:
        if name == "fp32" or "fp32" not in scores:
            continue
        d = (scores[name] - scores["fp32"]).abs()
        res[name + "_vs_fp32"] = {
            "max_abs_score_diff": float(d.max()), "mean_abs_score_diff": float(d.mean()),
            "fp32_score_std": float(scores["fp32"].std()),
            "rank_corr": float(np.corrcoef(scores["fp32"].cpu().numpy().argsort().argsort(),
                                           scores[name].cpu().numpy().argsort().argsort())[0, 1])}
    res["reference_published"] = "~40 ms per utterance at batch 32 (reference README.md:101-105; other hardware)"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
