"""Per-pass device time of the captured accumulation window (unprofiled): the clean-pass graph G0 and each
adversarial graph, replayed one at a time between HIP events, with the SincNet stream as a parallel branch
(default) or serialized (RADHIP_SINC_BRANCH=0). Same model / trainer / window as bench.py.

    python tools/pass_times.py [--reps 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from radhip.build import load_config
    from radhip.train import Trainer, total_optimizer_steps
    from radhip.window import WindowStep
    config = load_config("Phase6_Proposed.conf")
    config["training_config"]["accumulation_steps"] = 4
    config["batch_size"] = 8
    model = bench.build(config, dev, 0.0)
    tr = Trainer(model, config, dev, total_optimizer_steps(1, 400, 4), torch.bfloat16)
    out = {}
    for branch in ("1", "0"):
        os.environ["RADHIP_SINC_BRANCH"] = branch
        w = WindowStep(tr, 8, graphs=True)
        for k in range(4):
            w.add(k, np.zeros(8, dtype=np.int64))
        w.capture()
        g0, gadv = w.graphs
        res = {}
        for name, g in [("clean", g0)] + [(f"adv{k}", g) for k, g in enumerate(gadv)]:
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[name] = round(e0.elapsed_time(e1) / a.reps, 3)
        out["branch" if branch == "1" else "serial"] = res
        print(json.dumps({branch: res}), flush=True)
        del w
        torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
