"""Host-side time of each phase of bench.py's window step (augmentation + draws per micro-batch, graph
replays, optimizer step), to find where the CPU falls behind the GPU between windows.

    python tools/host_times.py [--steps 6]
"""
import argparse
import json
import os
import random as pyrandom
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--amp", default="fp16", choices=["bf16", "fp16"])
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from radhip.build import load_config
    from radhip.train import Augmenter, Trainer, total_optimizer_steps
    from radhip.window import WindowStep
    config = load_config("Phase6_Proposed.conf")
    config["training_config"]["accumulation_steps"] = 4
    config["batch_size"] = 8
    model = bench.build(config, dev, 0.0)
    tr = Trainer(model, config, dev, total_optimizer_steps(1, 400, 4),
                 torch.float16 if a.amp == "fp16" else torch.bfloat16)
    dc = config["data_config"]
    aug = Augmenter(dev, algo=dc.get("rawboost_algo", 0), rawboost_p=dc.get("rawboost_p", 1.0),
                    use_codec=dc.get("use_codec_aug", False), codec_p=dc.get("codec_p", 0.5))
    pool_x, pool_y = bench.synthetic_pool(64, 64000, 1234, dev)
    np.random.seed(1234)
    pyrandom.seed(1234)
    w = WindowStep(tr, 8)
    for k in range(4):
        w.add(k, np.zeros(8, dtype=np.int64))
    w.capture()
    w.reset_host()
    g0, gadv = w.graphs
    T = {}

    def clock(name, t):
        T.setdefault(name, []).append((time.perf_counter() - t) * 1e3)

    for step in range(a.steps):
        for i in range(4):
            t = time.perf_counter()
            idx = np.random.randint(0, 64, size=8)
            offs = [int(j) * 64000 for j in idx]
            plan = aug.draw([64000] * 8)
            lam, perm = tr.mixup_draw(8)
            clock("draw", t)
            t = time.perf_counter()
            aug.run(pool_x, offs, [64000] * 8, plan, perm, lam, out=w.xslot(i))
            clock("aug_run", t)
            t = time.perf_counter()
            w.add(i, pool_y[idx].numpy(), lam, perm)
            clock("window_add", t)
        t = time.perf_counter()
        tr.train_mode()
        w._stage()
        clock("stage", t)
        t = time.perf_counter()
        g0.replay()
        for g in gadv:
            g.replay()
        clock("replays", t)
        t = time.perf_counter()
        tr.micro += 4
        tr.n_seen += 32
        tr.optimizer_step()
        clock("optimizer_step", t)
        w.reset_host()
        t = time.perf_counter()
        torch.cuda.synchronize()
        clock("sync_wait", t)
    out = {k: [round(x, 2) for x in v[-4:]] for k, v in T.items()}
    print(json.dumps(out), flush=True)
    # pipelined as bench.py runs it (no host sync): device-timeline segments between events
    evs = []

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e
    t0 = time.perf_counter()
    for step in range(a.steps):
        ea = ev()
        for i in range(4):
            idx = np.random.randint(0, 64, size=8)
            offs = [int(j) * 64000 for j in idx]
            plan = aug.draw([64000] * 8)
            lam, perm = tr.mixup_draw(8)
            aug.run(pool_x, offs, [64000] * 8, plan, perm, lam, out=w.xslot(i))
            w.add(i, pool_y[idx].numpy(), lam, perm)
        tr.train_mode()
        w._stage()
        eb = ev()
        g0.replay()
        for g in gadv:
            g.replay()
        ec = ev()
        tr.micro += 4
        tr.n_seen += 32
        tr.optimizer_step()
        w.reset_host()
        ed = ev()
        evs.append((ea, eb, ec, ed))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    seg = {"aug_stage": [], "graphs": [], "optimizer": [], "to_next": []}
    for i, (ea, eb, ec, ed) in enumerate(evs):
        seg["aug_stage"].append(round(ea.elapsed_time(eb), 3))
        seg["graphs"].append(round(eb.elapsed_time(ec), 3))
        seg["optimizer"].append(round(ec.elapsed_time(ed), 3))
        if i + 1 < len(evs):
            seg["to_next"].append(round(ed.elapsed_time(evs[i + 1][0]), 3))
    print(json.dumps({"pipelined_wall_ms_per_step": round(wall, 2), **seg}), flush=True)


if __name__ == "__main__":
    main()
