"""Per-shape timing of the SincNet residual convolutions: csrc/sconv.hip (radhip.ops.SConv) vs MIOpen
(F.conv2d on channels_last bf16, what the bf16-autocast module path runs), forward and forward+backward,
at the Phase-6 shapes (B = 8 adversarial pass, B = 32 clean window pass).

    python tools/bench_sconv.py [--batch 8 32] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "robust-audio-deepfake-evolution_amd"))
from radhip.ops import SConv  # noqa: E402

# (name, C_in, C_out, KH, ph, H_in, W)
SHAPES = [("b0.conv2", 32, 32, 2, 0, 24, 21490), ("b1.conv1", 32, 32, 2, 1, 23, 7163), ("b1.conv2", 32, 32, 2, 0, 24, 7163),
          ("b2.conv1", 32, 64, 2, 1, 23, 2387), ("b2.conv2", 64, 64, 2, 0, 24, 2387), ("b2.ds", 32, 64, 1, 0, 23, 2387),
          ("b3.conv1", 64, 64, 2, 1, 23, 795), ("b3.conv2", 64, 64, 2, 0, 24, 795), ("b5.conv1", 64, 64, 2, 1, 23, 88)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[8, 32])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    from radhip import ops
    ops.SCONV_WCACHE = {}     # weight layouts prepared once per weight, as inside a training window
    rows = []
    for B in a.batch:
        for name, ci, co, kh, ph, H, W in SHAPES:
            x = torch.randn(B, ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            w = (0.1 * torch.randn(co, ci, kh, 3, device=dev)).requires_grad_(True)
            wb = w.detach().to(torch.bfloat16).requires_grad_(True)
            xr = x.clone().requires_grad_(True)
            y = F.conv2d(x, wb, None, 1, (ph, 1))
            dy = torch.randn_like(y)

            def mi_f():
                F.conv2d(x, wb, None, 1, (ph, 1))

            def mi_fb():
                F.conv2d(xr, wb, None, 1, (ph, 1)).backward(dy)

            def sc_f():
                SConv.apply(x, w, ph)

            def sc_fb():
                SConv.apply(xr, w, ph).backward(dy)
            r = {"B": B, "conv": name, "gflop_fwd": 2.0 * B * y.shape[2] * W * co * ci * kh * 3 / 1e9,
                 "miopen_fwd_us": timeit(mi_f, a.iters), "sconv_fwd_us": timeit(sc_f, a.iters),
                 "miopen_fwdbwd_us": timeit(mi_fb, a.iters), "sconv_fwdbwd_us": timeit(sc_fb, a.iters)}
            rows.append(r)
            print(json.dumps(r), flush=True)
    tot = {k: sum(r[k] for r in rows) for k in ("miopen_fwd_us", "sconv_fwd_us", "miopen_fwdbwd_us", "sconv_fwdbwd_us")}
    print(json.dumps({"total": tot}))


if __name__ == "__main__":
    main()
