"""SincNet block 0 at the bench's batch (B = 32, H = 23, W = 21490): the one-pass HIP forward / backward
(radhip.ops.Block0Fused) and the unfused kernels, timed with HIP events (us per pass), for PMC runs.

    python tools/bench_b0x.py [--B 32] [--reps 5] [--only fused|unfused]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--amp", default="bf16", choices=["bf16", "fp16"])
    a = ap.parse_args()
    from radhip.sinc import Residual_block
    torch.manual_seed(0)
    blk = Residual_block([1, 32], first=True).cuda().eval()
    N, H, W = a.B, 23, 21490
    dt = torch.bfloat16 if a.amp == "bf16" else torch.float16
    x = torch.randn(N, 1, H, W, device="cuda").as_strided((N, 1, H, W), (H * W, 1, W, 1)).requires_grad_(True)
    for mode in ("fused", "unfused"):
        if a.only and mode != a.only:
            continue
        os.environ["RADHIP_B0X"] = "1" if mode == "fused" else "0"
        with torch.autocast("cuda", dtype=dt):
            y = blk(x)
        dy = torch.randn_like(y)
        times = {"fwd": [], "bwd": []}
        for _ in range(a.reps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            with torch.autocast("cuda", dtype=dt):
                y = blk(x)
            e[1].record()
            y.backward(dy)
            e[2].record()
            torch.cuda.synchronize()
            times["fwd"].append(e[0].elapsed_time(e[1]) * 1e3)
            times["bwd"].append(e[1].elapsed_time(e[2]) * 1e3)
        print(mode, {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}, flush=True)


if __name__ == "__main__":
    main()
