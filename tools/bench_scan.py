"""Selective-scan fwd/bwd microbenchmark at the Phase-6 bench shape (B=8, L=201, Di=288, N=16,
both directions, bf16 storage); prints avg kernel time (HIP events on the launch stream) and the
achieved algorithmic GB/s (same accounting as radhip/ops.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402

from radhip import ops  # noqa: E402


def main(B=8, L=201, D=288, N=16, R=9, dirs=2, dt=torch.bfloat16, iters=50):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(dirs, B, L, D, device=dev, generator=g).to(dt).requires_grad_()
    delta = (0.5 * torch.randn(dirs, B, L, D, device=dev, generator=g)).to(dt).requires_grad_()
    xdbl = torch.randn(dirs, B, L, R + 2 * N, device=dev, generator=g).to(dt).requires_grad_()
    A_log = torch.log(torch.arange(1, N + 1, device=dev, dtype=torch.float32)).repeat(D, 1).requires_grad_()
    Dp = torch.ones(D, device=dev, requires_grad=True)
    bias = (0.1 * torch.randn(D, device=dev, generator=g)).requires_grad_()
    Bm, Cm = xdbl[..., R:R + N], xdbl[..., R + N:]
    dy = torch.randn(dirs, B, L, D, device=dev, generator=g)
    for _ in range(3):
        y = ops.SelectiveScan.apply(u, delta, A_log, Bm, Cm, Dp, bias)
        y.backward(dy)
    torch.cuda.synchronize()
    ops.TIMING = {}
    for _ in range(iters):
        y = ops.SelectiveScan.apply(u, delta, A_log, Bm, Cm, Dp, bias)
        y.backward(dy)
    torch.cuda.synchronize()
    timing, ops.TIMING = ops.TIMING, None
    for name, evs in timing.items():
        ms = sum(s.elapsed_time(e) for s, e, _ in evs) / len(evs)
        work = evs[0][2]
        print(f"{name:22s} {1e3 * ms:8.2f} us  {work / (ms * 1e-3) / 1e9:8.1f} GB/s  "
              f"({work / 1e6:.2f} MB algorithmic)  seg={os.environ.get('RADHIP_SCAN_BWD_SEG', '4')}", flush=True)


if __name__ == "__main__":
    main()
