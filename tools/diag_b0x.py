"""Diagnostics of the fused block-0 backward vs the unfused path: relative L2 error of every gradient, and of
d conv2.weight per tap, at a few shapes (tools only)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "robust-audio-deepfake-evolution_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402


class MP:
    def setenv(self, k, v):
        os.environ[k] = v


def main():
    import test_b0x_gpu as T
    mp = MP()
    for (N, H, W) in [(1, 2, 3), (1, 1, 6), (1, 1, 130), (1, 3, 400), (2, 23, 21490)]:
        blk = T._block(N + W + 1)
        x = T._x(N, H, W, seed=W + 1)
        y1, dx1, g1 = T._run(blk, x, True, mp, fused_bwd=True)
        y0, dx0, g0 = T._run(blk, x, False, mp)
        errs = {k: round(T._rel(g1[k], g0[k]), 6) for k in g0}
        print(N, H, W, "dx", round(T._rel(dx1, dx0), 7), errs, flush=True)
        a, b = g1["conv2.weight"], g0["conv2.weight"]
        print("   per tap", [[round(T._rel(a[:, :, kh, kw], b[:, :, kh, kw]), 4) for kw in range(3)] for kh in range(2)])
        print("   ratio", float((a * b).sum() / (b * b).sum()))


if __name__ == "__main__":
    main()
