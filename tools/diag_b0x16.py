"""Where the fused and unfused SincNet block-0 forwards differ in fp16 storage (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import torch  # noqa: E402

from test_b0x_gpu import _block, _x  # noqa: E402


class MP:
    def setenv(self, k, v):
        os.environ[k] = v


def run(blk, x, fused, dt):
    os.environ["RADHIP_B0X"] = "1" if fused else "0"
    with torch.no_grad(), torch.autocast("cuda", dtype=dt):
        return blk(x.clone())


for dt in (torch.bfloat16, torch.float16):
    for N, H, W in ((2, 23, 21490), (3, 23, 1001), (1, 5, 3)):
        blk = _block(N + W)
        x = _x(N, H, W, seed=W)
        y1, y0 = run(blk, x, True, dt), run(blk, x, False, dt)
        d = (y1.float() - y0.float()).abs()
        bad = (y1 != y0)
        print(dt, (N, H, W), "mismatches", int(bad.sum()), "of", y1.numel(), "max diff", float(d.max()),
              "max |y|", float(y0.float().abs().max()), flush=True)
        if bad.any():
            idx = bad.nonzero()[:5].tolist()
            for i in idx:
                print("   at", i, float(y1[tuple(i)]), float(y0[tuple(i)]))
            # per channel / per row histogram
            print("   channels", bad.sum((0, 2, 3)).tolist())
            print("   rows", bad.sum((0, 1, 3)).tolist())

# the test's criterion
from test_b0x_gpu import _same_forward  # noqa: E402
blk = _block(2 + 21490)
x = _x(2, 23, 21490, seed=21490)
y1, y0 = run(blk, x, True, torch.float16), run(blk, x, False, torch.float16)
d = (y1.float() - y0.float()).abs()
print("max abs diff", float(d.max()), "mismatch frac", float((y1 != y0).float().mean()), "same_forward",
      _same_forward(y1, y0))
