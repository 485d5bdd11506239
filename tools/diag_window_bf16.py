"""e_seq of tests/test_window_gpu.py (bf16 reference-order micro-steps vs fp32) under the current env (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"),
                os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_window_gpu as tw  # noqa: E402


def golden(name, _c={}):
    if name not in _c:
        _c[name] = dict(np.load(os.path.join(ROOT, "tests", "golden", name), allow_pickle=False))
    return _c[name]


ref32, _ = tw._grads_sequential(golden, torch.float32)
for dt in (torch.bfloat16, torch.float16):
    seq, _ = tw._grads_sequential(golden, dt)
    print(os.environ.get("VARIANT", "default"), dt, "e_seq", round(tw._rel(seq, ref32), 5), flush=True)
