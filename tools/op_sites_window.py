"""Which source lines issue the torch (non-radhip) device ops of one accumulation window as bench.py runs it
(Phase-6 config, micro-batch 8 x accumulation 4, fp16 autocast + GradScaler, FGM, the eager window: the same
launches the captured graphs replay). Prints op counts per (op, shape, source line), the radhip C-ABI calls
excluded (they do not go through the dispatcher), so the torch glue left around the hand-written kernels can be
attributed and removed.

  python tools/op_sites_window.py [--top 120]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

SKIP = {"view", "_unsafe_view", "t", "transpose.int", "permute", "expand", "unsqueeze", "squeeze.dim", "detach",
        "as_strided", "slice.Tensor", "select.int", "split.Tensor", "alias", "reshape", "empty.memory_format",
        "empty_like", "empty_strided", "_local_scalar_dense", "set_.source_Storage", "squeeze", "unbind.int",
        "split_with_sizes", "chunk", "lift_fresh", "record_stream"}


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func).replace("aten.", "").replace(".default", "")
        if name in SKIP:
            return out
        t0 = next((a for a in args if isinstance(a, torch.Tensor)), None)
        if t0 is not None and not t0.is_cuda:
            return out
        st = [f for f in traceback.extract_stack()[:-1]
              if ("/radhip/" in f.filename or "/models/" in f.filename) and "op_sites" not in f.filename]
        if st:
            loc = f"{st[-1].filename.split('/')[-1]}:{st[-1].lineno}"
        else:   # issued by the autograd engine: name the backward node running it
            node = torch._C._current_autograd_node()
            loc = f"<autograd {node.name()}>" if node is not None else "<autograd>"
        shp = tuple(t0.shape) if t0 is not None else ()
        dts = str(t0.dtype)[6:] if t0 is not None else ""
        self.c[(name, dts, shp, loc)] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=120)
    args = ap.parse_args()
    import bench
    from radhip.build import load_config
    from radhip.train import Trainer, total_optimizer_steps
    from radhip.window import WindowStep
    dev = torch.device("cuda", 0)
    config = load_config("Phase6_Proposed.conf")
    config["training_config"]["accumulation_steps"] = 4
    config["batch_size"] = 8
    model = bench.build(config, dev, 0.0)
    tr = Trainer(model, config, dev, total_optimizer_steps(1, 40, 4), torch.float16)
    B, K = 8, 4
    w = WindowStep(tr, B, graphs=False)
    rng = np.random.default_rng(0)

    def window():
        for k in range(K):
            w.xslot(k).copy_(torch.from_numpy(np.clip(0.1 * rng.standard_normal((B, 64600)), -1, 1)
                                              .astype(np.float32)))
            w.add(k, rng.integers(0, 2, B), 0.5, list(rng.permutation(B)))
        w.run()

    for _ in range(2):
        window()
    torch.cuda.synchronize()
    with Sites() as s:
        window()
    torch.cuda.synchronize()
    tot = collections.Counter()
    for (name, dts, shp, loc), v in s.c.items():
        tot[name] += v
    print(f"== torch device ops per window: {sum(s.c.values())}")
    for k, v in tot.most_common(40):
        print(f"{v:6d} {k}")
    print("== top (op, dtype, shape, site)")
    for (name, dts, shp, loc), v in s.c.most_common(args.top):
        print(f"{v:6d} {name:32s} {dts:8s} {str(shp):24s} {loc}")


if __name__ == "__main__":
    main()
