"""Diagnostics: which source lines issue the dtype casts / elementwise ops of one Phase-6 micro-step
(autocast dtype from AMP=fp16|bf16, default fp16 as bench.py; full-size model, B=2), and which SDPA backend the
WavLM attention takes."""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from radhip.build import apply_lora_to_wavlm, get_model, load_config  # noqa: E402


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func).replace("aten.", "").replace(".default", "")
        if name in ("view", "_unsafe_view", "t", "transpose.int", "permute", "expand", "unsqueeze", "squeeze.dim",
                    "detach", "as_strided", "slice.Tensor", "select.int", "split.Tensor", "alias", "reshape"):
            return out
        st = [f for f in traceback.extract_stack()[:-1]
              if ("/radhip/" in f.filename or "/models/" in f.filename) and "op_sites" not in f.filename]
        loc = f"{st[-1].filename.split('/')[-1]}:{st[-1].lineno}" if st else "<autograd>"
        key = name
        if name in ("_to_copy", "copy_", "clone", "contiguous") and hasattr(args[0], "dtype"):
            src = args[1] if name == "copy_" else args[0]
            dst = args[0] if name == "copy_" else out
            key = (f"{name} {str(src.dtype)[6:]}->{str(getattr(dst, 'dtype', '?'))[6:]} {tuple(src.shape)}"
                   f" c={int(src.is_contiguous())}{int(dst.is_contiguous())}")
        self.c[(key, loc)] += 1
        return out


AMP = {"fp16": torch.float16, "bf16": torch.bfloat16}[os.environ.get("AMP", "fp16")]


def main():
    dev = torch.device("cuda", 0)
    cfg = load_config("Phase6_Proposed.conf")
    torch.manual_seed(0)
    m = apply_lora_to_wavlm(get_model(cfg["model_config"], dev), cfg["training_config"])
    m.wavlm_stream._core().config.layerdrop = 0.0
    m.train()
    x = torch.randn(2, 64600, device=dev) * 0.1
    y = torch.tensor([0, 1], device=dev)
    for _ in range(2):
        with torch.autocast("cuda", dtype=AMP):
            _, out = m(x)
            loss = torch.nn.functional.cross_entropy(out.float(), y)
        loss.backward()
    torch.cuda.synchronize()
    with Sites() as s:
        with torch.autocast("cuda", dtype=AMP):
            _, out = m(x)
            loss = torch.nn.functional.cross_entropy(out.float(), y)
        loss.backward()
    torch.cuda.synchronize()
    tot = collections.Counter()
    for (k, loc), v in s.c.items():
        tot[k] += v
    print("== op totals (fwd+bwd, one pass)")
    for k, v in tot.most_common(40):
        print(f"{v:6d} {k}")
    print("== top (op, site)")
    for (k, loc), v in s.c.most_common(90):
        print(f"{v:6d} {k:40s} {loc}")
    return
    # SDPA backend with the WavLM attention shapes (B=2, H=16, T=201, Dh=64, float bias mask)
    from torch.profiler import ProfilerActivity, profile
    q = torch.randn(2, 16, 201, 64, device=dev, dtype=torch.bfloat16, requires_grad=True)
    bias = torch.randn(2, 16, 201, 201, device=dev, dtype=torch.bfloat16)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        o = torch.nn.functional.scaled_dot_product_attention(q, q, q, attn_mask=bias, dropout_p=0.1)
        o.sum().backward()
        torch.cuda.synchronize()
    print("== SDPA kernels")
    for e in prof.key_averages():
        if e.device_type.name == "CUDA" or "cuda" in str(e.device_type).lower():
            print(f"{e.count:4d} {e.key[:120]}")


if __name__ == "__main__":
    main()
