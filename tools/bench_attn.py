"""Micro-benchmark of the fused gated-bias attention (rdx_attn_fwd / rdx_attn_bwd) at the Phase-6 shape
(B = 8 (env B), T = 201, H = 16, 64-dim heads, dropout 0.1); also the program the PMC passes of
tools/gpu_prof.sh profile.
  B=32 python tools/bench_attn.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402

from radhip.ops import GatedAttention  # noqa: E402


def main():
    B, T, H = int(os.environ.get("B", "8")), 201, 16
    P = float(os.environ.get("P", "0.1"))
    dt = torch.float16 if os.environ.get("DT") == "fp16" else torch.bfloat16    # fp16: libradhip_f16.so
    E = H * 64
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * E, device=dev, dtype=dt)
    q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    q, k, v = (t.detach().requires_grad_(True) for t in (q, k, v))
    gate = torch.rand(B, T, H, device=dev) + 1.0
    tab = torch.randn(H, 2 * T - 1, device=dev)                 # WavLM's bias depends on key - query only
    i = torch.arange(T, device=dev)
    pb = tab[:, i[None, :] - i[:, None] + T - 1].contiguous()
    seed = torch.tensor([7], dtype=torch.int64, device=dev)
    do = torch.randn(B, T, E, device=dev, dtype=dt)
    for _ in range(3):
        o = GatedAttention.apply(q, k, v, gate, pb, seed, P, 0)
        o.backward(do)
    torch.cuda.synchronize()
    reps = 50
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    for _ in range(reps):
        o = GatedAttention.apply(q, k, v, gate, pb, seed, P, 0)
    ev[1].record()
    outs = [GatedAttention.apply(q, k, v, gate, pb, seed, P, 0) for _ in range(reps)]
    torch.cuda.synchronize()
    ev[2].record()
    for o in outs:
        o.backward(do)
    ev[3].record()
    torch.cuda.synchronize()
    fwd = ev[0].elapsed_time(ev[1]) / reps * 1e3
    bwd = ev[2].elapsed_time(ev[3]) / reps * 1e3
    fl = 2.0 * 2 * B * H * T * T * 64
    print(json.dumps({"B": B, "p": P, "split": os.environ.get("RADHIP_ATTN_SPLIT", "1"), "fwd_us": round(fwd, 2),
                      "bwd_us": round(bwd, 2), "fwd_tflops": round(fl / fwd / 1e6, 2),
                      "bwd_tflops": round(2.5 * fl / bwd / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
