"""Micro-benchmark of the hand-written kernels that dominate the bench step, at the window's batch shapes
(env B: 8 = an adversarial pass, 32 = the batched clean pass): the gated attention (forward, backward),
the WavLM positional conv (forward, backward) and the SincNet block-0 backward. It is also the program the
rocprofv3 PMC passes of tools/gpu_prof.sh profile (one counter group per run).

  B=32 python tools/bench_kernels.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402

from radhip.ops import Block0Convs, GatedAttention, PosConv, SConv, SConvBnSelu, posconv_weights  # noqa: E402

# the SincNet residual-stack convolutions of one pass (Residual_block, blocks 0-5): (C_in, C_out, KH, ph, H, W),
# conv1 (2x3 pad (1,1), with the BN+SELU epilogue), conv2 (2x3 pad (0,1)), conv_downsample (1x3)
SINCNET_CONVS = [(32, 32, 2, 0, 24, 21490),
                 (32, 32, 2, 1, 23, 7163), (32, 32, 2, 0, 24, 7163),
                 (32, 64, 2, 1, 23, 2387), (64, 64, 2, 0, 24, 2387), (32, 64, 1, 0, 23, 2387)] + \
                [c for w in (795, 265, 88) for c in ((64, 64, 2, 1, 23, w), (64, 64, 2, 0, 24, w))]


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    B, T, H = int(os.environ.get("B", "8")), 201, 16
    E = H * 64
    dev = "cuda"
    torch.manual_seed(0)
    out = {"B": B}
    # attention
    qkv = torch.randn(B, T, 3 * E, device=dev, dtype=torch.bfloat16)
    q, k, v = (t.detach().requires_grad_(True) for t in (qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]))
    gate = torch.rand(B, T, H, device=dev) + 1.0
    ii = torch.arange(T, device=dev)
    pb = torch.randn(H, 2 * T - 1, device=dev)[:, ii[None, :] - ii[:, None] + T - 1]   # relative-position bias
    seed = torch.tensor([7], dtype=torch.int64, device=dev)
    do = torch.randn(B, T, E, device=dev, dtype=torch.bfloat16)
    out["attn_fwd_us"] = timed(lambda: GatedAttention.apply(q, k, v, gate, pb, seed, 0.1, 0), 20)
    o = GatedAttention.apply(q, k, v, gate, pb, seed, 0.1, 0)
    out["attn_fwd_bwd_us"] = timed(lambda: torch.autograd.grad(GatedAttention.apply(q, k, v, gate, pb, seed, 0.1, 0),
                                                               (q, k, v), do), 20)
    del o
    # positional conv
    w = torch.randn(1024, 64, 128, device=dev) * 0.01
    bias = torch.randn(1024, device=dev) * 0.1
    wk, wkt = posconv_weights(w)
    h = torch.randn(B, T, E, device=dev, dtype=torch.bfloat16).requires_grad_(True)
    out["posconv_fwd_us"] = timed(lambda: PosConv.apply(h, wk, wkt, bias), 20)
    out["posconv_fwd_bwd_us"] = timed(lambda: torch.autograd.grad(PosConv.apply(h, wk, wkt, bias), h, do), 20)
    # SincNet block 0 (input [B, 1, 23, 21490], 32 channels)
    x = torch.randn(B, 1, 23, 21490, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w1 = (0.3 * torch.randn(32, 1, 2, 3, device=dev)).requires_grad_(True)
    wd = (0.3 * torch.randn(32, 1, 1, 3, device=dev)).requires_grad_(True)
    c, idn = Block0Convs.apply(x, w1, wd)
    gc = torch.randn(c.shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gi = torch.randn(idn.shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out["b0_fwd_bwd_us"] = timed(lambda: torch.autograd.grad(Block0Convs.apply(x, w1, wd), (x, w1, wd), (gc, gi)), 5)
    # SincNet convolutions: forward + backward (input and weight gradient) of every conv of one pass
    def sincnet_pass():
        for ci, co, kh, ph, H, W in SINCNET_CONVS:
            xs = torch.randn(B, ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            xs.requires_grad_(True)
            wt = (0.1 * torch.randn(co, ci, kh, 3, device=dev)).requires_grad_(True)
            if ph == 1 and kh == 2:
                z = torch.zeros(co, device=dev)
                y = SConvBnSelu.apply(xs, wt, ph, z, z, z + 1, z + 1, z)
            else:
                y = SConv.apply(xs, wt, ph)
            torch.autograd.grad(y, (xs, wt), torch.ones_like(y))
    out["sincnet_convs_fwd_bwd_us"] = timed(sincnet_pass, 3)
    print(json.dumps({kk: round(vv, 1) if isinstance(vv, float) else vv for kk, vv in out.items()}), flush=True)


if __name__ == "__main__":
    main()
