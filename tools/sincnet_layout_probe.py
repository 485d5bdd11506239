"""Probe: SincNet residual encoder fwd+bwd time at B=8 under layout / dtype variants (MIOpen)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch
from radhip.sinc import SincNetEncoder

def run(enc, x, amp, cl, iters=3):
    for it in range(iters + 1):
        if it == 1:
            torch.cuda.synchronize(); t0 = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            pooled = enc.conv_time.absmaxpool(x).unsqueeze(1)
            h = enc.selu(enc.first_bn(pooled))
            if cl:
                h = h.contiguous(memory_format=torch.channels_last)
            e = enc.encoder(h)
            out = torch.max(torch.abs(e), dim=2)[0]
        out.float().sum().backward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3

dev = "cuda"
x = torch.randn(8, 64600, device=dev) * 0.1
for amp in [True, False]:
    for cl in [False, True]:
        enc = SincNetEncoder().to(dev)
        enc.eval()
        if cl:
            enc = enc.to(memory_format=torch.channels_last)
        try:
            ms = run(enc, x, amp, cl)
            print(f"amp={amp} channels_last={cl}: {ms:.1f} ms fwd+bwd", flush=True)
        except Exception as e:
            print(f"amp={amp} channels_last={cl}: FAILED {e}", flush=True)
