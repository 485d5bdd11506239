"""Replay-idempotence probe: capture small fwd+bwd pieces, replay 3x, compare grads with eager."""
import torch
import torch.nn as nn

dev = "cuda"
torch.manual_seed(0)


def probe(label, mod, make_x):
    mod = mod.to(dev)
    x0 = make_x()
    params = [p for p in mod.parameters()]
    for p in params:
        p.grad = torch.zeros_like(p)
    gy = torch.randn_like(mod(x0))
    # eager reference
    out = mod(x0); out.backward(gy); torch.cuda.synchronize(); del out
    ref = [p.grad.clone() for p in params]
    x = x0.clone().requires_grad_(False)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            mod(x).backward(gy)
    torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mod(x).backward(gy)
    names = [n for n, _ in mod.named_parameters()]
    for r in range(3):
        for p in params:
            p.grad.zero_()
        g.replay(); torch.cuda.synchronize()
        bad = []
        for n, a, p in zip(names, ref, params):
            e = float((a - p.grad).norm() / (a.norm() + 1e-30))
            if e > 1e-4:
                bad.append((n, round(e, 3)))
        print(f"{label} replay {r}: {bad}", flush=True)


B, T, E = 4, 402, 144
probe("linear+gelu 3d", nn.Sequential(nn.Linear(E, 4 * E), nn.GELU(), nn.Linear(4 * E, E)),
      lambda: torch.randn(B, T, E, device=dev))
probe("linear 3d", nn.Linear(E, 4 * E), lambda: torch.randn(B, T, E, device=dev))
probe("linear 2d", nn.Linear(E, 4 * E), lambda: torch.randn(B * T, E, device=dev))
probe("linear 3d 512->1024", nn.Linear(512, 1024), lambda: torch.randn(B, 201, 512, device=dev))
conv = nn.Sequential(nn.Conv2d(1, 32, (2, 3), padding=(1, 1)), nn.BatchNorm2d(32), nn.SELU(),
                     nn.Conv2d(32, 32, (2, 3), padding=(0, 1)))
probe("conv nchw", conv, lambda: torch.randn(B, 1, 23, 21490, device=dev))
conv2 = nn.Sequential(nn.Conv2d(1, 32, (2, 3), padding=(1, 1)), nn.BatchNorm2d(32), nn.SELU(),
                      nn.Conv2d(32, 32, (2, 3), padding=(0, 1))).to(memory_format=torch.channels_last)
probe("conv nhwc", conv2, lambda: torch.randn(B, 1, 23, 21490, device=dev).contiguous(
    memory_format=torch.channels_last))


import sys
if len(sys.argv) > 1:
    import torch.nn.functional as F

    class BiasAfter(nn.Module):
        def __init__(self, act):
            super().__init__()
            self.lin = nn.Linear(E, 4 * E, bias=False)
            self.b = nn.Parameter(torch.randn(4 * E) * 0.1)
            self.act = act

        def forward(self, x):
            return self.act(self.lin(x) + self.b)

    class Scale(nn.Module):
        def forward(self, x):
            return x * 2.0

    mk = lambda: torch.randn(B, T, E, device=dev)
    probe("V-relu", nn.Sequential(nn.Linear(E, 4 * E), nn.ReLU()), mk)
    probe("V-scale", nn.Sequential(nn.Linear(E, 4 * E), Scale()), mk)
    probe("V-gelu-only", nn.Sequential(nn.Linear(E, 4 * E), nn.GELU()), mk)
    probe("V-explicit-bias-gelu", BiasAfter(nn.GELU()), mk)
    probe("V-gelu 2d", nn.Sequential(nn.Linear(E, 4 * E), nn.GELU()), lambda: torch.randn(B * T, E, device=dev))
    probe("V-gelu small", nn.Sequential(nn.Linear(E, 4 * E), nn.GELU()), lambda: torch.randn(2, 16, E, device=dev))
    # manual reduction of an in-graph produced tensor
    h = torch.randn(B * T, 4 * E, device=dev)
    gy = torch.randn_like(h)
    out = torch.empty(4 * E, device=dev)
    ref = (gy * 2.0).sum(0)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            out.copy_((gy * 2.0).sum(0))
    torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_((gy * 2.0).sum(0))
    for r in range(3):
        out.zero_(); g.replay(); torch.cuda.synchronize()
        print("manual mul+sum replay", r, float((out - ref).norm() / ref.norm()), flush=True)
    with torch.cuda.graph(g2 := torch.cuda.CUDAGraph()):
        out.copy_(F.gelu(h).sum(0))
    ref2 = F.gelu(h).sum(0)
    for r in range(3):
        out.zero_(); g2.replay(); torch.cuda.synchronize()
        print("manual gelu+sum replay", r, float((out - ref2).norm() / ref2.norm()), flush=True)
