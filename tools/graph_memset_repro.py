"""Does a captured hipMemsetAsync re-execute on every replay?  And do torch's multi-dim reductions of
an in-graph-produced tensor stay idempotent across replays?"""
import ctypes

import torch

dev = "cuda"
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]

buf = torch.zeros(64, dtype=torch.int32, device=dev)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    st = torch.cuda.current_stream().cuda_stream
    assert hip.hipMemsetAsync(buf.data_ptr(), 0, 256, st) == 0
    buf.add_(1)
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("memset+add replay", r, "buf[0] =", int(buf[0]), "(expect 1)", flush=True)


def red(label, shape, dims):
    x = torch.randn(*shape, device=dev)
    out = torch.empty(x.sum(dims).shape, device=dev)
    ref = (x * 2.0).sum(dims)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            out.copy_((x * 2.0).sum(dims))
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_((x * 2.0).sum(dims))
    errs = []
    for r in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        errs.append(float((out - ref).norm() / ref.norm()))
    print(label, shape, dims, ["%.1e" % e for e in errs], flush=True)


red("3d bias", (4, 402, 576), (0, 1))
red("conv bias", (4, 32, 24, 21490), (0, 2, 3))
red("conv bias nhwc-like", (4, 24, 21490, 32), (0, 1, 2))
red("2d", (1608, 576), 0)
red("big col", (65536, 64), 0)
red("full", (1 << 22,), 0)
