import torch
dev = "cuda"
torch.manual_seed(0)
def trial(shape, dim, between):
    x = torch.randn(*shape, device=dev)
    ref = x.sum(dim)
    out = torch.empty_like(ref)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2): out.copy_(x.sum(dim))
    torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_(x.sum(dim))
    if between == "allocfree":
        junk = [torch.full((1 << k,), float("nan"), device=dev) for k in range(10, 26)]
        del junk
    elif between == "alloc":
        keep = [torch.full((1 << k,), float("nan"), device=dev) for k in range(10, 26)]
    out.zero_()
    g.replay(); torch.cuda.synchronize()
    err = float((out - ref).abs().max() / ref.abs().max())
    print(f"shape={shape} dim={dim} between={between}: rel err {err:.2e}", flush=True)
for between in ["none", "alloc", "allocfree"]:
    for shape, dim in [((1608, 576), 0), ((804, 1024), 0), ((4, 32, 24, 21490), (0, 2, 3)), ((1608, 144), 0)]:
        trial(shape, dim, between)
