import torch, sys
dev = "cuda"
def run(lib, dtype, shape_in, fout):
    if lib: torch.backends.cuda.preferred_blas_library(lib)
    torch.manual_seed(0)
    lin = torch.nn.Linear(shape_in[-1], fout).to(dev)
    x = torch.randn(*shape_in, device=dev)
    def body():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype is not None, cache_enabled=False):
            y = lin(x)
        (y.float() ** 2).sum().backward()
    lin.zero_grad(); body(); torch.cuda.synchronize()
    ref_b, ref_w = lin.bias.grad.clone(), lin.weight.grad.clone()
    for p in lin.parameters(): p.grad.zero_()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2): body()
    torch.cuda.current_stream().wait_stream(s)
    for p in lin.parameters(): p.grad.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for p in lin.parameters(): p.grad.zero_()
    g.replay(); torch.cuda.synchronize()
    eb = float((lin.bias.grad - ref_b).abs().max() / ref_b.abs().max())
    ew = float((lin.weight.grad - ref_w).abs().max() / ref_w.abs().max())
    print(f"blas={lib} amp={dtype is not None} in={shape_in} out={fout}: rel err bias {eb:.2e} weight {ew:.2e}", flush=True)
for lib in ["cublaslt", "cublas"]:
    for amp in [torch.bfloat16, None]:
        for shp, fo in [((8, 201, 1024), 144), ((8, 201, 144), 576), ((8, 201, 576), 144), ((1608, 144), 1)]:
            try:
                run(lib, amp, shp, fo)
            except Exception as e:
                print("ERR", lib, amp, shp, e)
