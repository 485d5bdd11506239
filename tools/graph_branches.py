"""Do parallel branches of a captured HIP graph run concurrently on this ROCm?

Two chains of small (few-workgroup) matmuls, each on its own stream, forked from and joined back to the
capture stream. Prints eager serial / eager two-stream / graph two-stream / graph serial times.

    python tools/graph_branches.py
"""
import json
import time

import torch


def chain(a, n):
    for _ in range(n):
        a = a @ a * 0.5
    return a


def main():
    dev = "cuda"
    n = 200
    a = torch.randn(256, 256, device=dev, dtype=torch.bfloat16) * 0.05
    b = a.clone()
    main_s = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def serial():
        chain(a, n)
        chain(b, n)

    def branched():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            chain(a, n)
        with torch.cuda.stream(s2):
            chain(b, n)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def timeit(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps * 1e3

    res = {"eager_serial_ms": timeit(serial), "eager_branched_ms": timeit(branched)}
    graphs = {}
    for name, fn in (("serial", serial), ("branched", branched)):
        side = torch.cuda.Stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            fn()
        main_s.wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graphs[name] = g
        res[f"graph_{name}_ms"] = timeit(g.replay)
    print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
