"""Do two captured HIP graphs replayed on two streams run concurrently on this ROCm? Graph A is HBM-bound
(SincNet-sized bf16 copies), graph B a latency-bound chain of small GEMMs (WavLM-layer-sized at B = 8). Times A
alone, B alone, A then B on one stream, and A || B on two streams (and one graph holding both as parallel
branches, the way the model's SincNet branch is captured today).

  python tools/graph_concurrency.py
"""
import json

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 3)


def main():
    dev = "cuda"
    a_src = torch.randn(8 * 24 * 21490 * 32 // 2, device=dev).to(torch.bfloat16)
    a_dst = torch.empty_like(a_src)
    x = torch.randn(1608, 1024, device=dev).to(torch.bfloat16)
    ws = [torch.randn(1024, 1024, device=dev).to(torch.bfloat16) * 0.03 for _ in range(4)]

    def work_a():
        for _ in range(20):
            a_dst.copy_(a_src)

    def work_b():
        h = x
        for _ in range(60):
            for w in ws:
                h = torch.mm(h, w)
        return h

    s_main = torch.cuda.Stream()
    s_side = torch.cuda.Stream()
    ga, gb, gab = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(s_main):
        work_a(); work_b()
        torch.cuda.synchronize()
        with torch.cuda.graph(ga):
            work_a()
        with torch.cuda.graph(gb):
            work_b()
        with torch.cuda.graph(gab):
            cur = torch.cuda.current_stream()
            s_side.wait_stream(cur)
            with torch.cuda.stream(s_side):
                work_a()
            work_b()
            cur.wait_stream(s_side)
    torch.cuda.synchronize()
    main_s = torch.cuda.current_stream()

    def two_streams():
        s_side.wait_stream(main_s)
        with torch.cuda.stream(s_side):
            ga.replay()
        gb.replay()
        main_s.wait_stream(s_side)

    def eager_two():
        s_side.wait_stream(main_s)
        with torch.cuda.stream(s_side):
            work_a()
        work_b()
        main_s.wait_stream(s_side)

    gb2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s_main):
        with torch.cuda.graph(gb2):
            work_b()
    torch.cuda.synchronize()
    res_bb = {}
    for name, side in [("pool", s_side), ("hiprio", torch.cuda.Stream(priority=-1)), ("pool2", torch.cuda.Stream()),
                       ("pool3", torch.cuda.Stream())]:
        def bb(side=side):
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                gb2.replay()
            gb.replay()
            main_s.wait_stream(side)
        res_bb["B_par_B_" + name] = timed(bb)
    res_bb["B_then_B"] = timed(lambda: (gb.replay(), gb2.replay()))
    print(json.dumps(res_bb), flush=True)
    # A on a CU-masked stream (hipExtStreamCreateWithCUMask), B on the main stream
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    for ncu in (64, 128, 192):
        mask = (ctypes.c_uint32 * 8)()
        for i in range(ncu):
            mask[i // 32] |= (1 << (i % 32))
        sp = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(sp), ctypes.c_uint32(8), mask)
        if rc != 0:
            print(json.dumps({"cumask_rc": rc}), flush=True)
            break
        ms = torch.cuda.ExternalStream(sp.value)

        def mab(ms=ms):
            ms.wait_stream(main_s)
            with torch.cuda.stream(ms):
                ga.replay()
            gb.replay()
            main_s.wait_stream(ms)

        def ma(ms=ms):
            with torch.cuda.stream(ms):
                ga.replay()
            main_s.wait_stream(ms)
        res_bb[f"A_on_{ncu}cu"] = timed(ma)
        res_bb[f"A{ncu}cu_par_B"] = timed(mab)
    print(json.dumps(res_bb), flush=True)
    out = {"eager_A": timed(work_a), "eager_B": timed(work_b), "eager_A_then_B": timed(lambda: (work_a(), work_b())),
           "eager_two_streams": timed(eager_two), "A": timed(ga.replay), "B": timed(gb.replay), "A_then_B": timed(lambda: (ga.replay(), gb.replay())),
           "A_par_B_two_streams": timed(two_streams), "one_graph_two_branches": timed(gab.replay)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
