"""csrc/lgemm.hip against torch (hipBLASLt F.linear / matmul, plus the torch GELU / cast / add launches the fused
epilogues replace) at the detector head's GEMM shapes, fp16. Operands rotate over 4 copies; per shape the median of
7 rounds of a captured HIP graph of 50 calls (kernel time plus the in-graph launch gap). One JSON line per shape.

  python tools/bench_lgemm.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from radhip import _lib, ops  # noqa: E402

DT = torch.float16
# name, M, N, K, kind ("lin": F.linear with bias, "mm": no bias, "gelu": linear + GELU, "f32in": fp32 A cast first)
CASES = [("in_proj", 1608, 576, 144, "mm"), ("x_proj", 3216, 41, 288, "mm"), ("dt_proj", 3216, 288, 9, "mm"),
         ("out_proj", 1608, 144, 288, "mm"), ("ffn1_gelu", 1608, 576, 144, "gelu"), ("ffn2", 1608, 144, 576, "lin"),
         ("wavlm_proj", 1608, 144, 1024, "lin"), ("fusion_proj", 1608, 144, 288, "lin"),
         ("d_wavlm_proj", 1608, 1024, 144, "mm"), ("d_in_proj", 1608, 144, 576, "mm"), ("d_x_proj", 3216, 288, 41, "mm"),
         ("d_dt_proj", 3216, 9, 288, "mm"), ("d_out_proj", 1608, 288, 144, "mm"), ("d_ffn1", 1608, 144, 576, "mm"),
         ("B32_in_proj", 6432, 576, 144, "mm"), ("B32_x_proj", 12864, 41, 288, "mm"), ("B32_ffn2", 6432, 144, 576, "lin")]


def timeit(fns, rounds=7, reps=50):
    """per-call time of each variant from a captured HIP graph of `reps` calls (no host launch cost)"""
    graphs = {}
    for k, f in fns.items():
        f(0)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(2):
                f(i)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(reps):
                f(i)
        graphs[k] = g
    out = {k: [] for k in fns}
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, g in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[k].append(e0.elapsed_time(e1) / reps * 1e3)
    return {k: round(sorted(v)[len(v) // 2], 2) for k, v in out.items()}


def main():
    torch.manual_seed(0)
    for name, M, N, K, kind in CASES:
        sets = []
        for _ in range(4):
            a = torch.randn(M, K, device="cuda").to(DT)
            w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(DT)
            b = (0.1 * torch.randn(N, device="cuda")).to(DT)
            sets.append((a, w, b))
        bias = kind in ("lin", "gelu")

        def torch_fn(i):
            a, w, b = sets[i % 4]
            y = F.linear(a, w, b if bias else None)
            return F.gelu(y) if kind == "gelu" else y

        def lg_fn(i):
            a, w, b = sets[i % 4]
            return ops.lgemm(a, w, b if bias else None,
                             epilogue=_lib.EPI_BIAS_GELU if kind == "gelu" else _lib.EPI_BIAS)
        a, w, b = sets[0]
        ref = F.linear(a.float(), w.float(), b.float() if bias else None)
        got = lg_fn(0)
        got = got[0] if isinstance(got, tuple) else got
        err = float((got.float() - ref).abs().max() / ref.abs().max())
        t = timeit({"torch": torch_fn, "lgemm": lg_fn})
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "kind": kind, "err": round(err, 5), **t}), flush=True)


if __name__ == "__main__":
    main()
