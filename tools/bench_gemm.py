"""The WavLM layer GEMMs at the Phase-6 shapes: hand-written MFMA kernel (radhip.ops.gemm, csrc/gemm.hip) vs
hipBLASLt (torch F.linear), bf16 in / fp32 accumulate, same random operands; prints us and TFLOP/s.

  python tools/bench_gemm.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402

from radhip.ops import gemm  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
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
    rows = []
    for B in (8, 32):
        M = B * 201
        for name, N, K in (("qkv", 3072, 1040), ("out_proj", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096),
                           ("dx1", 1040, 3072), ("dffn2", 4096, 1024), ("dffn1", 1024, 4096)):
            a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
            bias = torch.randn(N, device="cuda").to(torch.bfloat16)
            t_ours = timed(lambda: gemm(a, b, bias))
            t_blas = timed(lambda: torch.nn.functional.linear(a, b, bias))
            fl = 2.0 * M * N * K
            rows.append({"B": B, "gemm": name, "M": M, "N": N, "K": K, "ours_us": round(t_ours, 1),
                         "hipblaslt_us": round(t_blas, 1), "ours_tflops": round(fl / t_ours / 1e6, 1),
                         "hipblaslt_tflops": round(fl / t_blas / 1e6, 1)})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
