"""Standalone timings of the split-precision GEMM (rdx_hgemm_x3) per eval shape and tile, and of the other x3
kernels, at the scoring batch (32 x 201 tokens). One JSON line per case: shape, tile / splits / group_m, us, and the
effective rate (3 bf16 MFMA products per fp32 flop counted: TFLOP/s of bf16 work, against the 2.5 PF dense peak).

    python tools/bench_x3.py [--batch 32] [--iters 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import torch  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from radhip import _lib, wavlm_x3
    dev = torch.device("cuda", 0)
    M = a.batch * 201
    shapes = {"qkv": (3072, 1024), "out": (1024, 1024), "ffn1": (4096, 1024), "ffn2": (1024, 4096)}
    cands = [(0, 1, 4), (1, 1, 4), (2, 1, 4), (4, 1, 4), (5, 1, 4), (2, 2, 4), (4, 2, 4), (4, 3, 4), (0, 1, 0),
             (1, 1, 0), (2, 1, 0)]
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        ah, al = wavlm_x3.planes(x)
        wp = wavlm_x3.planes(w)
        bias = torch.zeros(N, device=dev)
        epi = _lib.EPI_F32_GELU_SPLIT if name == "ffn1" else _lib.EPI_F32
        for c in cands:
            wavlm_x3.X3_POLICY[name] = c
            try:
                us = timeit(lambda: wavlm_x3.gemm(ah, al, wp, bias, epilogue=epi, pol=name), a.iters)
            except RuntimeError as ex:
                print(json.dumps({"shape": name, "cand": c, "error": str(ex)[:80]}), flush=True)
                continue
            tf = 3 * 2.0 * M * N * K / us / 1e6
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "tile": c[0], "splits": c[1], "group_m": c[2],
                              "us": round(us, 1), "bf16_tflops": round(tf, 1), "frac_2p5": round(tf / 2500, 3)}),
                  flush=True)
    # fp32 reference: hipBLASLt fp32 GEMMs of the same shapes
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        us = timeit(lambda: x @ w.t(), a.iters)
        print(json.dumps({"shape": name, "torch_fp32_us": round(us, 1),
                          "fp32_tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
