"""In-kernel stamps of csrc/pgemm.hip (rdx_pgemm_prof): per workgroup, the shader cycles spent in the prologue
(until stage 0 has landed), the K loop and the epilogue, against the MFMA-bound cycles of its tile, plus the launch
span and the clock from the 100 MHz real-time stamps. Operands are rotated over 6 copies as in the 24-layer pass.

  python tools/prof_pgemm.py [--cases 8:qkv:4:4,32:ffn1:2:4]   (B:gemm:tile:group_m)
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radhip import _lib  # noqa: E402

SHAPES = {"qkv": (3072, 1024), "out": (1024, 1024), "ffn1": (4096, 1024), "ffn2": (1024, 4096),
          "d_qkv": (1024, 3072)}
GEOM = {0: (256, 256), 2: (128, 256), 4: (128, 192), 10: (256, 256), 12: (128, 256), 14: (128, 192),
        20: (256, 256), 22: (128, 256), 24: (128, 192)}


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="8:qkv:4:4,8:qkv:3:4,8:ffn1:2:4,32:qkv:2:4,32:ffn1:2:4,32:ffn2:2:4,32:out:2:4")
    args = ap.parse_args()
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.manual_seed(0)
    for case in args.cases.split(","):
        B, name, tile, gm = case.split(":")
        B, tile, gm = int(B), int(tile), int(gm)
        N, K = SHAPES[name]
        M = B * 201
        BM, BN = GEOM[tile]
        grid = ((M + BM - 1) // BM) * ((N + BN - 1) // BN)
        sets = []
        for _ in range(6):
            a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
            bias = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
            sets.append((a, w, bias, torch.empty(M, N, device="cuda", dtype=torch.bfloat16)))
        prof = torch.zeros(grid, 8, dtype=torch.int64, device="cuda")
        for it in range(13):
            a, w, bias, c = sets[it % 6]
            rc = L.rdx_pgemm_prof(p(a), K, p(w), K, p(c), N, M, N, K, p(bias), tile, gm, p(prof), st)
            if rc != 0:
                raise RuntimeError(f"rdx_pgemm_prof rc {rc}")
        torch.cuda.synchronize()
        ref = sets[12 % 6][0].float() @ sets[12 % 6][1].float().t() + sets[12 % 6][2].float()
        err = float((sets[12 % 6][3].float() - ref).abs().max() / ref.abs().max()) if gm >= 0 and tile < 10 else -1.0
        d = prof.cpu().numpy().astype(np.int64)
        ts0, ts1, ts2, ts3, rt0, rt1 = (d[:, i] for i in range(6))
        span_us = (rt1.max() - rt0.min()) / 100.0
        clk_ghz = float(np.median((ts3 - ts0) / np.maximum(rt1 - rt0, 1) * 0.1))
        mfma_cyc = 2 * (BM // 2 // 16) * (BN // 4 // 16) * 2 * (K // 64) * 16   # per SIMD: 2 waves x MFMAs x 16
        xcc = (d[:, 6] >> 32) & 0xF
        hw = d[:, 6] & 0xFFFFFFFF
        cu = ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4)   # CU_ID | SH/SE bits: a per-XCC CU key
        slots = {}
        for x, c in zip(xcc, cu):
            slots[(int(x), int(c))] = slots.get((int(x), int(c)), 0) + 1
        fl = 2.0 * M * N * K
        row = {"case": case, "M": M, "N": N, "K": K, "tile": [BM, BN], "grid": grid, "err": round(err, 5),
               "span_us": round(float(span_us), 2), "tflops_span": round(fl / span_us / 1e6, 1),
               "clock_ghz": round(clk_ghz, 3),
               "prologue_cyc": [int(np.median(ts1 - ts0)), int(np.max(ts1 - ts0))],
               "loop_cyc": [int(np.median(ts2 - ts1)), int(np.max(ts2 - ts1))],
               "epilogue_cyc": [int(np.median(ts3 - ts2)), int(np.max(ts3 - ts2))],
               "mfma_bound_loop_cyc": mfma_cyc,
               "start_skew_us": round(float(np.percentile(rt0 - rt0.min(), 90)) / 100.0, 2),
               "wg_per_cu_max": max(slots.values()), "cus_used": len(slots)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
