"""csrc/pgemm.hip (deep-pipelined 8-wave GEMM) on the WavLM encoder GEMM shapes (M = 1608 / 6432 tokens) against
hipBLASLt and csrc/wgemm.hip, bf16 in, fp32 accumulate, random operands rotated over 6 copies so the weights do
not stay L2-resident between calls (as in the 24-layer pass). Every result is checked against an fp32 torch
reference; prints one JSON line per shape with us / TFLOP/s per variant.

  python tools/bench_pgemm.py [--tiles 3,4,1:4] [--wg 21,5,6] [--B 8,32] [--shapes qkv,ffn1] [--reps 30]
  pgemm variants are TILE[:GROUP_M] (csrc/pgemm.hip tile codes; GROUP_M 0 = column-panel order).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from radhip import _lib  # noqa: E402

EPI = {"bias": 0, "gelu": 1, "gelu_bwd": 2}
SHAPES = (("qkv", 3072, 1024, "bias"), ("out", 1024, 1024, "bias"), ("ffn1", 4096, 1024, "gelu"),
          ("ffn2", 1024, 4096, "bias"), ("d_ffn2", 4096, 1024, "gelu_bwd"), ("d_ffn1", 1024, 4096, "bias"),
          ("d_out", 1024, 1024, "bias"), ("d_qkv", 1024, 3072, "bias"))


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timed(fns, reps):
    for f in fns:
        f()
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fns[i % len(fns)]()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps * 1e3)
    out.sort()
    return out[len(out) // 2]


def gelu_grad(u):
    return 0.5 * (1 + torch.erf(u * 0.7071067811865476)) + u * 0.3989422804014327 * torch.exp(-0.5 * u * u)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="3,4,1,2,6,7,8,9,5")
    ap.add_argument("--wg", default="")
    ap.add_argument("--B", default="8,32")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--no-blas", action="store_true")
    args = ap.parse_args()
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.manual_seed(0)
    for B in [int(b) for b in args.B.split(",")]:
        M = B * 201
        for name, N, K, epi in SHAPES:
            if args.shapes and name not in args.shapes.split(","):
                continue
            sets = []
            for _ in range(6):
                a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
                w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
                bias = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16) if epi != "gelu_bwd" else None
                aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "gelu_bwd" else None
                sets.append((a, w, bias, aux))
            a, w, bias, aux = sets[0]
            ref = a.float() @ w.float().t()
            if bias is not None:
                ref = ref + bias.float()
            if epi == "gelu":
                want = ref.to(torch.bfloat16).float()
                want_v = F.gelu(want).to(torch.bfloat16).float()
            elif epi == "gelu_bwd":
                want = (ref.to(torch.bfloat16).float() * gelu_grad(aux.float())).to(torch.bfloat16).float()
            else:
                want = ref
            fl = 2.0 * M * N * K
            row = {"B": B, "gemm": name, "M": M, "N": N, "K": K, "epilogue": epi}

            if not args.no_blas:
                def blas(s):
                    a_, w_, b_, x_ = s
                    if epi == "bias":
                        return lambda: F.linear(a_, w_, b_)
                    if epi == "gelu":
                        return lambda: F.gelu(F.linear(a_, w_, b_))
                    return lambda: torch.mm(a_, w_.t()) * x_
                t = timed([blas(s) for s in sets], args.reps)
                row["hipblaslt"] = [round(t, 2), round(fl / t / 1e6, 1)]
            outs = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in sets]
            vs = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if epi == "gelu" else None for _ in sets]

            def check_and_time(key, launch):
                rc = launch(0)()
                if rc != 0:
                    row[key] = f"rc {rc}"
                    return
                torch.cuda.synchronize()
                err = float((outs[0].float() - want).abs().max() / want.abs().max())
                if epi == "gelu":
                    err = max(err, float((vs[0].float() - want_v).abs().max() / want_v.abs().max()))
                t = timed([launch(i) for i in range(len(sets))], args.reps)
                row[key] = [round(t, 2), round(fl / t / 1e6, 1), round(err, 5)]

            for tname in [x for x in args.wg.split(",") if x]:
                tile = int(tname)

                def wl(i, tile=tile):
                    a_, w_, b_, x_ = sets[i]
                    return lambda: L.rdx_wgemm_bf16(p(a_), K, p(w_), K, p(outs[i]), N, M, N, K, p(b_), EPI[epi],
                                                    p(x_), N, p(vs[i]), N, tile, st)
                check_and_time(f"wg{tname}", wl)
            for tname in [x for x in args.tiles.split(",") if x]:
                tile, gm = (int(v) for v in tname.split(":")) if ":" in tname else (int(tname), 0)

                def pl(i, tile=tile, gm=gm):
                    a_, w_, b_, x_ = sets[i]
                    return lambda: L.rdx_pgemm_bf16(p(a_), K, p(w_), K, p(outs[i]), N, M, N, K, p(b_), EPI[epi],
                                                    p(x_), N, p(vs[i]), N, tile, gm, st)
                check_and_time(f"pg{tname}", pl)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
