"""csrc/hgemm.hip (8-wave ping-pong GEMM) on the WavLM encoder GEMM shapes (M = 1608 / 6432 tokens) against
hipBLASLt, csrc/wgemm.hip and csrc/pgemm.hip, bf16 or fp16 in, fp32 accumulate, random operands rotated over 6
copies so the weights do not stay L2-resident between calls (as in the 24-layer pass). Every result is checked
against an fp32 torch reference; one JSON line per shape with [us, TFLOP/s, rel err] per variant. Variants are
timed in interleaved rounds in one process (cdna_hip_programming.md rule 24); the median round is reported.

  python tools/bench_hgemm.py [--hg 0,2:1:0,4:2] [--wg 5,6] [--pg 4:4] [--B 8,32] [--shapes qkv,ffn1] [--f16]
  hgemm variants are TILE[:SPLITS[:GROUP_M]] (csrc/hgemm.hip tile codes).
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

from radhip import _lib, ops  # noqa: E402

EPI = {"bias": 0, "gelu": 1, "gelu_bwd": 2}
SHAPES = (("qkv", 3072, 1024, "bias"), ("out", 1024, 1024, "bias"), ("ffn1", 4096, 1024, "gelu"),
          ("ffn2", 1024, 4096, "bias"), ("d_ffn2", 4096, 1024, "gelu_bwd"), ("d_ffn1", 1024, 4096, "bias"),
          ("d_out", 1024, 1024, "bias"), ("d_qkv", 1024, 3072, "bias"))


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def gelu_grad(u):
    return 0.5 * (1 + torch.erf(u * 0.7071067811865476)) + u * 0.3989422804014327 * torch.exp(-0.5 * u * u)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hg", default="0,1,2,3,4,5")
    ap.add_argument("--wg", default="")
    ap.add_argument("--pg", default="")
    ap.add_argument("--B", default="8,32")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--f16", action="store_true")
    args = ap.parse_args()
    dt = torch.float16 if args.f16 else torch.bfloat16
    L = _lib.lib16() if args.f16 else _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.manual_seed(0)
    for B in [int(b) for b in args.B.split(",")]:
        M = B * 201
        for name, N, K, epi in SHAPES:
            if args.shapes and name not in args.shapes.split(","):
                continue
            sets = []
            for _ in range(6):
                a = torch.randn(M, K, device="cuda").to(dt)
                w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
                bias = (0.1 * torch.randn(N, device="cuda")).to(dt) if epi != "gelu_bwd" else None
                aux = torch.randn(M, N, device="cuda").to(dt) if epi == "gelu_bwd" else None
                sets.append((a, w, bias, aux))
            a, w, bias, aux = sets[0]
            ref = a.float() @ w.float().t()
            if bias is not None:
                ref = ref + bias.float()
            if epi == "gelu":
                want = ref.to(dt).float()
                want_v = F.gelu(want).to(dt).float()
            elif epi == "gelu_bwd":
                want = (ref.to(dt).float() * gelu_grad(aux.float())).to(dt).float()
            else:
                want = ref
            fl = 2.0 * M * N * K
            row = {"B": B, "gemm": name, "M": M, "N": N, "K": K, "epilogue": epi, "dtype": str(dt)[6:]}
            outs = [torch.empty(M, N, device="cuda", dtype=dt) for _ in sets]
            vs = [torch.empty(M, N, device="cuda", dtype=dt) if epi == "gelu" else None for _ in sets]
            variants = {}

            if not args.no_blas:
                def blas(i):
                    a_, w_, b_, x_ = sets[i]
                    if epi == "bias":
                        return lambda: F.linear(a_, w_, b_)
                    if epi == "gelu":
                        return lambda: F.gelu(F.linear(a_, w_, b_))
                    return lambda: torch.mm(a_, w_.t()) * x_
                variants["hipblaslt"] = [blas(i) for i in range(len(sets))]

            def add(key, launch):
                rc = launch(0)()
                if rc != 0:
                    row[key] = f"rc {rc}"
                    return
                torch.cuda.synchronize()
                err = float((outs[0].float() - want).abs().max() / want.abs().max())
                if epi == "gelu":
                    err = max(err, float((vs[0].float() - want_v).abs().max() / want_v.abs().max()))
                row[key + "_err"] = round(err, 5)
                variants[key] = [launch(i) for i in range(len(sets))]

            for tname in [x for x in args.wg.split(",") if x]:
                tile = int(tname)

                def wl(i, tile=tile):
                    a_, w_, b_, x_ = sets[i]
                    return lambda: L.rdx_wgemm_bf16(p(a_), K, p(w_), K, p(outs[i]), N, M, N, K, p(b_), EPI[epi],
                                                    p(x_), N, p(vs[i]), N, tile, st)
                add(f"wg{tname}", wl)
            for tname in [x for x in args.pg.split(",") if x]:
                tile, gm = (int(v) for v in tname.split(":")) if ":" in tname else (int(tname), 0)

                def pl(i, tile=tile, gm=gm):
                    a_, w_, b_, x_ = sets[i]
                    return lambda: L.rdx_pgemm_bf16(p(a_), K, p(w_), K, p(outs[i]), N, M, N, K, p(b_), EPI[epi],
                                                    p(x_), N, p(vs[i]), N, tile, gm, st)
                add(f"pg{tname}", pl)
            for tname in [x for x in args.hg.split(",") if x]:
                parts = [int(v) for v in tname.split(":")]
                tile, splits, gm = (parts + [1, 0][len(parts) - 1:])[:3]
                ws = cnt = None
                nws = ncnt = 0
                if splits != 1:
                    nws = int(L.rdx_hgemm_ws_bytes(M, N, tile, splits) if splits > 1
                              else L.rdx_hgemm_sk_ws_bytes(M, N, K, tile))
                    ncnt = int(L.rdx_hgemm_counters(M, N, tile))
                    if nws <= 0:
                        row[f"hg{tname}"] = "no split geometry"
                        continue
                    ws = torch.empty(nws, device="cuda", dtype=torch.uint8)
                    cnt = torch.zeros(ncnt, device="cuda", dtype=torch.int32)

                def hl(i, tile=tile, splits=splits, gm=gm, ws=ws, cnt=cnt, nws=nws, ncnt=ncnt):
                    a_, w_, b_, x_ = sets[i]
                    return lambda: L.rdx_hgemm(p(a_), K, p(w_), K, p(outs[i]), N, M, N, K, p(b_), EPI[epi], p(x_), N,
                                               p(vs[i]), N, tile, splits, gm, p(ws), nws, p(cnt), ncnt, st)
                add(f"hg{tname}", hl)

            # interleaved rounds: every variant once per round, median over rounds
            times = {k: [] for k in variants}
            for fns in variants.values():
                for f in fns:
                    f()
            torch.cuda.synchronize()
            for _ in range(args.rounds):
                for k, fns in variants.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(args.reps):
                        fns[i % len(fns)]()
                    e1.record()
                    torch.cuda.synchronize()
                    times[k].append(e0.elapsed_time(e1) / args.reps * 1e3)
            for k, ts in times.items():
                ts.sort()
                t = ts[len(ts) // 2]
                row[k] = [round(t, 2), round(fl / t / 1e6, 1)]
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
