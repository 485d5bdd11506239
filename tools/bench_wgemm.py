"""The WavLM encoder GEMMs at the Phase-6 shapes (M = 1608 / 6432 tokens): csrc/wgemm.hip (every tile
configuration, its epilogue fused) against hipBLASLt (torch F.linear / mm + the unfused epilogue), bf16 in,
fp32 accumulate, random operands rotated over 6 copies (weights do not stay L2-resident between calls, as in
the 24-layer pass). Checks each result against an fp32 torch reference and prints us and TFLOP/s per shape.

  python tools/bench_wgemm.py [--tiles 0,1,12x4] [--B 8,32] [--reps 30]   (TxS: tile T split-K S)
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
SHAPES = (("qkv", 3072, 1024, "bias"), ("out_proj", 1024, 1024, "bias"), ("ffn1", 4096, 1024, "gelu"),
          ("ffn2", 1024, 4096, "bias"), ("d_ffn2", 4096, 1024, "gelu_bwd"), ("d_ffn1", 1024, 4096, "bias"),
          ("d_out", 1024, 1024, "bias"), ("d_qkv", 1024, 3072, "bias"))


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timed(fns, reps):
    """fns: one callable per operand copy; median of 5 rounds of reps launches (us per launch)."""
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
    ap.add_argument("--tiles", default="0,1,2,3,4,5")
    ap.add_argument("--B", default="8,32")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    tiles = [t for t in args.tiles.split(",")]
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
                ref_u = ref.to(torch.bfloat16)
                ref_v = F.gelu(ref_u.float()).to(torch.bfloat16)
            elif epi == "gelu_bwd":
                ref = (ref.to(torch.bfloat16).float() * gelu_grad(aux.float())).to(torch.bfloat16)
            fl = 2.0 * M * N * K

            def blas(s):
                a_, w_, b_, x_ = s
                if epi == "bias":
                    return lambda: F.linear(a_, w_, b_)
                if epi == "gelu":
                    return lambda: F.gelu(F.linear(a_, w_, b_))
                return lambda: torch.mm(a_, w_.t()) * x_
            t_blas = timed([blas(s) for s in sets], args.reps)
            row = {"B": B, "gemm": name, "M": M, "N": N, "K": K, "epilogue": epi,
                   "hipblaslt_us": round(t_blas, 2), "hipblaslt_tflops": round(fl / t_blas / 1e6, 1)}
            outs = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in sets]
            vs = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if epi == "gelu" else None for _ in sets]
            for tname in tiles:
                tile, splits = (int(v) for v in tname.split("x")) if "x" in tname else (int(tname), 1)
                if splits > K // 64:
                    continue
                nws = max(int(L.rdx_wgemm_ws_bytes(M, N, tile, splits)), 16)
                ncn = max(int(L.rdx_wgemm_counters(M, N, tile)), 1)
                ws = torch.empty(nws, dtype=torch.uint8, device="cuda")
                cnt = torch.zeros(ncn, dtype=torch.int32, device="cuda")

                def ours(i, tile=tile, splits=splits, ws=ws, cnt=cnt, nws=nws, ncn=ncn):
                    a_, w_, b_, x_ = sets[i]
                    return lambda: L.rdx_wgemm_bf16_ex(p(a_), K, p(w_), K, p(outs[i]), N, M, N, K, p(b_), EPI[epi],
                                                       p(x_), N, p(vs[i]), N, tile, splits, p(ws), nws, p(cnt), ncn,
                                                       st)
                rc = ours(0)()
                if rc != 0:
                    row[f"t{tname}"] = f"rc {rc}"
                    continue
                torch.cuda.synchronize()
                got = outs[0].float()
                want = ref_u.float() if epi == "gelu" else (ref.float() if epi == "gelu_bwd" else ref)
                err = float((got - want).abs().max() / want.abs().max())
                if epi == "gelu":
                    err = max(err, float((vs[0].float() - ref_v.float()).abs().max() / ref_v.float().abs().max()))
                t = timed([ours(i) for i in range(len(sets))], args.reps)
                row[f"t{tname}_us"] = round(t, 2)
                row[f"t{tname}_tflops"] = round(fl / t / 1e6, 1)
                row[f"t{tname}_err"] = float(f"{err:.2e}")
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
