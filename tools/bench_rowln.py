"""Micro-benchmark of the row LayerNorm backward (csrc/rowln.hip) at the head's shapes: M = B * 201 rows
(B = 8 adversarial, 32 clean), C = 144 (PN-BiMamba norms, norm_f) and 1024 (ln_wavlm), x fp32 / bf16.
RADHIP_LIB selects a variant library for A/B.

  python tools/bench_rowln.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402

from radhip._lib import check, lib  # noqa: E402
from radhip.ops import _p  # noqa: E402

F32, BF16 = 0, 1


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 2)


def main():
    dev = "cuda"
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {"lib": os.path.basename(os.environ.get("RADHIP_LIB", "libradhip.so"))}
    for B in (8, 32):
        M = B * 201
        for C in (144, 1024):
            for xdt in (torch.float32, torch.bfloat16):
                x = torch.randn(M, C, device=dev).to(xdt)
                dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
                g = torch.rand(C, device=dev) + 0.5
                mean = x.float().mean(1)
                rstd = torch.rsqrt(x.float().var(1, unbiased=False) + 1e-5)
                dx = torch.empty_like(x)
                dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
                xc = F32 if xdt == torch.float32 else BF16

                def run():
                    check(lib().rdx_row_ln_bwd(BF16, _p(dy), xc, _p(x), _p(mean), _p(rstd), _p(g), _p(dx), _p(dg),
                                               _p(db), M, C, st), "row_ln_bwd")
                t = timed(run)
                # parity of this variant against torch (fp32)
                dg.zero_(); db.zero_()
                run()
                xr = x.float().requires_grad_()
                y = torch.nn.functional.layer_norm(xr, (C,), g, torch.zeros(C, device=dev), 1e-5)
                y.backward(dy.float())
                err = (dx.float() - xr.grad).abs().max().item() / xr.grad.abs().max().item()
                errg = (dg - (dy.float() * ((x.float() - mean[:, None]) * rstd[:, None])).sum(0)).abs().max().item()
                out[f"B{B}_C{C}_{str(xdt)[6:]}"] = {"us": t, "dx_rel": round(err, 6), "dg_abs": round(errg, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
