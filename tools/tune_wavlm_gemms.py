"""Tune hipBLASLt / rocBLAS solutions (PyTorch TunableOp) for the WavLM encoder layer's GEMMs only, at the window's
pass shapes (M = 8 * 201 adversarial, 32 * 201 clean), in the call forms radhip/wavlm_fused.py uses:
F.linear with bias for the forward (q/k/v with the 16 LoRA columns, out_proj, FFN1, FFN2) and torch.mm for the
input gradients. Writes the table named by --out (to load with PYTORCH_TUNABLEOP_ENABLED=1 and tuning off; the
product does not ship one: the tuned solutions gained 2 % on these GEMMs).

Tune only these shapes, never the whole step: with tuning on over a training step, TunableOp runs every rocBLAS
solution that rocBLAS accepts for the head's n = 1 strided-batched GEMM (tn_201_1_144_B_32, the attention-pooling
bmm of the clean pass's backward) and one of them faults the GPU (gpurun_out/tune3).

  python tools/tune_wavlm_gemms.py --out robust-audio-deepfake-evolution_amd/radhip/tuned/gfx950_wavlm.csv
"""
import argparse
import os

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.path.abspath(a.out))
    tun.set_max_tuning_duration(40)
    tun.set_numerical_check_tolerances(True, 0.05, 0.02)   # reject any solution whose output is off
    dev = "cuda"
    E = 1024
    bf = torch.bfloat16
    wext = torch.randn(3 * E, E + 16, device=dev).to(bf)
    bqkv = torch.randn(3 * E, device=dev).to(bf)
    wo, w1, w2 = (torch.randn(r, c, device=dev).to(bf) * 0.02 for r, c in ((E, E), (4 * E, E), (E, 4 * E)))
    bo, b1, b2 = (torch.randn(n, device=dev).to(bf) for n in (E, 4 * E, E))
    for B in (8, 32):
        M = B * 201
        x1 = torch.randn(M, E + 16, device=dev).to(bf)
        x = torch.randn(M, E, device=dev).to(bf)
        u = torch.randn(M, 4 * E, device=dev).to(bf)
        q = torch.randn(M, 3 * E, device=dev).to(bf)
        for name, fn in [("qkv", lambda: F.linear(x1, wext, bqkv)), ("out", lambda: F.linear(x, wo, bo)),
                         ("ffn1", lambda: F.linear(x, w1, b1)), ("ffn2", lambda: F.linear(u, w2, b2)),
                         ("ffn2_dgrad", lambda: torch.mm(x, w2)), ("ffn1_dgrad", lambda: torch.mm(u, w1)),
                         ("out_dgrad", lambda: torch.mm(x, wo)), ("qkv_dgrad", lambda: torch.mm(q, wext))]:
            fn()
            torch.cuda.synchronize()
            print(f"B={B} {name} tuned", flush=True)
    # torch 2.10 has no tunable.write_file(): the table is written when the TunableOp context is destroyed at
    # process exit (the file named by set_filename); list what was tuned here
    for r in tun.get_results():
        print("result", r, flush=True)
    print("will write at exit:", tun.get_filename(), flush=True)


if __name__ == "__main__":
    main()
