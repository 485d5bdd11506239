"""Micro-benchmark of the WavLM layer's row kernels (csrc/wavlm_layer.hip) at the window's pass shapes
(M = B * 201 rows: B = 8 adversarial, B = 32 clean), with variants that isolate the LoRA / gate / dropout
parts, next to a device copy of the same bytes (the HBM floor at that size) and the hipBLASLt GEMMs of a layer.

  python tools/bench_wl.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from radhip._lib import check, lib  # noqa: E402
from radhip.ops import _p  # noqa: E402


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
    E, H, r = 1024, 16, 8
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for B in (8, 32):
        M = B * 201
        o = {}
        h = torch.randn(M, E, device=dev)
        gm, bt = torch.rand(E, device=dev) + 0.5, torch.randn(E, device=dev) * 0.1
        wg, bg, gc = torch.randn(8, 64, device=dev) * 0.1, torch.randn(8, device=dev) * 0.1, torch.rand(H, device=dev)
        aq, av = ((torch.randn(r, E, device=dev) * 0.05).to(torch.bfloat16),
                  (torch.randn(r, E, device=dev) * 0.05).to(torch.bfloat16))   # 16-bit lora_A (the kernels' input)
        seed = torch.tensor([1234], dtype=torch.int64, device=dev)
        x1 = torch.empty(M, E + 16, device=dev, dtype=torch.bfloat16)
        gate = torch.empty(M, H, device=dev)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)

        def ln1(lora, p, sd=True):
            check(lib().rdx_wl_ln1_fwd(_p(h), _p(gm), _p(bt), 1e-5, _p(wg), _p(bg), _p(gc), _p(aq) if lora else None,
                                       _p(av) if lora else None, 8, _p(seed) if sd else None, 11, 12, p, _p(x1),
                                       E + 16, _p(gate), _p(mean), _p(rstd), M, E, st), "ln1")
        o["copy_h_fp32"] = timed(lambda: h.clone())
        o["ln1_fwd_lora_p0.1"] = timed(lambda: ln1(True, 0.1))
        o["ln1_fwd_lora_p0"] = timed(lambda: ln1(True, 0.0, False))
        o["ln1_fwd_nolora"] = timed(lambda: ln1(False, 0.0, False))
        delta = torch.randn(M, E, device=dev).to(torch.bfloat16)
        h2 = torch.empty(M, E, device=dev)
        x2 = torch.empty(M, E, device=dev, dtype=torch.bfloat16)
        o["add_ln_fwd_p0.1"] = timed(lambda: check(lib().rdx_wl_add_ln_fwd(
            _p(h), _p(delta), _p(seed), 3, 0.1, _p(h2), _p(gm), _p(bt), 1e-5, _p(x2), _p(mean), _p(rstd), M, E, st), "x"))
        o["add_ln_fwd_p0"] = timed(lambda: check(lib().rdx_wl_add_ln_fwd(
            _p(h), _p(delta), None, 3, 0.0, _p(h2), _p(gm), _p(bt), 1e-5, _p(x2), _p(mean), _p(rstd), M, E, st), "x"))
        dx1 = torch.randn(M, E + 16, device=dev).to(torch.bfloat16)
        dgate = torch.randn(M, H, device=dev)
        dres = torch.randn(M, E, device=dev)
        dh = torch.empty(M, E, device=dev)

        def ln1b(lora, p, sd=True):
            check(lib().rdx_wl_ln1_bwd(_p(dx1), E + 16, _p(dgate), _p(h), _p(mean), _p(rstd), _p(gm), _p(bt), _p(wg),
                                       _p(bg), _p(gc), _p(aq) if lora else None, _p(av) if lora else None, 8,
                                       _p(seed) if sd else None, 11, 12, p, _p(dres), _p(dh), None, M, E, st), "ln1b")
        o["ln1_bwd_lora_p0.1"] = timed(lambda: ln1b(True, 0.1))
        o["ln1_bwd_lora_p0"] = timed(lambda: ln1b(True, 0.0, False))
        o["ln1_bwd_nolora"] = timed(lambda: ln1b(False, 0.0, False))
        o["ln_bwd"] = timed(lambda: check(lib().rdx_wl_ln_bwd(
            _p(dx1), E + 16, _p(h), _p(mean), _p(rstd), _p(gm), _p(dres), _p(dh), _p(seed), 3, 0.1, _p(x2), M, E, st),
            "lnb"))
        dqkv = torch.randn(M, 3 * E, device=dev).to(torch.bfloat16)
        gs = [torch.zeros(r, E, device=dev), torch.zeros(E, r, device=dev), torch.zeros(r, E, device=dev),
              torch.zeros(E, r, device=dev)]
        o["lora_grad_p0.1"] = timed(lambda: check(lib().rdx_wl_lora_grad(
            _p(dqkv), 3 * E, _p(x1), E + 16, _p(dx1), E + 16, _p(seed), 11, 12, 0.1, 4.0, _p(gs[0]), _p(gs[1]),
            _p(gs[2]), _p(gs[3]), M, E, r, st), "lg"))
        u = torch.randn(M, 4 * E, device=dev).to(torch.bfloat16)
        v = torch.empty_like(u)
        o["gelu_fwd"] = timed(lambda: check(lib().rdx_wl_gelu(0, _p(u), None, _p(v), u.numel(), st), "g"))
        o["gelu_bwd"] = timed(lambda: check(lib().rdx_wl_gelu(1, _p(u), _p(u), _p(v), u.numel(), st), "g"))
        o["copy_u_bf16"] = timed(lambda: u.clone())
        # the gated attention forward (C ABI, p = 0.1 with the keep-mask words the fused backward reads)
        from radhip.ops import attn_keep_mask
        qkv = torch.randn(M, 3 * E, device=dev).to(torch.bfloat16)
        ob = torch.empty(M, E, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B, H, 201, device=dev)
        rel = torch.randn(H, 2 * 201 - 1, device=dev) * 0.1
        km = attn_keep_mask(B, 201, H, 0.1, dev)

        def attn():
            check(lib().rdx_attn_fwd(_p(qkv), 3 * E, ctypes.c_void_p(qkv.data_ptr() + 2 * E), 3 * E,
                                     ctypes.c_void_p(qkv.data_ptr() + 4 * E), 3 * E, _p(gate), _p(rel), _p(seed), 0,
                                     0.1, 0.125, _p(ob), E, _p(lse), _p(km) if km is not None else None, B, 201, H, 64,
                                     st), "attn_fwd")
        o["attn_fwd"] = timed(attn)
        # the layer's hipBLASLt GEMMs (forward and input gradients)
        wext = torch.randn(3 * E, E + 16, device=dev).to(torch.bfloat16)
        bq = torch.randn(3 * E, device=dev).to(torch.bfloat16)
        wo, w1, w2 = (torch.randn(a, b, device=dev).to(torch.bfloat16) for a, b in ((E, E), (4 * E, E), (E, 4 * E)))
        b1, b2 = torch.randn(4 * E, device=dev).to(torch.bfloat16), torch.randn(E, device=dev).to(torch.bfloat16)
        xa = torch.randn(M, E, device=dev).to(torch.bfloat16)
        o["gemm_qkv"] = timed(lambda: F.linear(x1, wext, bq))
        o["gemm_out"] = timed(lambda: F.linear(xa, wo, b2))
        o["gemm_ffn1"] = timed(lambda: F.linear(xa, w1, b1))
        o["gemm_ffn2"] = timed(lambda: F.linear(u, w2, b2))
        o["gemm_ffn2_dgrad"] = timed(lambda: torch.mm(xa, w2))
        o["gemm_ffn1_dgrad"] = timed(lambda: torch.mm(u, w1))
        o["gemm_out_dgrad"] = timed(lambda: torch.mm(xa, wo))
        o["gemm_qkv_dgrad"] = timed(lambda: torch.mm(dqkv, wext))
        res[f"B{B}"] = o
        print(json.dumps({f"B{B}": o}), flush=True)


if __name__ == "__main__":
    main()
