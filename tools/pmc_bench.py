"""HBM bytes per launch of every kernel of a bench.py run, from the two rocprofv3 PMC passes of
tools/gpu_pmc_bench.sh (FETCH_SIZE, WRITE_SIZE over the bench's own launches: warm-up, capture, timed and
kernel-timing replays, i.e. the bench's launch mix), written as profiles/pmc_traffic.json; bench.py reads
`hbm_bytes_per_launch` of its dominant kernel into roofline.traffic.

Counter conventions (MI355X_MICROARCH.md §HBM): both counters count KiB; on gfx950 FETCH_SIZE reads half the bytes
of a wide (16-byte per lane) coalesced read, so it is doubled (the hand-written kernels load with 16-byte loads;
narrower loads make this an overestimate); WRITE_SIZE is counted as is.

  python tools/pmc_bench.py gpurun_out/<tag> > profiles/pmc_traffic.json
"""
import collections
import csv
import gzip
import json
import os
import re
import sys

# bench.py kernel-timing names -> kernel-name patterns of one launch of that operation
OPS = {
    "wgemm": r"wgemm_kernel<", "b0x_bwd": r"b0x_bwd_kernel", "b0x_fwd": r"b0x_fwd_kernel",
    "sconv_fwd": r"sconv_fwd_kernel<\d+, \d+, \d+, false>", "sconv_dgrad_bnselu": r"sconv_fwd_kernel<\d+, \d+, \d+, true>",
    "sconv_wgrad": r"sconv_wgrad_kernel<", "attn_fwd": r"attn_fwd_kernel<", "attn_bwd": r"attn_bwd_fused_kernel<",
    "selective_scan_fwd": r"scan_fwd_seg_kernel<|s2::fwd_chunk_kernel<|s2::carry_kernel<0>|s2::fwd_out_kernel<",
    "selective_scan_bwd": r"[^_]scan_bwd_kernel<|s2::bwd_chunk_kernel<|s2::carry_kernel<1>|s2::bwd_out_kernel<",
    "pgemm": r"pgemm_kernel<", "hgemm": r"hgemm_kernel<", "lgemm": r"lgemm_kernel<", "sincconv_mfma": r"sincconv_mfma_kernel",
    "wgrad_acc": r"wgrad_part_kernel|wgrad_reduce_kernel", "wgrad_many": r"wgrad_part_many_kernel|wgrad_reduce_many_kernel", "posconv_fwd": r"posconv2?_kernel<false>",
    "posconv_bwd": r"posconv2?_kernel<true>", "fe_conv0": r"fe_conv0_kernel", "fe_ln_gelu": r"fe_ln_gelu_kernel", "sincconv_absmaxpool": r"sincconv_absmaxpool_kernel",
    "fe_conv_gemm": r"gemm_nt_kernel|strided_gemm", "layer_wsum_fwd": r"lws_fwd_kernel", "layer_wsum_bwd": r"lws_bwd_kernel",
}


def load(path, counter):
    """dispatch id -> (kernel name, KiB) for one counter."""
    out = {}
    with gzip.open(path, "rt") as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            name, v = r["Kernel_Name"], float(r["Counter_Value"])
            if key in out:
                out[key] = (name, out[key][1] + v)
            else:
                out[key] = (name, v)
    return out


def main(d):
    fetch = load(os.path.join(d, "FETCH_SIZE.csv.gz"), "FETCH_SIZE")
    write = load(os.path.join(d, "WRITE_SIZE.csv.gz"), "WRITE_SIZE")
    res = {"note": "HBM bytes per launch, rocprofv3 PMC over bench.py's own launches (tools/gpu_pmc_bench.sh): "
                   "2 x FETCH_SIZE (gfx950 wide-load correction) + WRITE_SIZE, KiB -> bytes, averaged over every "
                   "launch of the operation's kernels in the run (both passes run the same deterministic bench)"}
    for op, pat in OPS.items():
        rx = re.compile(pat)
        fk = [v for n, v in fetch.values() if rx.search(n)]
        wk = [v for n, v in write.values() if rx.search(n)]
        if not fk or not wk:
            continue
        # wgrad_acc, scan2 and similar two-kernel ops: count launches of the first alternative that occurs
        alts = [re.compile(a) for a in pat.split("|")]
        first = next(a for a in alts if any(a.search(n) for n, _ in fetch.values()))
        nl = max(1, sum(1 for n, _ in fetch.values() if first.search(n)))
        f_b = 2 * 1024 * sum(fk) / nl
        w_b = 1024 * sum(wk) / max(1, sum(1 for n, _ in write.values() if first.search(n)))
        res[op] = {"hbm_bytes_per_launch": round(f_b + w_b), "fetch_bytes_per_launch": round(f_b),
                   "write_bytes_per_launch": round(w_b), "launches": nl}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
