"""HBM bytes per launch of the hand-written kernels from the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
tools/gpu_prof.sh, written to profiles/pmc_traffic.json (bench.py reads `hbm_bytes_per_launch` of the
dominant kernel into roofline.traffic).

Counter conventions (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): both counters are in KiB;
on gfx950 FETCH_SIZE reads exactly half the bytes of a wide (16 B per lane) coalesced read, so it is
doubled here (these kernels read with 16-byte loads); WRITE_SIZE is exact for 16-byte
stores and counted as is (the 2-byte output stores are uncalibrated: reported raw).
The bench's launches of these operations are 1 clean pass at 4 x 8 utterances and 4 adversarial passes at 8 per
window, so the per-launch figure is the 1:4 mix of the B = 32 and B = 8 measurements.

  python tools/pmc_traffic.py gpurun_out/prof_r01 > profiles/pmc_traffic.json
"""
import collections
import csv
import json
import os
import sys


# bench.py operation -> the kernels of one launch of it
OPS = {"attn_fwd": ("attn_fwd",), "attn_bwd": ("attn_bwd",), "posconv_fwd": ("posconv_kernel<false>",),
       "posconv_bwd": ("posconv_kernel<true>",), "sincnet_b0_bwd": ("b0_bwd_kernel",)}


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main(d):
    res = {}
    for B in (8, 32):
        f = per_kernel(os.path.join(d, f"attn_FETCH_SIZE_{B}.csv"), "FETCH_SIZE")
        w = per_kernel(os.path.join(d, f"attn_WRITE_SIZE_{B}.csv"), "WRITE_SIZE")
        rows = {k: {"fetch_kib": f.get(k, 0.0), "write_kib": w.get(k, 0.0),
                    "hbm_bytes": 2 * 1024 * f.get(k, 0.0) + 1024 * w.get(k, 0.0)}
                for k in sorted(set(f) | set(w)) if "rdx::" in k}
        res[f"B{B}"] = {"kernels": rows}
        for op, keys in OPS.items():
            res[f"B{B}"][op] = sum(v["hbm_bytes"] for k, v in rows.items() if any(x in k for x in keys))
    out = {"note": ("HBM bytes per launch from rocprofv3 PMC (FETCH_SIZE x 2 gfx950 correction + WRITE_SIZE, "
                    "KiB -> bytes); per-launch value = (B32 + 4 B8) / 5, the bench's launch mix")}
    for k in OPS:
        out[k] = {"hbm_bytes_per_launch": round((res["B32"][k] + 4 * res["B8"][k]) / 5),
                  "B8": round(res["B8"][k]), "B32": round(res["B32"][k])}
    out["detail"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
