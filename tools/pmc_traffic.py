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
       "posconv_bwd": ("posconv_kernel<true>",), "sincnet_b0_bwd": ("b0_bwd_kernel",),
       "sconv_fwd": ("sconv_fwd_kernel",), "sconv_wgrad": ("sconv_wgrad_kernel",)}


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name].append(float(r["Counter_Value"]))
    return {k: (sum(v), len(v)) for k, v in vals.items()}


def main(d):
    res = {}
    for B in (8, 32):
        f = per_kernel(os.path.join(d, f"attn_FETCH_SIZE_{B}.csv"), "FETCH_SIZE")
        w = per_kernel(os.path.join(d, f"attn_WRITE_SIZE_{B}.csv"), "WRITE_SIZE")
        rows = {}
        for k in sorted(set(f) | set(w)):
            if "rdx::" not in k:
                continue
            fs, fn = f.get(k, (0.0, 1))
            ws, wn = w.get(k, (0.0, 1))
            rows[k] = {"fetch_kib": fs / fn, "write_kib": ws / wn, "dispatches": max(fn, wn),
                       "hbm_bytes": 2 * 1024 * fs / fn + 1024 * ws / wn}
        res[f"B{B}"] = {"kernels": rows}
        for op, keys in OPS.items():
            # sconv_fwd_kernel<..., true> is the bench's "sconv_dgrad_bnselu", not "sconv_fwd"
            sel = [v for k, v in rows.items() if any(x in k for x in keys) and not (op == "sconv_fwd" and "true>" in k)]
            tot = sum(v["hbm_bytes"] * v["dispatches"] for v in sel)
            cnt = sum(v["dispatches"] for v in sel)
            # bytes per dispatch of this operation, over all its shapes / template variants
            res[f"B{B}"][op] = (tot, cnt)
    out = {"note": ("HBM bytes per launch from rocprofv3 PMC (FETCH_SIZE x 2 gfx950 correction + WRITE_SIZE, "
                    "KiB -> bytes); per-launch value at the bench's launch mix (see 'mix')")}
    for k in OPS:
        (t32, c32), (t8, c8) = res["B32"][k], res["B8"][k]
        if c32 + c8 == 0:
            continue
        # the window runs every SincNet pass at B = 32 (clean pass + the batched adversarial passes,
        # radhip/window.py); the WavLM kernels keep the 1 x B32 : 4 x B8 mix
        sinc = k.startswith("sconv") or k.startswith("sincnet")
        per = round(t32 / max(c32, 1)) if sinc else round((t32 + 4 * t8) / max(c32 + 4 * c8, 1))
        out[k] = {"hbm_bytes_per_launch": per, "B8": round(t8 / max(c8, 1)), "B32": round(t32 / max(c32, 1)),
                  "mix": "B32 only" if sinc else "(B32 + 4 B8) / 5"}
    out["detail"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
