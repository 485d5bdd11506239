"""Per-pass wall time and per-queue / per-category busy time of the last window in a rocprofv3 kernel trace of
bench.py: the clean pass (from the window's last pad_mixup to the first FGM attack) and each adversarial chain
link (FGM attack to the next one).

    python tools/pass_split.py gpurun_out/<tag>/kernel_trace.csv.gz [window index from the end, default 1]
"""
import collections
import csv
import gzip
import sys


def cat(n):
    if "Cijk" in n:
        return "gemm"
    if any(k in n for k in ("sconv", "bnselu", "tail_", "b0_", "sincconv", "igemm")):
        return "sinc"
    if "attn" in n:
        return "attn"
    if "wl_" in n:
        return "wl"
    if any(k in n for k in ("scan", "dwconv", "bigate")):
        return "mamba"
    return "rdx-other" if n.startswith("rdx") else "torch"


def main(path):
    rows = list(csv.DictReader(gzip.open(path, "rt")))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    fgm = [i for i, r in enumerate(rows) if "fgm_norm" in r["Kernel_Name"]]
    pad = [i for i, r in enumerate(rows) if "pad_mixup" in r["Kernel_Name"]]
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    last = fgm[len(fgm) - 4 * w:len(fgm) - 4 * (w - 1)]
    p = [i for i in pad if i < last[0]][-1]
    segs = [("clean", p, last[0])] + [(f"adv{j}", last[j], last[j + 1]) for j in range(3)]
    opt = [i for i, r in enumerate(rows) if i > last[-1] and "adam" in r["Kernel_Name"].lower()]
    segs.append(("adv3", last[-1], opt[0] if opt else len(rows)))
    for name, a, b in segs:
        seg = rows[a:b]
        t0, t1 = seg[0]["s"], max(r["e"] for r in seg)
        byq, byc, cnt = collections.defaultdict(float), collections.defaultdict(float), collections.Counter()
        for r in seg:
            d = (r["e"] - r["s"]) / 1e3
            byq[r["Queue_Id"]] += d
            byc[cat(r["Kernel_Name"])] += d
            cnt[cat(r["Kernel_Name"])] += 1
        print(f"{name:6s} wall {(t1 - t0) / 1e3:7.0f} us  kernels {len(seg)}  busy by queue",
              {k: round(v) for k, v in sorted(byq.items())})
        print("       ", {k: (round(v), cnt[k]) for k, v in sorted(byc.items(), key=lambda x: -x[1])})


if __name__ == "__main__":
    main(sys.argv[1])
