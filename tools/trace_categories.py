"""Per-step category and top-kernel split of a rocprofv3 kernel trace of bench.py (one step = one window of
accumulation_steps micro-batches; the window's 4 micro-batch preparations each launch pad_mixup_kernel).

    python tools/trace_categories.py gpurun_out/<tag>/kernel_trace.csv.gz [--steps 2] [--top 40]
"""
import argparse
import collections
import csv
import gzip
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import categorize  # noqa: E402


def cat(n):
    if n.startswith("igemm") or "naive_conv" in n or "batched_transpose" in n or "SubTensorOp" in n:
        return "conv (MIOpen)"
    return categorize(n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(gzip.open(a.trace, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "pad_mixup" in r["Kernel_Name"]]
    ss = rows[idx[-4 * a.steps]:]
    c = collections.defaultdict(float)
    cn = collections.Counter()
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in ss:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = cat(n)
        c[k] += d
        cn[k] += 1
        s = re.sub(r"\(.*", "", n).replace("void ", "")[:90]
        per[s][0] += 1
        per[s][1] += d
    t0 = int(ss[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in ss)
    S = a.steps
    print(f"# wall {(t1 - t0) / 1e6 / S:.2f} ms/step, busy {sum(c.values()) / 1e3 / S:.2f} ms/step")
    for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
        print(f"{v / 1e3 / S:8.2f} ms/step {cn[k] / S:7.0f} launches  {k}")
    print(f"# top {a.top} kernels (ms/step, launches/step, avg us)")
    for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e3 / S:8.3f} {n / S:7.0f} {t / n:9.1f}  {k}")


if __name__ == "__main__":
    main()
