"""Per-kernel summary of the last N iterations of a rocprofv3 --kernel-trace CSV, an iteration delimited by the
launches of a marker kernel (e.g. rdx::x3::fe_conv0_kernel, once per scoring batch): warm-up work (MIOpen find,
first-use weight preparation) falls outside the window.

  python tools/trace_tail.py kernel_trace.csv --marker fe_conv0_kernel --iters 4 [--top 40]
"""
import argparse
import csv
import gzip
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", required=True)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    with op(a.trace, "rt") as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(f)]
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < a.iters:
        raise SystemExit(f"only {len(marks)} marker launches")
    lo = marks[-a.iters]
    win = rows[lo:]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[n][0] += 1
        agg[n][1] += e - s
    busy = sum(v[1] for v in agg.values())
    wall = win[-1][1] - win[0][0]
    print(f"last {a.iters} iterations: {len(win)} launches ({len(win) / a.iters:.0f} per iteration), kernel time "
          f"{busy / 1e6 / a.iters:.3f} ms per iteration, wall {wall / 1e6 / a.iters:.3f} ms per iteration "
          f"(GPU busy {100 * busy / wall:.1f} %)")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e6 / a.iters:8.3f} ms/it {c / a.iters:6.1f} x {t / c / 1e3:9.2f} us {100 * t / busy:5.1f}%  {n[:100]}")


if __name__ == "__main__":
    main()
