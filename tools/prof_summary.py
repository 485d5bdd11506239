"""Steady-state summary of a rocprofv3 --kernel-trace CSV of `bench.py`.

The bench's warm-up includes MIOpen find-mode benchmarking (naive reference convolutions, >100 ms
each), which swamps rocprof's whole-run stats. This keeps the last `--micro` micro-batches: they are
delimited by `pad_mixup_kernel` launches, which happen once per micro-batch at its start. It prints
per-kernel busy time per micro-batch, the category split, and wall vs busy time.

  python tools/prof_summary.py gpurun_out/prof_r01/kernel_trace.csv.gz --micro 8 > profiles/r01_steady_state.txt
"""
import argparse
import csv
import gzip
import re
from collections import defaultdict


def categorize(name):
    n = name
    if n.startswith("rdx::") or "rdx::" in n[:40] or n.startswith("b0x_"):   # b0x_bwd_kernel: csrc/b0fused.hip
        return "radhip (hand-written HIP)"
    if n.startswith("Cijk_") or "gemm" in n.lower() and "conv" not in n.lower():
        return "GEMM (hipBLASLt/rocBLAS)"
    if "conv" in n.lower() or "Im2" in n or "Col2Im" in n or "batched_transpose" in n or "naive_conv" in n:
        return "conv (MIOpen/CK)"
    if "copy_kernel" in n or "bfloat16_copy" in n or "tofloat32" in n:
        return "dtype casts / copies"
    if "batch_norm" in n:
        return "batch norm"
    if "reduce_kernel" in n:
        return "reductions"
    if "attention" in n.lower() or "fmha" in n.lower() or "softmax" in n.lower():
        return "attention / softmax"
    if "elementwise" in n or "vectorized" in n:
        return "elementwise"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--micro", type=int, default=8)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--accum", type=int, default=4, help="micro-batches per step (with --before)")
    ap.add_argument("--before", default=None,
                    help="end the window at the first launch whose name contains this (bench.py: 'ts_acc_kernel', "
                         "the first clock stamp of the kernel-timing replay, so the window is the timed region)")
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    with op(a.trace, "rt") as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(f)]
    rows.sort()
    if a.before:
        # the timed region precedes the stamped kernel-timing replay; warm-up and capture precede both
        first = next((i for i, r in enumerate(rows) if a.before in r[2]), None)
        if first is None:
            raise SystemExit(f"no launch named {a.before}")
        rows = rows[:first]
    marks = [i for i, r in enumerate(rows) if "pad_mixup_kernel" in r[2]]
    if a.before:
        # the kernel-timing replay's first step stages its micro-batches (their pad_mixup launches) before its
        # first stamped graph: the timed region ends at the first of those
        if len(marks) < a.accum:
            raise SystemExit("too few micro-batch markers")
        rows = rows[:marks[-a.accum]]
        marks = marks[:-a.accum]
    if len(marks) < a.micro + 1:
        raise SystemExit(f"only {len(marks)} micro-batch markers")
    lo = marks[-a.micro - 1] if len(marks) > a.micro else marks[0]
    lo = marks[-a.micro]
    win = rows[lo:]
    t0, t1 = win[0][0], max(r[1] for r in win)
    per = defaultdict(lambda: [0, 0])
    cat = defaultdict(float)
    busy = 0
    for s, e, n in win:
        short = re.sub(r"\(.*", "", n)[:100]
        if "at::native::" in n and len(short) < 40:   # a templated name cut at its first parenthesis
            short = n[:160]
        per[short][0] += 1
        per[short][1] += e - s
        cat[categorize(n)] += e - s
        busy += e - s
    m = a.micro
    # time with at least one kernel running (concurrent branches overlap: the kernel sum can exceed the wall)
    union, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    src = f"the timed region (before the first {a.before})" if a.before else "the end of the trace"
    print(f"# steady-state window: last {m} micro-batches of {src} ({len(win)} kernels, {len(win) / m:.0f}/micro-batch)")
    print(f"# wall {1e-6 * (t1 - t0) / m:.2f} ms/micro-batch, kernel sum {1e-6 * busy / m:.2f} ms/micro-batch, "
          f"GPU busy (any kernel running) {1e-6 * union / m:.2f} ms/micro-batch ({100.0 * union / (t1 - t0):.1f} %)")
    print("# category split (ms per micro-batch)")
    for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
        print(f"{k:32s} {1e-6 * v / m:9.3f}")
    print(f"# top {a.top} kernels (ms per micro-batch, launches per micro-batch, avg us)")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{1e-6 * t / m:9.3f} {c / m:8.1f} {1e-3 * t / c:10.2f}  {k}")
    print("# radhip kernels")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        if categorize(k) == "radhip (hand-written HIP)":
            print(f"{1e-6 * t / m:9.3f} {c / m:8.1f} {1e-3 * t / c:10.2f}  {k}")
    print("# other kernels (torch / hipBLASLt / runtime)")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        if categorize(k) != "radhip (hand-written HIP)":
            print(f"{1e-6 * t / m:9.3f} {c / m:8.1f} {1e-3 * t / c:10.2f}  {k}")


if __name__ == "__main__":
    main()
