"""Average duration per (kernel, grid size) in the kernel traces tools/ab_prof.sh wrote, side by side.

  python tools/ab_prof_read.py TAG N pattern [pattern ...]
"""
import csv
import gzip
import re
import sys
from collections import defaultdict


def load(path, pats):
    acc = defaultdict(lambda: [0.0, 0])
    with gzip.open(path, "rt") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not any(re.search(p, name) for p in pats):
                continue
            key = (name[:70], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))
            a = acc[key]
            a[0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a[1] += 1
    return acc


def main():
    tag, n, pats = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    runs = [load(f"gpurun_out/{tag}_{i}.csv.gz", pats) for i in range(n)]
    keys = sorted(set().union(*runs))
    for k in keys:
        cells = []
        for r in runs:
            t, c = r.get(k, (0.0, 0))
            cells.append(f"{t / c:8.2f} ({c:4d})" if c else "       -       ")
        print(f"{k[0]:70s} grid {k[1]:8d}  " + "  ".join(cells))


if __name__ == "__main__":
    main()
