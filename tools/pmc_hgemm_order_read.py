"""Pairs the FETCH_SIZE rows of a tools/pmc_hgemm_order.py run (rocprofv3 counter_collection.csv) with its plan
(the script's JSON output): per (shape, group_m) the mean fetch per measured launch (2 x FETCH_SIZE KiB, the gfx950
wide-load correction of MI355X_MICROARCH.md) against the algorithmic A + B bytes.

  python tools/pmc_hgemm_order_read.py PLAN.json COUNTERS.csv
"""
import csv
import json
import sys


def main():
    plan = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    rows = [r for r in csv.DictReader(open(sys.argv[2])) if "hgemm_kernel" in r.get("Kernel_Name", "")]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
    vals = [float(r["Counter_Value"]) for r in rows]
    i = 0
    out = []
    for p in plan:
        seg = vals[i:i + p["launches"]]
        i += p["launches"]
        meas = seg[p["warmup"]:]
        fetch = 2 * 1024 * sum(meas) / len(meas)
        out.append({**p, "fetch_bytes": round(fetch), "fetch_over_alg_read": round(fetch / p["alg_read_bytes"], 2)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
