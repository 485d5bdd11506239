"""One-screen summary of a bench.py JSON line: throughput, the roofline object and the timed HIP kernels.

  python tools/brief.py gpurun_out/r01g/bench.json
"""
import json
import sys


def main(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.strip().startswith("{")]
    if not lines:
        raise SystemExit(f"{path}: no JSON line")
    d = json.loads(lines[-1])
    print("VALUE", d["value"], d["unit"], "ms/step", d["ms_per_step"], "loss", d.get("final_loss"))
    r = d.get("roofline") or {}
    print("ROOF", r.get("kernel"), r.get("achieved"), r.get("unit"), "frac", r.get("frac"),
          "avg_ms", r.get("avg_launch_ms"), "traffic", r.get("traffic"))
    rows = sorted((d.get("kernels") or {}).items(), key=lambda kv: -kv[1]["total_ms"])
    for k, v in rows:
        print(f"  {k:24s} {v['launches']:6d} x {1e3 * v['avg_ms']:8.1f} us = {v['total_ms']:8.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
