"""Top-N rows of a rocprofv3 --stats kernel_stats.csv: name (shortened), calls, total ms, avg us, share.

  python tools/stats_top.py kernel_stats.csv [N]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print(f"total kernel time {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} launches")
    for r in rows[:n]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e6:9.3f} ms {int(r['Calls']):6d} x {float(r['AverageNs']) / 1e3:9.2f} us {100 * t / tot:5.1f}%  "
              f"{r['Name'][:110]}")


if __name__ == "__main__":
    main()
