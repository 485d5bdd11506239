"""SincNet / WavLM overlap inside the clean pass of the last window of a rocprofv3 kernel trace (bench.py): stream ids,
the first SincNet-backward launch against the end of the WavLM backward, and the busy-time overlap.

  python tools/stream_overlap.py kernel_trace.csv[.gz]
"""
import csv
import gzip
import sys

SINC = ("sconv", "b0x", "tail_", "bnselu", "sincconv", "sincnet", "res_tail")


def main():
    p = sys.argv[1]
    op = gzip.open if p.endswith(".gz") else open
    with op(p, "rt") as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"], r["Queue_Id"])
                for r in csv.DictReader(f)]
    rows.sort()
    stop = next((i for i, r in enumerate(rows) if "ts_acc_kernel" in r[2]), len(rows))
    rows = rows[:stop]
    marks = [i for i, r in enumerate(rows) if "pad_mixup_kernel" in r[2]]
    seg = rows[marks[-8]:marks[-4]]   # the last timed step (the stamped replay stages its micro-batches after it)
    fgm = next((i for i, r in enumerate(seg) if "fgm_norm" in r[2]), len(seg))
    clean = seg[:fgm]
    t0 = clean[0][0]
    streams = {}
    for s, e, n, sid, q in clean:
        k = "sinc" if any(x in n for x in SINC) else "other"
        streams.setdefault((k, sid, q), 0)
        streams[(k, sid, q)] += 1
    print("clean pass launches by (kind, stream, queue):", streams)
    sb = [(s, e, n) for s, e, n, _, _ in clean if "tail_bwd" in n or "b0x_bwd" in n or "sconv_wgrad" in n]
    pc = [(s, e) for s, e, n, _, _ in clean if "posconv2_kernel<true>" in n]
    ub = [(s, e) for s, e, n, _, _ in clean if "upsample_nearest1d_backward" in n]
    if sb:
        print(f"first SincNet backward launch at {(sb[0][0] - t0) / 1e6:.2f} ms, last end {(sb[-1][1] - t0) / 1e6:.2f}")
    if pc:
        print(f"WavLM backward ends (posconv backward) at {(pc[-1][1] - t0) / 1e6:.2f} ms")
    if ub:
        print(f"fusion backward (interp) at {(ub[0][0] - t0) / 1e6:.2f} ms")
    print(f"clean pass wall {(clean[-1][1] - t0) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
