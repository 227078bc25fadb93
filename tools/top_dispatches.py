"""The longest dispatches of a rocprofv3 kernel trace, written beside every committed kernel-stats summary
(VERDICT r3 item 5): a dispatch far above its kernel's median carries its own evidence -- start / end timestamps,
queue, stream, and every dispatch that overlapped it in time -- so a device-level event (all queues stalled
together) can be told from one kernel's slow run without re-running anything.

usage: python3 tools/top_dispatches.py <run_kernel_trace.csv> [N=10] > profiles/<name>_top_dispatches.txt
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, n=10):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((e - s, s, e, r["Queue_Id"], r.get("Stream_Id", ""), r["Dispatch_Id"], r["Kernel_Name"]))
    if not rows:
        print("no dispatches")
        return
    med = defaultdict(list)
    for d, *_, k in rows:
        med[k].append(d)
    med = {k: statistics.median(v) for k, v in med.items()}
    t0 = min(r[1] for r in rows)
    print(f"# {path}: {len(rows)} dispatches; the {n} longest (times in us from the first dispatch's start)")
    print(f"# {'dur_us':>10} {'x_median':>8} {'start_us':>12} {'end_us':>12} queue stream dispatch  overlapping  kernel")
    for d, s, e, q, st, di, k in sorted(rows, reverse=True)[:n]:
        over = sum(1 for r in rows if r[1] < e and r[2] > s) - 1
        name = k.replace("(anonymous namespace)::", "").split("(")[0]
        print(f"  {d / 1e3:10.1f} {d / med[k]:8.1f} {(s - t0) / 1e3:12.1f} {(e - t0) / 1e3:12.1f} {q:>5} {st:>6} {di:>8}  "
              f"{over:11d}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
