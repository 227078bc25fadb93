#!/usr/bin/env python3
"""Per-level durations of the alignment kernels from a rocprofv3 kernel trace.

usage: tools/level_times.py <run_kernel_trace.csv> [levels]

Each chain (one HIP stream) launches K0 (older builds), then per level (coarsest first) K1 -> K2 -> K3.  The trace is
split by stream, cut into chains at every K0, and the average duration of each (level, kernel) and the
gap from the previous kernel's end to this kernel's start (launch + dependency latency) are printed, in us.
"""
import collections
import csv
import sys


def kind(name):
    for tag, k in (("align_init_kernel", "K0"), ("align_residual_kernel", "K1"), ("align_scale_kernel", "K2"),
                   ("align_weights_kernel", "K3")):
        if tag in name:
            return k
    return None


def main():
    path = sys.argv[1]
    levels = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    by_stream = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = kind(r["Kernel_Name"])
        if k:
            by_stream[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    chains = []
    for s, ev in by_stream.items():
        ev.sort()
        if any(e[2] == "K0" for e in ev):  # builds with a separate init kernel: a chain starts at K0
            cur = None
            for e in ev:
                if e[2] == "K0":
                    cur = [e]
                    chains.append(cur)
                elif cur is not None:
                    cur.append(e)
        else:  # the init runs inside the first K1: a chain is 3 * levels kernels from a K1
            ev = ev[next(i for i, e in enumerate(ev) if e[2] == "K1"):]
            chains += [[None] + ev[i:i + 3 * levels] for i in range(0, len(ev), 3 * levels)]
    span = []
    for c in chains:
        if len(c) != 1 + 3 * levels:
            continue
        if c[0] is None:
            c[0] = (c[1][0], c[1][0], "K0")
        span.append((c[-1][1] - c[0][0]) / 1e3)
        for i, (t0, t1, k) in enumerate(c):
            lvl = "-" if i == 0 else levels - 1 - (i - 1) // 3
            dur[(lvl, k)].append((t1 - t0) / 1e3)
            if i:
                gap[(lvl, k)].append((t0 - c[i - 1][1]) / 1e3)
    print(f"chains: {len(span)}  chain span avg {sum(span) / max(1, len(span)):.1f} us")
    print(f"{'level':>5} {'kernel':>6} {'avg us':>8} {'gap us':>8}")
    tot_d = tot_g = 0.0
    for key in sorted(dur, key=lambda x: (x[0] != "-", -x[0] if x[0] != "-" else 0, x[1])):
        d = sum(dur[key]) / len(dur[key])
        g = sum(gap[key]) / len(gap[key]) if gap[key] else 0.0
        tot_d += d
        tot_g += g
        print(f"{key[0]:>5} {key[1]:>6} {d:8.1f} {g:8.1f}")
    print(f"total kernel {tot_d:.1f} us, total gaps {tot_g:.1f} us")


if __name__ == "__main__":
    main()
