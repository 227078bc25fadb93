"""Per-kernel statistics of a rocprofv3 kernel trace, split by launch shape.

rocprofv3's own `--stats` summary averages every launch of a kernel together, so the 128-pair K2V launches of the
headline and the 256 / 512-pair launches of the batch-scaling lines end up in one mean.  This splits the trace by
(kernel, grid) and prints, per launch shape: count, median / mean / p10 / p90 duration and the total, so the dominant
kernel's per-launch time -- and from it the bench line's roofline fraction -- can be recomputed from tracked files.

usage: python3 tools/headline_kernel_stats.py <run_kernel_trace.csv> [--wg-size 512] > profiles/<name>_headline_kernel_stats.csv

K2V (`align_scale_refv_kernel`) runs one 512-thread workgroup per pair, so its Grid_Size_X / 512 is the pairs of the
launch; the `pairs` column is filled for it and for K2R (`align_scale_ref_kernel`, 512 or 1024 threads).
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("svo::", "")
    return n.split("(")[0].strip()


def pct(v, q):
    v = sorted(v)
    i = min(len(v) - 1, max(0, int(round(q * (len(v) - 1)))))
    return v[i]


def main(path):
    groups = defaultdict(list)
    wg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
            groups[k].append(d)
            wg[k] = int(r.get("Workgroup_Size_X", 0) or 0)
    w = csv.writer(sys.stdout, lineterminator="\n")
    w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "workgroup_x", "pairs", "count", "median_us", "mean_us", "p10_us",
                "p90_us", "min_us", "max_us", "total_ms"])
    for k in sorted(groups, key=lambda k: -sum(groups[k])):
        v = groups[k]
        name, gx, gy, gz = k
        pairs = ""
        if "align_scale_ref" in name and wg[k]:
            pairs = gx // wg[k]
        w.writerow([name, gx, gy, gz, wg[k], pairs, len(v), round(statistics.median(v), 2), round(statistics.mean(v), 2),
                    round(pct(v, 0.1), 2), round(pct(v, 0.9), 2), round(min(v), 2), round(max(v), 2),
                    round(sum(v) / 1e3, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
