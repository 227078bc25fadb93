"""Per-kernel average of rocprofv3 PMC counters (tools/pmc_run.sh pass directories).

usage: python3 tools/pmc_summary.py [--by-level=L] gpurun_out/pmc/p1 [gpurun_out/pmc/p2 ...]
Prints, per kernel (template arguments kept, call arguments dropped), the mean per dispatch of every
counter found, plus derived ratios where the inputs are present (SQ cycle counters are quad-cycles).
"""
import collections
import csv
import glob
import os
import re
import sys


def kname(full):
    m = re.search(r"(\w+_kernel(<[^>]*>)?)", full)
    return m.group(1) if m else full.split("(")[0]


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    args = sys.argv[1:]
    levels = 0
    if args and args[0].startswith("--by-level="):  # tag the align kernels with their pyramid level
        levels = int(args.pop(0).split("=")[1])
    for d in args:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per_dispatch = collections.defaultdict(float)
            names = {}
            order = collections.defaultdict(list)  # queue -> align dispatches in order
            for r in csv.DictReader(open(path)):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per_dispatch[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = kname(r["Kernel_Name"])
                if levels and "align_" in r["Kernel_Name"]:
                    order[r["Queue_Id"]].append(int(r["Dispatch_Id"]))
            for q, ds in order.items():  # per chain: K1 K2 K3 per level, coarsest first
                for i, disp in enumerate(str(x) for x in sorted(set(ds))):
                    names[disp] += f" L{levels - 1 - (i // 3) % levels}"
            for (disp, ctr), v in per_dispatch.items():
                vals[names[disp]][ctr].append(v)
    for k in sorted(vals):
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        print(f"== {k}  ({max(len(v) for v in vals[k].values())} dispatches)")
        for n in sorted(c):
            print(f"   {n:28s} {c[n]:.4g}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                if n in c:
                    print(f"   {n + ' / WAVE_CYCLES':42s} {c[n] / wc:.3f}")
        if "SQ_BUSY_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
            print(f"   {'VALU issue per busy SQ cycle':42s} {c['SQ_ACTIVE_INST_VALU'] / c['SQ_BUSY_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
