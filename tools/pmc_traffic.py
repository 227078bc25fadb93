"""HBM traffic of the align chain from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs).

Correction per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes of a wide read,
so it is doubled; WRITE_SIZE is taken as is.  Both are KiB per dispatch.  Traffic of one chain launch
(= one bench step over all pairs) = sum over the chain's kernels of the per-dispatch bytes, divided by
the number of bench steps in the profiled process: dispatches of align_scale_kernel (K2, once per level
and chain) / (levels x --chains); the bench's 512-pair reference-mode batch runs as four concurrent chains.

usage: python3 tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> --pairs P --features N --levels L
       --patch S > profiles/pmc_traffic.json
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(pass_dir, counter):
    tot = collections.Counter()
    runs = 0
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if "svo::align" not in name or r["Counter_Name"] != counter:
                continue
            tot[name.split("(")[0]] += float(r["Counter_Value"]) * 1024.0
            if any(k in name for k in ("align_scale_kernel", "align_scale_ref_kernel", "align_scale_refv_kernel")):
                # K2 / K2R / K2V: once per level and chain
                runs += 1
    return tot, runs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--pairs", type=int, default=512)
    ap.add_argument("--features", type=int, default=2000)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--patch", type=int, default=5)
    ap.add_argument("--chains", type=int, default=4, help="concurrent chains per bench step (bench.py n_chains)")
    a = ap.parse_args()
    fetch, runs_f = per_kernel(a.fetch_dir, "FETCH_SIZE")
    write, runs_w = per_kernel(a.write_dir, "WRITE_SIZE")
    assert runs_f and runs_w, "no align dispatches found"
    runs_f, runs_w = runs_f / (a.chains * a.levels), runs_w / (a.chains * a.levels)
    kernels = sorted(set(fetch) | set(write))
    per = {k: {"read": 2.0 * fetch[k] / runs_f, "write": write[k] / runs_w} for k in kernels}
    total = sum(v["read"] + v["write"] for v in per.values())
    print(json.dumps({
        "pairs": a.pairs, "features": a.features, "levels": a.levels, "patch": a.patch, "chains": a.chains,
        "hbm_bytes_per_launch": round(total), "hbm_bytes_per_pair": round(total / a.pairs),
        "per_kernel_bytes_per_launch": {k: {kk: round(vv) for kk, vv in v.items()} for k, v in per.items()},
        "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KiB -> bytes",
        "calibration_note": "MI355X_MICROARCH.md calibrates the FETCH_SIZE x2 only for 16-B/lane coalesced streams; "
                            "the 8-B/lane accesses of K1 / K2V (and K2R) are uncalibrated, so the read bytes are an estimate",
    }, indent=1))


if __name__ == "__main__":
    main()
