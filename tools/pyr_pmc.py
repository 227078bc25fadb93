"""Per-kernel breakdown of one pyramid build (tools/pyr_measure.sh output): launch durations from the kernel trace and
HBM-side bytes from the FETCH_SIZE / WRITE_SIZE passes, against each launch's algorithmic bytes (KITTI shape, 1536
frames, 5 levels; the level-l launch of pyr_dn_kernel is told apart by its grid).

FETCH_SIZE is reported raw and doubled (MI355X_MICROARCH.md: gfx950 counts half the bytes of a wide streaming read);
these kernels read dwords per lane, a width the guide leaves uncalibrated, so the algorithmic column is the yardstick.
usage: python3 tools/pyr_pmc.py gpurun_out/pyr > profiles/r05_pyramid_pmc.json
"""
import collections
import csv
import glob
import json
import os
import sys

N, W, H, L = 1536, 1241, 376, 5


def dims():
    w, h, out = W, H, []
    for _ in range(L):
        out.append((w, h))
        w, h = (w + 1) // 2, (h + 1) // 2
    return out


def key(name, grid_x, grid_y):
    if "pyr_l01_kernel" in name:
        return "pyr_l01_kernel (L0 gradient + L1 of both stacks)"
    if "pyr_dn_kernel" in name:
        return f"pyr_dn_kernel grid {grid_x}x{grid_y}"
    return name.split("(")[0][:60]


def main():
    d = sys.argv[1]
    dur = collections.defaultdict(list)
    grid_threads = {}  # trace key -> total work-items (the counter passes' Grid_Size)
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        grid_threads[key(r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"])] = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])
        dur[key(r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"])].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = {}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        acc = collections.defaultdict(list)
        for path in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                if r["Counter_Name"] == cname:
                    acc[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024.0)
        ctr[cname] = acc
    dm = dims()
    px = [w * h for w, h in dm]
    alg = {"pyr_l01_kernel": (N * px[0], N * (px[0] + 2 * px[1]))}
    for l in range(2, L):
        alg[f"dn L{l}"] = (N * 2 * px[l - 1], N * 2 * px[l])
    out = {"frames": N, "shape": [W, H, L], "kernels": []}
    # order the pyr_dn launches by duration (level 2 is the largest)
    dn = sorted((k for k in dur if k.startswith("pyr_dn_kernel")), key=lambda k: -sorted(dur[k])[len(dur[k]) // 2])
    names = [k for k in dur if k.startswith("pyr_l01")] + dn
    labels = ["pyr_l01_kernel"] + [f"dn L{l}" for l in range(2, 2 + len(dn))]
    for k, lab in zip(names, labels):
        v = sorted(dur[k])
        med_us = v[len(v) // 2] / 1e3
        ar, aw = alg[lab]

        def pick(cname):
            for (kn, gsize), vals in ctr[cname].items():
                if ("pyr_l01_kernel" in kn and lab == "pyr_l01_kernel") or (
                        "pyr_dn_kernel" in kn and gsize == grid_threads[k]):
                    return sorted(vals)[len(vals) // 2]
            return None
        f, w = pick("FETCH_SIZE"), pick("WRITE_SIZE")
        out["kernels"].append({
            "kernel": lab, "trace_key": k, "launches": len(v), "median_us": round(med_us, 1),
            "algorithmic_read_B": ar, "algorithmic_write_B": aw,
            "algorithmic_GBps": round((ar + aw) / (med_us * 1e-6) / 1e9, 1),
            "frac_of_8TBps": round((ar + aw) / (med_us * 1e-6) / 8e12, 4),
            "FETCH_SIZE_raw_B": f, "FETCH_SIZE_x2_B": None if f is None else 2 * f, "WRITE_SIZE_B": w})
    tot_us = sum(x["median_us"] for x in out["kernels"])
    tot_b = sum(x["algorithmic_read_B"] + x["algorithmic_write_B"] for x in out["kernels"])
    out["sum_median_us"] = round(tot_us, 1)
    out["algorithmic_B"] = tot_b
    out["frac_of_8TBps_kernels_only"] = round(tot_b / (tot_us * 1e-6) / 8e12, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
