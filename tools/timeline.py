"""Per-step CU-time budget of the headline from per-workgroup records.

Runs the headline workload (config 2: 512 pairs, 2000 features, patch 5, 5 levels, the reference's median semantics,
detector cell order) on the diagnostic build `make timeline` (build/timeline/libsvo_hip.so: every K1 / K2V / K3
workgroup records its start and end on the chip-wide 100 MHz clock and the CU it ran on), then splits the steps' CU
time into K2V, K1, K3 and idle:

  * wall     first workgroup start to last workgroup end, per step;
  * CU time  256 CUs x wall; per CU the union of each kernel's workgroup intervals (K1 / K3 share a CU between
             several workgroups; K2V holds a whole CU); `idle` = CU time no K1 / K2V / K3 workgroup held;
  * K2V      per-pair durations (median, p10, p90, max, by level) against the single-pair latency, and per launch
             (a chain's 128 pairs at one level) the spread of its workgroups' starts and its span;
  * lower bounds  sum(K2V pair durations) / 256 and (sum(K2V) + K1 + K3 CU time) / 256.

usage: python3 tools/timeline.py [--distinct D] [--steps K] [--json out.json]   (the timeline library is picked up from
semi-direct-visual-odometry_amd/build/timeline unless SVO_LIB_DIR says otherwise)
"""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SVO_LIB_DIR", os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "timeline"))
sys.path.insert(0, ROOT)
import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402
from svo_amd import _capi  # noqa: E402

REC = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("kind", "<u4"), ("level", "<u4"), ("block", "<u4"), ("hw", "<u4"),
                ("xcc", "<u4"), ("pair_base", "<u4")])
KIND = {1: "K1", 2: "K2V", 3: "K3"}
TICK_US = 0.01  # s_memrealtime: 100 MHz


def read(tag, reset=False):
    f = getattr(_capi.lib(), f"svo_debug_timeline_{tag}")
    f.restype = ctypes.c_int32
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int32]
    n = ctypes.c_uint32(0)
    if reset:
        assert f(None, 0, ctypes.byref(n), 1) == 0
        return None
    buf = np.zeros(1 << 18, REC)
    assert f(buf.ctypes.data, buf.nbytes, ctypes.byref(n), 0) == 0
    if n.value > len(buf):
        raise SystemExit(f"timeline: {n.value} records overflow the {len(buf)}-record buffer; run fewer steps")
    return buf[:n.value]


def union_len(iv):
    """Total length of the union of (start, end) intervals."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def pct(a, q):
    return float(np.percentile(a, q)) if len(a) else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=512)
    ap.add_argument("--distinct", type=int, default=512)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    P, NF, L, PATCH = args.pairs, 2000, 5, 5
    D = max(1, min(args.distinct, P))
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(16) as ex:
        scenes = list(ex.map(lambda i: synth.make_pair(seed=synth.SEED_BASE + i, n_features=NF, patch_size=PATCH,
                                                       nthreads=1, cell_order=30), range(D)))
    ctx = svo_amd.default_context()
    c = scenes[0].camera
    cam = svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])
    ps = svo_amd.PyramidSet(3 * P, c["width"], c["height"], L, ctx)
    idx = [i % D for i in range(P)]
    for c0 in range(0, P, 64):
        ks = idx[c0:c0 + 64]
        ps.upload(3 * c0, np.stack([im for k in ks for im in (scenes[k].ref_img, scenes[k].kf_img, scenes[k].cur_img)]))
    ps.build()
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    frames = np.arange(3 * P, dtype=np.int32).reshape(P, 3)
    poses = np.stack([np.concatenate([scenes[k].ref_pose, scenes[k].kf_pose, scenes[k].cur_init_pose]) for k in idx])
    nfeat = np.array([[scenes[k].n_ref, scenes[k].n_kf] for k in idx], np.int32)
    cat = lambda f: np.ascontiguousarray(np.concatenate([getattr(scenes[k], f) for k in idx]))
    b.set_pairs(0, ps, ps, ps, frames, poses, nfeat, cat("px"), cat("bearing"), cat("point"),
                cat("has_point").astype(np.uint8))
    for _ in range(args.warmup):
        b.run()
    ctx.synchronize()
    read("k13", reset=True)
    read("k2v", reset=True)
    ctx.synchronize()
    for _ in range(args.steps):
        b.run()
    ctx.synchronize()
    r = np.concatenate([read("k13"), read("k2v")])
    r = r[r["kind"] > 0]
    t_first = int(r["t0"].min())
    # HW_ID (gfx9): CU_ID [11:8], SH_ID [12], SE_ID [15:13]; XCC_ID [3:0]
    cu = ((r["xcc"] & 0xF) * 256 + ((r["hw"] >> 13) & 0x7) * 32 + ((r["hw"] >> 12) & 1) * 16 + ((r["hw"] >> 8) & 0xF)).astype(np.int64)
    ncu = len(np.unique(cu))
    wall = (int(r["t1"].max()) - t_first) * TICK_US
    step_ms = wall / args.steps / 1e3
    per_cu = defaultdict(lambda: defaultdict(list))
    for row, c_ in zip(r, cu):
        per_cu[int(c_)][int(row["kind"])].append((int(row["t0"]), int(row["t1"])))
    cu_time = {k: 0.0 for k in ("K1", "K2V", "K3", "K1|K3", "any")}
    for c_, kinds in per_cu.items():
        for k, iv in kinds.items():
            cu_time[KIND[k]] += union_len(iv) * TICK_US
        cu_time["K1|K3"] += union_len(kinds.get(1, []) + kinds.get(3, [])) * TICK_US
        cu_time["any"] += union_len([x for iv in kinds.values() for x in iv]) * TICK_US
    total = 256 * wall
    k2 = r[r["kind"] == 2]
    d2 = (k2["t1"] - k2["t0"]).astype(np.float64) * TICK_US
    by_level = {int(l): {"pairs": int((k2["level"] == l).sum()), "median_us": round(float(np.median(d2[k2["level"] == l])), 1),
                         "p90_us": round(pct(d2[k2["level"] == l], 90), 1), "max_us": round(float(d2[k2["level"] == l].max()), 1)}
                for l in np.unique(k2["level"])}
    # launches: (step, level, pair_base); steps told apart by start-time order within each (level, pair_base)
    launches = defaultdict(list)
    for row in k2:
        launches[(int(row["level"]), int(row["pair_base"]))].append(row)
    spans, start_spread, slowest, inflation = [], [], [], []
    for key, rows in launches.items():
        rows = sorted(rows, key=lambda x: int(x["t0"]))
        n_per = len(rows) // args.steps
        for s in range(args.steps):
            grp = rows[s * n_per:(s + 1) * n_per]
            if not grp:
                continue
            t0s = np.array([int(x["t0"]) for x in grp])
            t1s = np.array([int(x["t1"]) for x in grp])
            dur = (t1s - t0s) * TICK_US
            spans.append((t1s.max() - t0s.min()) * TICK_US)
            start_spread.append((t0s.max() - t0s.min()) * TICK_US)
            slowest.append(dur.max())
            inflation.append((t1s.max() - t0s.min()) * TICK_US / np.median(dur))
    k1 = r[r["kind"] == 1]
    k3 = r[r["kind"] == 3]

    def wg_stats(rows):  # per-workgroup durations by level (workgroups that returned at once excluded: < 2 us)
        d = (rows["t1"] - rows["t0"]).astype(np.float64) * TICK_US
        keep = d >= 2.0
        out = {}
        for l in np.unique(rows["level"]):
            m = keep & (rows["level"] == l)
            if m.any():
                out[int(l)] = {"workgroups": int(m.sum()), "median_us": round(float(np.median(d[m])), 1),
                               "p90_us": round(pct(d[m], 90), 1)}
        return out

    # co-residency: for each K1 / K3 workgroup, the mean number of K1 / K3 workgroups resident on its CU over its life
    def coresidency(kinds):
        vals = []
        for c_, kd in per_cu.items():
            iv = sorted(x for k in kinds for x in kd.get(k, []))
            if not iv:
                continue
            ev = sorted([(s_, 1) for s_, _ in iv] + [(e_, -1) for _, e_ in iv])
            cur, last, area, busy = 0, ev[0][0], 0, 0
            for t, dlt in ev:
                if cur > 0:
                    area += cur * (t - last)
                    busy += t - last
                cur += dlt
                last = t
            if busy:
                vals.append(area / busy)
        return round(float(np.mean(vals)), 2) if vals else None
    out = {
        "workload": f"config 2 headline: {P} pairs ({D} distinct scenes), {NF} features, patch {PATCH}, {L} levels, "
                    f"reference median semantics, cell order; diagnostic build (make timeline)",
        "steps": args.steps, "cus_seen": ncu, "step_ms": round(step_ms, 4),
        "cu_time_per_step_ms_x_cu": {k: round(v / args.steps / 1e3, 4) for k, v in cu_time.items()},
        "cu_time_per_step_frac": {
            "K2V": round(cu_time["K2V"] / total, 4), "K1": round(cu_time["K1"] / total, 4),
            "K3": round(cu_time["K3"] / total, 4), "K1|K3": round(cu_time["K1|K3"] / total, 4),
            "idle": round(1 - cu_time["any"] / total, 4)},
        "k2v_pair_us": {"count": int(len(d2)), "median": round(float(np.median(d2)), 1), "mean": round(float(d2.mean()), 1),
                        "p10": round(pct(d2, 10), 1), "p90": round(pct(d2, 90), 1), "max": round(float(d2.max()), 1),
                        "by_level": by_level},
        "k2v_launch_us": {"count": len(spans), "span_median": round(float(np.median(spans)), 1),
                          "start_spread_median": round(float(np.median(start_spread)), 1),
                          "start_spread_p90": round(pct(start_spread, 90), 1),
                          "slowest_pair_median": round(float(np.median(slowest)), 1),
                          "span_over_median_pair": round(float(np.median(inflation)), 3)},
        "k1_workgroups": int(len(k1)), "k3_workgroups": int(len(k3)),
        "k1_workgroup_us_by_level": wg_stats(k1), "k3_workgroup_us_by_level": wg_stats(k3),
        "k1k3_workgroups_resident_per_busy_cu": coresidency((1, 3)),
        "lower_bounds_ms": {
            "k2v_only": round(float(d2.sum()) / 256 / args.steps / 1e3, 4),
            "k2v_plus_k1k3_cu_time": round((float(d2.sum()) + cu_time["K1|K3"]) / 256 / args.steps / 1e3, 4)},
    }
    # per pair and level, its K2V durations over the steps (does a pair's cost at one level predict the next?)
    per_pair = defaultdict(list)
    for row, d in zip(k2, d2):
        per_pair[(int(row["pair_base"]) + int(row["block"]), int(row["level"]))].append(float(d))
    pairs_idx = sorted({p_ for p_, _ in per_pair})
    lv = sorted({l_ for _, l_ in per_pair}, reverse=True)
    mat = np.array([[np.mean(per_pair.get((p_, l_), [np.nan])) for l_ in lv] for p_ in pairs_idx])
    corr = {}
    for i in range(len(lv) - 1):
        a_, b_ = mat[:, i], mat[:, i + 1]
        ok = ~np.isnan(a_) & ~np.isnan(b_)
        corr[f"L{lv[i]}->L{lv[i + 1]}"] = round(float(np.corrcoef(a_[ok], b_[ok])[0, 1]), 3) if ok.sum() > 2 else None
    out["k2v_pair_duration_corr_between_levels"] = corr
    # the same pair and level in different steps (run-to-run repeatability of a pair's K2V time)
    rep = [np.std(v) / np.mean(v) for v in per_pair.values() if len(v) > 1]
    out["k2v_pair_duration_cv_across_steps_median"] = round(float(np.median(rep)), 4) if rep else None
    # one chain's critical path: per (chain, step) the launches in order K1 K2V K3 per level; each launch's span (first
    # workgroup start to last end) and the gap from the previous launch's last end to its first start
    launches_all = defaultdict(list)
    for row in r:
        launches_all[(int(row["pair_base"]), int(row["level"]), int(row["kind"]))].append((int(row["t0"]), int(row["t1"])))
    spans_k = defaultdict(list)
    gaps_k = defaultdict(list)
    order = [(l_, k_) for l_ in sorted({int(x) for x in r["level"]}, reverse=True) for k_ in (1, 2, 3)]
    for pb in sorted({int(x) for x in r["pair_base"]}):
        seq = []
        for l_, k_ in order:
            iv = sorted(launches_all.get((pb, l_, k_), []))
            n_per = len(iv) // args.steps if iv else 0
            for st_ in range(args.steps):
                grp = sorted(iv, key=lambda x: x[0])[st_ * n_per:(st_ + 1) * n_per] if n_per else []
                if grp:
                    seq.append((st_, l_, k_, min(x[0] for x in grp), max(x[1] for x in grp)))
        seq.sort(key=lambda x: x[3])
        for i_, (st_, l_, k_, a0, a1) in enumerate(seq):
            spans_k[KIND[k_]].append((a1 - a0) * TICK_US)
            if i_:
                gaps_k[KIND[k_]].append((a0 - seq[i_ - 1][4]) * TICK_US)
    out["chain_launch_span_us_median"] = {k: round(float(np.median(v)), 1) for k, v in spans_k.items()}
    out["chain_gap_before_launch_us_median"] = {k: round(float(np.median(v)), 1) for k, v in gaps_k.items()}
    out["chain_gap_before_launch_us_mean"] = {k: round(float(np.mean(v)), 1) for k, v in gaps_k.items()}
    # CU occupancy over time, in 25 us bins from the first workgroup start: CUs holding a K2V workgroup, CUs holding
    # only K1 / K3 workgroups, idle CUs (every step; the step boundaries show as the idle peaks)
    binw = 2500  # ticks (25 us)
    nb = int((int(r["t1"].max()) - t_first) // binw) + 1
    k2b = np.zeros(nb)
    k13b = np.zeros(nb)
    for c_, kd in per_cu.items():
        for kinds, acc in (((2,), k2b), ((1, 3), k13b)):
            iv = sorted(x for k in kinds for x in kd.get(k, []))
            merged = []
            for s_, e_ in iv:
                if merged and s_ <= merged[-1][1]:
                    merged[-1][1] = max(merged[-1][1], e_)
                else:
                    merged.append([s_, e_])
            for s_, e_ in merged:
                a0, a1 = s_ - t_first, e_ - t_first
                for b_ in range(int(a0 // binw), int(a1 // binw) + 1):
                    lo_, hi_ = max(a0, b_ * binw), min(a1, (b_ + 1) * binw)
                    if hi_ > lo_:
                        acc[b_] += (hi_ - lo_) / binw
    k13b = np.minimum(k13b, 256 - k2b)
    out["occupancy_25us_bins"] = {"k2v_cus": [round(x, 1) for x in k2b], "k1k3_only_cus": [round(x, 1) for x in k13b],
                                  "idle_cus": [round(256 - a - b_, 1) for a, b_ in zip(k2b, k13b)]}
    print(json.dumps({k: v for k, v in out.items() if k != "occupancy_25us_bins"}, indent=1))
    idle = out["occupancy_25us_bins"]["idle_cus"]
    print("idle CUs per 25 us bin:", " ".join(f"{x:.0f}" for x in idle))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
