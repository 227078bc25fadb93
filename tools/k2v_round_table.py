"""The reference's nth_element rounds on real config-2 residual vectors, tabulated.

For config-2 scenes (seeds 0x5EED0000 + i, 2000 features, patch 5, 5 levels) the oracle returns every level's residual
vector (oracle.image_align_vectors); both passes of computeMedian / computeMAD (src/algorithm.cpp:834-865) are run
through the numpy round model (tests/introselect_rounds.py, pinned to std::nth_element) and every round is tabulated:
segment S, Ks (swaps), the cut, the kept side, the discarded side.  K2V runs a round as a block round while S exceeds
its one-wave size, so the table splits rounds into block and one-wave rounds.  `--one-wave` sets that size: 1024 (the
default) reproduces profiles/r06_k2v_round_table.json; the product layouts use 2048 since DESIGN 19.7.

Item 3 (two pairs per CU on 4-byte keys): for the same vectors, how often distinct doubles share the top 32 bits of the
order-preserving 64-bit key (the 4-byte key), and how often a round's pivot -- the value every comparison of the round
is made against -- or the final vec[nth - 1] / vec[nth] shares its bucket with a distinct value (where a 4-byte key
would decide a comparison differently from the reference's double `<`).

usage: python3 tools/k2v_round_table.py [--scenes N] [--one-wave 1024|2048] [--json out.json]
"""
import argparse
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O  # noqa: E402
import svo_amd.synth as synth  # noqa: E402
from introselect_rounds import DBL_MAX, rounds  # noqa: E402



def key32(v):
    """Top 32 bits of the order-preserving u64 image of a double (a 4-byte sort key)."""
    b = np.ascontiguousarray(v, np.float64).view(np.uint64)
    k = np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))
    return (k >> np.uint64(32)).astype(np.uint32)


def passes(v, n_valid):
    """Both passes' round lists [(S, Ks, cut - first, kept, discarded, pivot)] and the pass inputs."""
    out, vecs = [], []
    x = np.array(v, np.float64)
    for P in range(2):
        nth = n_valid // 2
        vecs.append(x.copy())
        rs = []
        gen = rounds(x, nth)
        lo = None
        try:
            while True:
                f0, l0, p, ks, ng, nl, cut, a = next(gen)
                S = l0 - f0
                kept = (l0 - cut) if cut <= nth else (cut - f0)
                rs.append((S, ks, cut - f0, kept, S - kept, p))
                if cut == nth and lo is None and nth >= 1:
                    lo = float(a[nth - 1])
        except StopIteration as e:
            first, last, a = e.value
        a[first:last] = np.sort(a[first:last])
        hi = float(a[nth])
        if lo is None:
            lo = float(a[nth - 1]) if nth >= 1 else 0.0
        out.append((rs, lo, hi))
        r = (lo + hi) / 2.0 if len(x) % 2 == 0 and nth >= 1 else hi
        if P == 0:
            x = np.abs(np.array(v, np.float64) - r)
            x[np.array(v) >= DBL_MAX] = DBL_MAX
    return out, vecs


def collisions(vec, pivots, lo, hi):
    """(distinct-value pairs sharing a 4-byte key, pivots whose key bucket holds another distinct value, whether
    vec[nth-1] / vec[nth] do)."""
    fin = vec[vec < DBL_MAX]
    u = np.unique(fin)  # distinct values, sorted
    k = key32(u)
    same = k[1:] == k[:-1]  # adjacent distinct values with one key (sorted, so every shared bucket shows here)
    bad_keys = set(k[1:][same].tolist())
    piv_bad = sum(1 for p in pivots if p < DBL_MAX and int(key32(np.array([p]))[0]) in bad_keys)
    fin_bad = int(int(key32(np.array([lo]))[0]) in bad_keys) + int(int(key32(np.array([hi]))[0]) in bad_keys)
    return int(same.sum()), piv_bad, fin_bad


def scene_vectors(i):
    s = synth.make_pair(seed=synth.SEED_BASE + i, n_features=2000, patch_size=5, nthreads=1, cell_order=30)
    pyr = [O.build_pyramid(im, 5)[0] for im in (s.ref_img, s.kf_img, s.cur_img)]
    pair = O.make_pair(pyr[0], pyr[1], pyr[2], s.ref_pose, s.kf_pose, s.n_ref, s.n_kf, s.px, s.bearing, s.point,
                       s.has_point)
    return O.image_align_vectors(s.camera, 5, 0, 4, pair, s.cur_init_pose, 0)


def analyse(i):
    vecs, nvs = scene_vectors(i)
    rows = []
    for lvl, (v, nv) in enumerate(zip(vecs, nvs)):
        res, pin = passes(v, nv)
        for P, (rs, lo, hi) in enumerate(res):
            c = collisions(pin[P], [r[5] for r in rs], lo, hi)
            rows.append({"scene": i, "level": 4 - lvl, "pass": P, "rounds": [r[:5] for r in rs], "pairs_same_key": c[0],
                         "pivots_in_shared_bucket": c[1], "final_in_shared_bucket": c[2]})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=16)
    ap.add_argument("--one-wave", type=int, default=1024)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    one_wave = args.one_wave
    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        rows = [r for rs in ex.map(analyse, range(args.scenes)) for r in rs]
    summary = {"scenes": args.scenes, "vectors": len(rows) // 2, "one_wave": one_wave}
    for P in (0, 1):
        blk, onew, lops, small_ks = [], [], [], []
        for r in rows:
            if r["pass"] != P:
                continue
            b = [x for x in r["rounds"] if x[0] > one_wave]
            blk.append(len(b))
            onew.append(len(r["rounds"]) - len(b))
            lops += [x for x in b if x[4] < 0.3 * x[0]]       # rounds that discard < 30 % of the segment
            small_ks += [x for x in b if x[1] <= 64]          # rounds whose exchange is <= 64 swaps
        allb = [x for r in rows if r["pass"] == P for x in r["rounds"] if x[0] > one_wave]
        summary[f"pass{P}"] = {
            "block_rounds_per_call_mean": round(float(np.mean(blk)), 2), "block_rounds_max": int(max(blk)),
            "one_wave_rounds_per_call_mean": round(float(np.mean(onew)), 2),
            "block_rounds_discarding_lt_30pct_mean": round(len(lops) / len(blk), 2),
            "block_rounds_ks_le_64_mean": round(len(small_ks) / len(blk), 2),
            "block_round_ks_over_S_median": round(float(np.median([x[1] / x[0] for x in allb])), 4),
            "block_round_discard_frac_median": round(float(np.median([x[4] / x[0] for x in allb])), 4),
        }
    tot_pairs = sum(r["pairs_same_key"] for r in rows)
    piv = sum(r["pivots_in_shared_bucket"] for r in rows)
    fin = sum(r["final_in_shared_bucket"] for r in rows)
    calls = len(rows)
    summary["key32"] = {
        "distinct_value_pairs_sharing_a_key_per_vector_mean": round(tot_pairs / calls, 1),
        "vectors_with_any_shared_key": sum(1 for r in rows if r["pairs_same_key"] > 0),
        "pivots_in_a_shared_bucket": piv, "finals_in_a_shared_bucket": fin, "pass_vectors": calls,
        "pass_vectors_with_a_pivot_or_final_in_a_shared_bucket":
            sum(1 for r in rows if r["pivots_in_shared_bucket"] or r["final_in_shared_bucket"]),
    }
    # an example call: level 0 of scene 0, both passes
    ex = [r for r in rows if r["scene"] == 0 and r["level"] == 0]
    summary["example_scene0_level0"] = {f"pass{r['pass']}": [list(x) for x in r["rounds"]] for r in ex}
    summary["columns"] = "rounds: (S, Ks, cut - first, kept, discarded)"
    print(json.dumps(summary, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
