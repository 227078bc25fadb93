#!/usr/bin/env python3
"""Per-phase cycle breakdown of align_pairs_kernel (diagnostic build: SVO_PHASE_STAMPS=1).

Phases per level: P1 (visibility/projection), S1 (residuals), median, MAD, S5 (weights + normal
equations), P6 (solve + update).  Prints the mean shader cycles per phase and level over all pairs.
Never quote these runs' wall time: the stamps serialise lane 0.
"""
import argparse
import json
import os
import sys

os.environ["SVO_PHASE_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402
from common import gpu_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=512)
ap.add_argument("--distinct", type=int, default=8)
ap.add_argument("--features", type=int, default=2000)
args = ap.parse_args()

scenes = [synth.make_pair(seed=synth.SEED_BASE + i, n_features=args.features, nthreads=16) for i in range(args.distinct)]
pairs = [scenes[i % args.distinct] for i in range(args.pairs)]
b, ps = gpu_batch(pairs, 5, 0, 4)
b.run()
b.results()
st = b.phase_stamps().astype(np.int64)  # [pair][level][8]
names = ["P1 vis/proj", "S1 residual", "median", "MAD", "S5 normal-eq", "P6 solve"]
out = {}
for lvl in range(4, -1, -1):
    d = np.diff(st[:, lvl, :7], axis=1).mean(axis=0)
    out[f"level{lvl}"] = {n: float(v) for n, v in zip(names, d)}
    print(f"level {lvl}: " + "  ".join(f"{n}={v:9.0f}" for n, v in zip(names, d)))
tot = np.diff(st[:, :, :7], axis=2).mean(axis=0).sum(axis=0)
print("total  : " + "  ".join(f"{n}={v:9.0f}" for n, v in zip(names, tot)), " sum", tot.sum())
span = (st[:, 0, 6] - st[:, 4, 0]).astype(np.float64)
print("per-pair span cycles: mean %.0f min %.0f max %.0f" % (span.mean(), span.min(), span.max()))
print(json.dumps(out))
