"""Pose difference between the two robust-scale semantics on many config-2 scenes (GPU): the batch is
aligned with MEDIAN_REFERENCE (the reference's libstdc++ nth_element post-state) and MEDIAN_EXACT (true
order statistics); prints the max / percentiles of max |delta| over the Sophus params (sign-canonical)
and writes the per-scene deltas to a JSON file.  usage: median_modes_delta.py N_SCENES OUT.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402
from common import canon, gpu_batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
out_path = sys.argv[2] if len(sys.argv) > 2 else None
chunk = 64
deltas = []
for c0 in range(0, n, chunk):
    pairs = [synth.make_pair(seed=synth.SEED_BASE + i, n_features=2000, cell_order=30, nthreads=16)
             for i in range(c0, min(n, c0 + chunk))]
    res = {}
    for mode in (svo_amd.MEDIAN_REFERENCE, svo_amd.MEDIAN_EXACT):
        b, ps = gpu_batch(pairs, 5, 0, 4, median_mode=mode)
        b.run()
        res[mode] = b.results()[0]
        b.close()
    d = np.abs(canon(res[svo_amd.MEDIAN_REFERENCE]) - canon(res[svo_amd.MEDIAN_EXACT])).max(axis=1)
    deltas.extend(d.tolist())
    print(f"scenes {c0}..{c0 + len(pairs) - 1}: max {d.max():.3e}", flush=True)
d = np.array(deltas)
summary = {"scenes": len(d), "max": float(d.max()), "p50": float(np.percentile(d, 50)),
           "p99": float(np.percentile(d, 99)), "count_above_1e-6": int((d > 1e-6).sum()),
           "count_above_1e-5": int((d > 1e-5).sum())}
print(json.dumps(summary))
if out_path:
    with open(out_path, "w") as f:
        json.dump({"summary": summary, "per_scene_max_abs_param_delta": deltas}, f)
