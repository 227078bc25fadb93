"""K2V vs the oracle on many random residual vectors (development check; GPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import svo_amd  # noqa: E402
import oracle as O  # noqa: E402

DBL_MAX = np.finfo(np.float64).max


def ref(v, n):
    med = O.median(v, n, 0)
    d = np.abs(v - med)
    d[v >= DBL_MAX] = DBL_MAX
    return med, O.median(d, n, 0)


bad = 0
tot = 0
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
    rng = np.random.default_rng(1000 + seed)
    for nf in (40, 400, 1200, 1700, 1800, 2000, 2007, 2100, 2416):
        for pv in (1.0, 0.8):
            v = rng.normal(0, 8, nf * 25)
            vis = np.repeat(rng.random(nf) < pv, 25)
            if not vis.any():
                vis[:25] = True
            v[~vis] = DBL_MAX
            n = int(vis.sum())
            mc, dc = ref(v, n)
            m, d, dg = svo_amd.debug_robust_scale(v, n, impl=svo_amd.SCALE_K2V, diagnostics=True)
            tot += 1
            if m != mc or d != dc:
                bad += 1
                m2, d2 = svo_amd.debug_robust_scale(v, n, impl=svo_amd.SCALE_K2R)
                print(f"seed {seed} nf {nf} pv {pv}: K2V med {m!r} mad {d!r} | oracle {mc!r} {dc!r} | K2R ok {m2 == mc and d2 == dc} "
                      f"| med ok {m == mc} | diag {dg[:10].tolist()}", flush=True)
print(f"{bad} / {tot} mismatches")
sys.exit(3 if bad else 0)
