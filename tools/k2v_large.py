"""Reference-mode batch time against the vector size (diagnostic): 256 pairs of nf features (patch 5, 5 levels,
8 scenes), median of 5 runs after a warm-up (run + results, host clock).  The robust-scale kernel comes from
SVO_SCALE_IMPL (unset: K2V where the vector fits its registers; 1: K2R), so run it once per setting:
    python3 tools/k2v_large.py 2000 2400 2600        (SVO_LIB_DIR=<a variant build>: another K2V library)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402

P, D, PATCH, L = 256, 8, 5, 5
ctx = svo_amd.default_context()
for nf in [int(a) for a in sys.argv[1:]] or [2000, 2400, 2600]:
    sc = [synth.make_pair(seed=synth.SEED_BASE + 1300 + i, n_features=nf, patch_size=PATCH) for i in range(D)]
    c = sc[0].camera
    cam = svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])
    ps = svo_amd.PyramidSet(3 * D, c["width"], c["height"], L, ctx)
    ps.upload(0, np.stack([im for s in sc for im in (s.ref_img, s.kf_img, s.cur_img)]))
    ps.build()
    nmax = max(s.n_ref + s.n_kf for s in sc)
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, nmax, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    for i in range(P):
        s = sc[i % D]
        d = i % D
        b.set_pair(i, (ps, 3 * d), (ps, 3 * d + 1), (ps, 3 * d + 2), s.ref_pose, s.kf_pose, s.cur_init_pose,
                   s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
    b.run()
    b.results()
    runs = []
    for _ in range(5):
        t0 = time.perf_counter()
        b.run()
        poses, err, st = b.results()
        runs.append(time.perf_counter() - t0)
    kern = [b.traces(0)[l].scale_kernel for l in range(L)]
    print(f"nf {nf} slots {nmax * PATCH * PATCH} SVO_SCALE_IMPL={os.environ.get('SVO_SCALE_IMPL', 'auto')} "
          f"kernels {kern}: {np.median(runs) * 1e3:.3f} ms per 256-pair run ({P / np.median(runs):.0f} pairs/s)",
          flush=True)
    b.close()
    ps.clear() if hasattr(ps, "clear") else None
