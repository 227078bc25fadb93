"""Diagnostic: per-phase cycle counts of the robust-scale kernel (K2) on a config-2 batch.

Needs the stamps build (`make -C semi-direct-visual-odometry_amd stamps`) and a GPU:
    SVO_LIB_DIR=semi-direct-visual-odometry_amd/build/stamps python3 tools/k2_stamps.py
Not part of the product or the test suite.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SVO_LIB_DIR", os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "stamps"))

import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402
from svo_amd import _capi  # noqa: E402

PHASES = ["count", "hist", "find", "bracket", "gather", "medsel", "madsel", "fallback", "end"]


def main():
    P, nf, L, patch, D = 512, 2000, 5, 5, 8
    ctx = svo_amd.Context(0)
    scenes = [synth.make_pair(seed=synth.SEED_BASE + i, n_features=nf, patch_size=patch, nthreads=16, cell_order=30)
              for i in range(D)]
    cam = scenes[0].camera
    camera = svo_amd.PinholeCamera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"])
    ps = svo_amd.PyramidSet(3 * P, cam["width"], cam["height"], L, ctx)
    base = np.stack([im for s in scenes for im in (s.ref_img, s.kf_img, s.cur_img)])
    for first in range(0, P, D):
        ps.upload(3 * first, base[:3 * min(D, P - first)])
    ps.build()
    batch = svo_amd.AlignBatch(camera, patch, 0, L - 1, P, nf, ctx)
    for i in range(P):
        s = scenes[i % D]
        batch.set_pair(i, (ps, 3 * i), (ps, 3 * i + 1), (ps, 3 * i + 2), s.ref_pose, s.kf_pose, s.cur_init_pose,
                       s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
    batch.run()
    ctx.synchronize()
    lib = _capi.lib()
    fn = lib.svo_debug_stamps
    fn.restype = ctypes.c_int32
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    st = np.zeros((4096, 16), dtype=np.uint64)
    assert fn(st.ctypes.data_as(ctypes.c_void_p), st.nbytes) == 0
    st = st[:P * 5].reshape(P, 5, 16).astype(np.int64)
    for level in range(L - 1, -1, -1):
        s = st[:, level]
        d = np.diff(s[:, :10], axis=1)
        row = " ".join(f"{p}={np.median(d[:, i]):.0f}" for i, p in enumerate(PHASES))
        tot = np.median(s[:, 9] - s[:, 0])
        med_slow = int(np.sum(s[:, 10] >= 1000000))
        mad_slow = int(np.sum(s[:, 12] == 1))
        print(f"level {level}: total={tot:.0f} cyc (max {np.max(s[:, 9] - s[:, 0]):.0f})  {row}  | median cnt "
              f"med={np.median(s[:, 10] % 1000000):.0f} max={np.max(s[:, 10] % 1000000):.0f} slow={med_slow}  "
              f"mad cand med={np.median(s[:, 11]):.0f} max={np.max(s[:, 11]):.0f} slow={mad_slow}")
        if np.any(s[:, 14]):  # realtime (100 MHz) workgroup start / end, per half-batch chain
            for c0 in range(0, P, P // 2):
                t0, t1 = s[c0:c0 + P // 2, 14], s[c0:c0 + P // 2, 15]
                print(f"          chain @{c0}: starts spread {(t0.max() - t0.min()) / 100:.1f} us, "
                      f"wg duration med {np.median(t1 - t0) / 100:.1f} us max {(t1 - t0).max() / 100:.1f} us, "
                      f"first start -> last end {(t1.max() - t0.min()) / 100:.1f} us")
        if np.any(s[:, 13]):  # SVO_K2_DUP build: a second key sweep before the gather
            print(f"          second key sweep={np.median(s[:, 13] - s[:, 4]):.0f}  gather after it="
                  f"{np.median(s[:, 5] - s[:, 13]):.0f}")


if __name__ == "__main__":
    main()
