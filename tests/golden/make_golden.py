#!/usr/bin/env python3
"""Regenerates tests/golden/*.npz: small synthetic inputs and the CPU oracle's outputs on them.

The reference itself cannot run here, so these goldens freeze the oracle's answers
(pinned by tests/test_oracle_kats.py) on inputs small enough to commit:
  align_small.npz   one frame pair at a quarter-KITTI camera (320x96), 120 features, patch 5,
                    3 levels; ImageAlignment outputs under both median semantics (0 = reference
                    libstdc++ nth_element, 1 = exact order statistics) with per-level traces
  feature_small.npz FeatureAlignment (patch 7) on the same pair's level-0 gradients, 64 candidates
  pyramid_small.npz image + gradient stacks of the three frames (4 levels)
Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
import svo_amd.synth as synth  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MINI = dict(width=320, height=96, fx=721.5377 / 4, fy=721.5377 / 4, cx=609.5593 / 4, cy=172.8540 / 4)
SEED = synth.SEED_BASE + 4242


def mini_pair():
    c = synth.default_config(n_features=120, patch_size=5, width=MINI["width"], height=MINI["height"],
                             null_point_fraction=0.05, nthreads=4)
    c.fx, c.fy, c.cx, c.cy = MINI["fx"], MINI["fy"], MINI["cx"], MINI["cy"]
    import ctypes
    H, W, N = c.height, c.width, c.n_features
    imgs = [np.zeros((H, W), np.uint8) for _ in range(3)]
    poses = [np.zeros(7) for _ in range(4)]
    px, br, pt = np.zeros((N, 2)), np.zeros((N, 3)), np.zeros((N, 3))
    hp = np.zeros(N, np.uint8)
    nr, nk = ctypes.c_int32(), ctypes.c_int32()
    p = synth._p
    n = synth.lib().svo_synth_pair(ctypes.byref(c), ctypes.c_uint64(SEED), *[p(i) for i in imgs], *[p(q) for q in poses],
                                   ctypes.byref(nr), ctypes.byref(nk), p(px), p(br), p(pt), p(hp))
    return dict(kf_img=imgs[0], ref_img=imgs[1], cur_img=imgs[2], kf_pose=poses[0], ref_pose=poses[1],
                cur_true_pose=poses[2], cur_init_pose=poses[3], n_ref=nr.value, n_kf=nk.value, px=px[:n],
                bearing=br[:n], point=pt[:n], has_point=hp[:n])


def trace_arrays(tr):
    keys = ["level", "n_ref_vis", "n_vis", "status", "median", "mad", "sigma", "chi2", "lambda_", "err"]
    out = {f"trace_{k}": np.array([getattr(t, k) for t in tr]) for k in keys}
    out["trace_H"] = np.array([list(t.H) for t in tr])
    out["trace_g"] = np.array([list(t.g) for t in tr])
    out["trace_dx"] = np.array([list(t.dx) for t in tr])
    return out


def main():
    s = mini_pair()
    cam = MINI
    L = 3
    pyr = {k: O.build_pyramid(s[k], 4) for k in ("ref_img", "kf_img", "cur_img")}
    np.savez_compressed(os.path.join(OUT, "pyramid_small.npz"),
                        **{f"{k}_stack": v[0] for k, v in pyr.items()}, **{f"{k}_grad": v[1] for k, v in pyr.items()})
    pl = [O.build_pyramid(s[k], L)[0] for k in ("ref_img", "kf_img", "cur_img")]
    pair = O.make_pair(pl[0], pl[1], pl[2], s["ref_pose"], s["kf_pose"], s["n_ref"], s["n_kf"], s["px"], s["bearing"],
                       s["point"], s["has_point"])
    outs = {}
    for mode in (0, 1):
        pose, err, st, tr = O.image_align(cam, 5, 0, L - 1, pair, s["cur_init_pose"], median_mode=mode, trace=True)
        outs.update({f"m{mode}_pose": pose, f"m{mode}_err": err, f"m{mode}_status": st})
        outs.update({f"m{mode}_{k}": v for k, v in trace_arrays(tr).items()})
    np.savez_compressed(os.path.join(OUT, "align_small.npz"), **s, **outs, camera=np.array(
        [cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["width"], cam["height"]]), patch=5, levels=L, seed=SEED)
    rg, cg = pyr["ref_img"][1][:cam["width"] * cam["height"]], pyr["cur_img"][1][:cam["width"] * cam["height"]]
    rg = rg.reshape(cam["height"], cam["width"])
    cg = cg.reshape(cam["height"], cam["width"])
    rng = np.random.default_rng(11)
    ref_px = s["px"][:64].copy()
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    init[0] = [2.0, 2.0]  # out of frame
    px, err, st = O.feature_align(cam, 7, rg, cg, ref_px, init)
    np.savez_compressed(os.path.join(OUT, "feature_small.npz"), ref_grad=rg, cur_grad=cg, ref_px=ref_px, init_px=init,
                        px=px, err=err, status=st, patch=7)
    print("wrote goldens to", OUT)


if __name__ == "__main__":
    main()
