#!/usr/bin/env python3
"""Regenerates tests/golden/select_small.npz and pose_ba_small.npz: small inputs and the CPU oracle's
outputs on them (the reference cannot run here; the oracle is pinned by
tests/test_feature_selection.py and tests/test_pose_ba.py).
  select_small.npz   a 160x96 textured image; gradientMagnitudeWithSSC (threshold 40, 60 candidates,
                     16-px cells, with and without bucketing, two cells pre-occupied) and
                     gradientMagnitudeByValue (threshold 40, 16-px cells)
  pose_ba_small.npz  64 features (9 without a point); optimizePose called twice on one object (the first
                     call sees no visible flags), exact-median semantics
Run from the repo root:  python tests/golden/make_golden_select_ba.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def select_case():
    rng = np.random.default_rng(77)
    img = rng.integers(0, 256, (25, 41)).astype(np.uint8)
    img = np.kron(img, np.ones((4, 4), np.uint8))[:96, :160]
    img = (img.astype(np.int32) + rng.integers(-6, 7, img.shape)).clip(0, 255).astype(np.uint8)
    img[:, :40] = 90
    occ = np.zeros((96 // 16 + 1, 160 // 16 + 1), np.uint8)
    occ[0, 0] = occ[3, 5] = 1
    out = dict(img=img, occ=occ)
    for name, bucket in (("b", True), ("nb", False)):
        px, resp, occ_after, nk = O.feature_select_ssc(img, 40, 60, bucket, 16, occ)
        out.update({f"ssc_{name}_px": px, f"ssc_{name}_resp": resp, f"ssc_{name}_occ": occ_after,
                    f"ssc_{name}_nk": np.int32(nk)})
    px, resp, _ = O.feature_select_by_value(img, 40, 16, occ)
    out.update(val_px=px, val_resp=resp)
    return out


def ba_case():
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(78)
    n = 64
    P = rng.normal(size=(n, 3)) * [4, 2, 3] + [0, 0, 12]
    true = np.concatenate([Rotation.from_rotvec([0.01, -0.02, 0.005]).as_quat(), [0.3, -0.1, 0.5]])
    pc = Rotation.from_quat(true[:4]).apply(P) + true[4:]
    b = pc / np.linalg.norm(pc, axis=1, keepdims=True) + rng.normal(size=(n, 3)) * 2e-3
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    has = np.ones(n, np.uint8)
    has[rng.choice(n, 9, replace=False)] = 0
    init = true.copy()
    init[4:] += [0.02, -0.01, 0.015]
    p1, e1, s1, v1 = O.optimize_pose(b, P, has, [], init)
    p2, e2, s2, v2 = O.optimize_pose(b, P, has, v1, p1)
    return dict(bearing=b, point=P, has_point=has, init=init, pose1=p1, err1=np.float64(e1), status1=np.int32(s1),
                vis1=v1, pose2=p2, err2=np.float64(e2), status2=np.int32(s2), vis2=v2)


if __name__ == "__main__":
    np.savez_compressed(os.path.join(OUT, "select_small.npz"), **select_case())
    np.savez_compressed(os.path.join(OUT, "pose_ba_small.npz"), **ba_case())
    print("wrote select_small.npz, pose_ba_small.npz")
