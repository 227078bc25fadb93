"""Shared helpers for the parity tests: synthetic pairs, oracle runs, GPU batches."""
import numpy as np

import oracle as O
import svo_amd
import svo_amd.synth as synth

KITTI = dict(fx=721.5377, fy=721.5377, cx=609.5593, cy=172.8540, width=1241, height=376)


def canon(p):
    """Quaternion sign canonicalisation (q and -q are the same rotation)."""
    p = np.array(p, dtype=np.float64)
    if p.ndim == 1:
        return p if p[3] >= 0 else np.concatenate([-p[:4], p[4:]])
    s = np.where(p[:, 3:4] >= 0, 1.0, -1.0)
    return np.concatenate([p[:, :4] * s, p[:, 4:]], axis=1)


def make_pairs(n, seed0=synth.SEED_BASE, **kw):
    return [synth.make_pair(seed=seed0 + i, **kw) for i in range(n)]


def oracle_pyramids(s, levels):
    return [O.build_pyramid(im, levels)[0] for im in (s.ref_img, s.kf_img, s.cur_img)]


def oracle_align(s, patch, min_level, max_level, mode=0, trace=True, init=None):
    pyr = oracle_pyramids(s, max_level + 1)
    pair = O.make_pair(pyr[0], pyr[1], pyr[2], s.ref_pose, s.kf_pose, s.n_ref, s.n_kf, s.px, s.bearing, s.point,
                       s.has_point)
    return O.image_align(s.camera, patch, min_level, max_level, pair,
                         s.cur_init_pose if init is None else init, median_mode=mode, trace=trace)


def gpu_batch(pairs, patch, min_level, max_level, ctx=None, max_features=None, median_mode=svo_amd.MEDIAN_EXACT):
    """Upload every pair (3 frames each) into one PyramidSet and one AlignBatch; returns (batch, set)."""
    cam = pairs[0].camera
    camera = svo_amd.PinholeCamera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"])
    ps = svo_amd.PyramidSet(3 * len(pairs), cam["width"], cam["height"], max_level + 1, ctx)
    imgs = np.stack([im for s in pairs for im in (s.ref_img, s.kf_img, s.cur_img)])
    ps.upload(0, imgs)
    ps.build()
    mf = max_features or max(max(len(s.px) for s in pairs), 1)
    b = svo_amd.AlignBatch(camera, patch, min_level, max_level, len(pairs), mf, ctx, median_mode=median_mode)
    for i, s in enumerate(pairs):
        b.set_pair(i, (ps, 3 * i), (ps, 3 * i + 1), (ps, 3 * i + 2), s.ref_pose, s.kf_pose, s.cur_init_pose,
                   s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
    return b, ps
