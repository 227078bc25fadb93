"""Lazy chain joins (csrc/capi.hip svo_ctx::pending_batch): a reference-mode batch of >= 512 pairs runs as
four chains, and back-to-back runs of that batch are ordered per chain instead of each run forking after every chain of
the previous one; anything else that uses the context stream joins the pending chains first.  Every interleaving
below must give each pair its scene's pose bit for bit (the oracle pins the scenes' poses, 1e-9):

* runs back to back, then results;
* a run, then set_pairs with the pairs on other scenes (it overwrites the buffers the pending chains use), a run;
* a run of batch A, then a run of batch B on the same context (B joins A's chains first), both read back;
* a run, then a FeatureAlignment call, then results.
"""
import numpy as np
import pytest

import svo_amd
import svo_amd.synth as synth
from common import canon, oracle_align

P, D, NF, PATCH, L = 512, 8, 2000, 5, 5
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    ctx = svo_amd.default_context()
    sc = [synth.make_pair(seed=synth.SEED_BASE + 1500 + i, n_features=NF, patch_size=PATCH) for i in range(D)]
    c = sc[0].camera
    ps = svo_amd.PyramidSet(3 * D, c["width"], c["height"], L, ctx)
    ps.upload(0, np.stack([im for s in sc for im in (s.ref_img, s.kf_img, s.cur_img)]))
    ps.build()
    cam = svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])
    ref = [oracle_align(s, PATCH, 0, L - 1, mode=0, trace=False) for s in sc]
    return ctx, sc, ps, cam, ref


def packed(sc, idx):
    frames = np.array([[3 * k, 3 * k + 1, 3 * k + 2] for k in idx], np.int32)
    poses = np.stack([np.concatenate([sc[k].ref_pose, sc[k].kf_pose, sc[k].cur_init_pose]) for k in idx])
    n_feat = np.array([[sc[k].n_ref, sc[k].n_kf] for k in idx], np.int32)
    cat = lambda f: np.concatenate([getattr(sc[k], f) for k in idx])
    return frames, poses, n_feat, cat("px"), cat("bearing"), cat("point"), cat("has_point")


def check(poses, st, idx, ref, first_pose):
    for i, k in enumerate(idx):
        pc, _, stc = ref[k][:3]
        assert st[i] == stc, (i, k)
        assert np.abs(canon(poses[i]) - canon(pc)).max() <= 1e-9, (i, k)
        if k in first_pose:
            assert np.array_equal(poses[i], first_pose[k]), (i, k)
        else:
            first_pose[k] = poses[i].copy()


def test_gpu_lazy_join_interleavings(setup):
    ctx, sc, ps, cam, ref = setup
    seen = {}
    idx_a = [i % D for i in range(P)]
    idx_b = [(7 * i + 3) % D for i in range(P)]
    a = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    a.set_pairs(0, ps, ps, ps, *packed(sc, idx_a))
    for _ in range(3):  # back to back: per-chain order only
        a.run()
    p, _, st = a.results()
    check(p, st, idx_a, ref, seen)
    a.run()  # pending chains, then new pairs over the same buffers
    a.set_pairs(0, ps, ps, ps, *packed(sc, idx_b))
    a.run()
    a.run()
    p, _, st = a.results()
    check(p, st, idx_b, ref, seen)
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    b.set_pairs(0, ps, ps, ps, *packed(sc, idx_a))
    a.run()
    b.run()  # another batch: a's chains are joined first
    a.run()
    pb, _, stb = b.results()
    pa, _, sta = a.results()
    check(pb, stb, idx_a, ref, seen)
    check(pa, sta, idx_b, ref, seen)
    a.run()  # a synchronous entry point between a run and its results
    s = sc[0]
    fa = svo_amd.FeatureAlignment(7)
    px = np.ascontiguousarray(s.px[:32] + 0.5)
    fa.align_batch(ps, 0, ps, 2, s.px[:32], px, cam)
    p, _, st = a.results()
    check(p, st, idx_b, ref, seen)
    b.close()
    a.close()
