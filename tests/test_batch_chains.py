"""The production batch path at bench scale: one batch of 131 pairs with
2000 features each runs as two concurrent half-batch chains (capi.hip run_batch / sub_batch, the tail not
a multiple of 8), staged through the pinned ring (set_pair: ~130 KB a pair, so the 8 MB ring wraps twice)
with a FeatureAlignment call in between (another pinned user drains the ring).  Every pair must match the
oracle (pose <= 1e-9, status exact) and repeat its own single-pair run bit for bit; the bulk
svo_align_batch_set_pairs path must give the identical batch.  Both median modes."""
import numpy as np
import pytest
import torch  # noqa: F401  (before libsvo_hip initialises HIP: torch's own HIP runtime then finds the GPU too)

import svo_amd
import svo_amd.synth as synth
from common import canon, oracle_align

P, D, NF, PATCH, L = 131, 4, 2000, 5, 5


def scenes():
    return [synth.make_pair(seed=synth.SEED_BASE + 300 + i, n_features=NF, patch_size=PATCH) for i in range(D)]


def camera_of(s):
    c = s.camera
    return svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])


def pyramids(sc, ctx):
    c = sc[0].camera
    ps = svo_amd.PyramidSet(3 * D, c["width"], c["height"], L, ctx)
    ps.upload(0, np.stack([im for s in sc for im in (s.ref_img, s.kf_img, s.cur_img)]))
    ps.build()
    return ps


def packed(sc, pairs):
    d = len(sc)
    frames = np.array([[3 * (i % d), 3 * (i % d) + 1, 3 * (i % d) + 2] for i in pairs], np.int32)
    poses = np.stack([np.concatenate([sc[i % d].ref_pose, sc[i % d].kf_pose, sc[i % d].cur_init_pose]) for i in pairs])
    n_feat = np.array([[sc[i % d].n_ref, sc[i % d].n_kf] for i in pairs], np.int32)
    cat = lambda f: np.concatenate([getattr(sc[i % d], f) for i in pairs])
    return frames, poses, n_feat, cat("px"), cat("bearing"), cat("point"), cat("has_point")


def test_packed_layout():
    """CPU: the bulk call's packed rows are pair after pair, in pair order."""
    sc = [synth.make_pair(seed=7 + i, n_features=30) for i in range(2)]
    frames, poses, n_feat, px, br, pt, hp = packed(sc, [0, 1, 2])
    assert frames.shape == (3, 3) and poses.shape == (3, 21) and n_feat.shape == (3, 2)
    assert px.shape == (90, 2) and np.array_equal(px[60:], sc[0].px) and np.array_equal(px[30:60], sc[1].px)
    assert np.array_equal(frames[1], [3, 4, 5])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [svo_amd.MEDIAN_REFERENCE, svo_amd.MEDIAN_EXACT])
def test_gpu_two_chain_batch(mode):
    ctx = svo_amd.default_context()
    sc = scenes()
    ps = pyramids(sc, ctx)
    cam = camera_of(sc[0])
    fa = svo_amd.FeatureAlignment(PATCH, 0, 3, ctx)
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=mode)
    for i in range(P):
        s = sc[i % D]
        b.set_pair(i, (ps, 3 * (i % D)), (ps, 3 * (i % D) + 1), (ps, 3 * (i % D) + 2), s.ref_pose, s.kf_pose,
                   s.cur_init_pose, s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
        if i == 40:  # another user of the pinned block mid-way: drains the ring's pending copies
            px = sc[0].px[:16].copy()
            fa.align_batch(ps, [0], ps, 2, sc[0].px[:16], px, cam)
    b.run()
    poses, err, st = b.results()
    # the oracle per distinct scene (oracle median_mode 0 = the reference's nth_element)
    omode = 0 if mode == svo_amd.MEDIAN_REFERENCE else 1
    ref = [oracle_align(s, PATCH, 0, L - 1, mode=omode, trace=False) for s in sc]
    for i in range(P):
        pc, ec, stc = ref[i % D][:3]
        assert st[i] == stc, i
        assert np.abs(canon(poses[i]) - canon(pc)).max() <= 1e-9, i
        # pairs of the same scene in both chains: bit-identical
        assert np.array_equal(poses[i], poses[i % D]) and err[i] == err[i % D], i
    # single-pair runs repeat the batch bit for bit (one pair from each chain and the tail)
    for i in (1, 66, 130):
        s = sc[i % D]
        b1 = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, 1, NF, ctx, median_mode=mode)
        b1.set_pair(0, (ps, 3 * (i % D)), (ps, 3 * (i % D) + 1), (ps, 3 * (i % D) + 2), s.ref_pose, s.kf_pose,
                    s.cur_init_pose, s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
        b1.run()
        p1, e1, s1 = b1.results()
        assert np.array_equal(p1[0], poses[i]) and e1[0] == err[i] and s1[0] == st[i], i
        b1.close()
    # the bulk form: the same batch from one svo_align_batch_set_pairs call (and one of 2 calls), with the
    # features in host memory (uploaded on the context's copy stream) or on the device (torch tensors)
    for split, on_dev in ((P, False), (57, False), (P, True)):
        bb = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=mode)
        for lo in range(0, P, split):
            hi = min(P, lo + split)
            args = packed(sc, range(lo, hi))
            if on_dev:
                feats = [torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0") for a in args[3:]]
                torch.cuda.synchronize()
                args = (*args[:3], *feats)
            bb.set_pairs(lo, ps, ps, ps, *args)
        bb.run()
        pb, eb, sb = bb.results()
        assert np.array_equal(pb, poses) and np.array_equal(eb, err) and np.array_equal(sb, st)
        bb.close()
    b.close()


@pytest.mark.gpu
def test_gpu_wide_launch_instantiation():
    """Two chains of 132 pairs (the 2000-feature vectors fit K2V, so both chains run it; trace field
    scale_kernel): every pair against the oracle's std::nth_element path and bit for bit against a single-pair
    run of its scene.  K2R's own batch instantiations are covered by tests/test_config4.py."""
    ctx = svo_amd.default_context()
    sc = scenes()
    ps = pyramids(sc, ctx)
    cam = camera_of(sc[0])
    n = 264
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, n, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    b.set_pairs(0, ps, ps, ps, *packed(sc, range(n)))
    b.run()
    poses, err, st = b.results()
    ref = [oracle_align(s, PATCH, 0, L - 1, mode=0, trace=False) for s in sc]
    for i in range(n):
        pc, ec, stc = ref[i % D][:3]
        assert st[i] == stc, i
        assert np.abs(canon(poses[i]) - canon(pc)).max() <= 1e-9, i
    for d in range(D):
        s = sc[d]
        b1 = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, 1, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
        b1.set_pair(0, (ps, 3 * d), (ps, 3 * d + 1), (ps, 3 * d + 2), s.ref_pose, s.kf_pose, s.cur_init_pose,
                    s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
        b1.run()
        p1, e1, s1 = b1.results()
        b1.close()
        for i in (d, d + 132, n - D + d):  # both chains
            assert np.array_equal(p1[0], poses[i]) and e1[0] == err[i] and s1[0] == st[i], (d, i)
    b.close()
