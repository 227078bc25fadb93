"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Tolerances:
  * pyramid / gradient levels, visibility and pixel counts ....... bit-exact
  * Tukey scale (median, MAD, sigma) ............................. bit-exact (exact-order-statistic oracle)
  * H, g (summation order differs) ................................ 1e-10 relative to max |entry|
  * final pose vs the exact-statistic oracle ....................... 1e-9 (Sophus params, sign-canonical)
  * final pose vs the reference semantics (libstdc++ nth_element) .. 1e-5 (north_star tolerance)
  * FeatureAlignment (px, err, status) ........................... bit-exact
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
import svo_amd
import svo_amd.synth as synth
from common import canon, gpu_batch, make_pairs, oracle_align
from svo_amd._capi import check, lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pairs4():
    return make_pairs(4)


def test_pyramid_bitexact():
    rng = np.random.default_rng(7)
    s = synth.make_pair()
    for (h, w, lv) in [(376, 1241, 5), (37, 101, 4), (64, 64, 3), (5, 7, 2), (3, 3, 2), (17, 300, 6), (300, 17, 6),
                       (129, 4096, 3), (3, 9, 4), (4, 33, 5), (600, 900, 7), (95, 311, 4),
                       # strip seams where 62 owner lanes would put the right halo on lane 63: odd widths
                       # in (244n, 248n], and the own == 61 edge either side of them
                       (40, 489, 3), (37, 739, 4), (20, 1239, 3), (21, 977, 3), (22, 991, 3), (18, 488, 3),
                       (19, 245, 3), (23, 733, 5)]:
        imgs = [rng.integers(0, 256, (h, w), dtype=np.uint8) for _ in range(2)]
        if (h, w) == (376, 1241):
            imgs = [s.ref_img, s.cur_img] + imgs
        ps = svo_amd.PyramidSet(len(imgs), w, h, lv)
        ps.upload(0, np.stack(imgs))
        ps.build()
        for i, im in enumerate(imgs):
            oi, og = O.build_pyramid(im, lv)
            li, lg = O.unpack_levels(oi, w, h, lv), O.unpack_levels(og, w, h, lv)
            for l in range(lv):
                assert np.array_equal(ps.download(i, l, False), li[l]), (h, w, i, l, "image")
                assert np.array_equal(ps.download(i, l, True), lg[l]), (h, w, i, l, "gradient")


def _check_traces(tr_gpu, tr_cpu, min_level, max_level, exact_levels):
    for l in range(max_level, min_level - 1, -1):
        g, c = tr_gpu[l], tr_cpu[l]
        assert (g.n_ref_vis, g.n_vis, g.status) == (c.n_ref_vis, c.n_vis, c.status), (l, g.n_vis, c.n_vis)
        if l in exact_levels:
            assert g.median == c.median and g.mad == c.mad and g.sigma == c.sigma, l
        else:
            assert abs(g.sigma - c.sigma) <= 1e-9 * abs(c.sigma), l
        Hg = np.tril(np.array(g.H).reshape(6, 6))
        Hc = np.tril(np.array(c.H).reshape(6, 6))
        assert np.abs(Hg - Hc).max() <= 1e-10 * np.abs(Hc).max(), l
        gg, gc = np.array(g.g), np.array(c.g)
        assert np.abs(gg - gc).max() <= 1e-9 * max(np.abs(gc).max(), 1e-300), l
        assert abs(g.chi2 - c.chi2) <= 1e-10 * c.chi2, l


@pytest.mark.parametrize("cfg", [dict(patch=5, min_level=0, max_level=4, nf=2000),   # config 2
                                 dict(patch=4, min_level=0, max_level=2, nf=200),    # config 1 (5x5 footprint)
                                 dict(patch=7, min_level=1, max_level=3, nf=600)])
def test_align_matches_exact_oracle(cfg):
    pairs = make_pairs(3, n_features=cfg["nf"], patch_size=cfg["patch"])
    b, ps = gpu_batch(pairs, cfg["patch"], cfg["min_level"], cfg["max_level"])
    b.run()
    poses, err, st = b.results()
    for i, s in enumerate(pairs):
        pose_c, err_c, st_c, tr_c = oracle_align(s, cfg["patch"], cfg["min_level"], cfg["max_level"], mode=1)
        _check_traces(b.traces(i), tr_c, cfg["min_level"], cfg["max_level"], exact_levels={cfg["max_level"]})
        assert np.abs(canon(poses[i]) - canon(pose_c)).max() <= 1e-9
        assert abs(err[i] - err_c) <= 1e-9 * abs(err_c)
        assert st[i] == st_c


def test_align_reference_semantics_pose_tolerance(pairs4):
    b, ps = gpu_batch(pairs4, 5, 0, 4)
    b.run()
    poses, err, st = b.results()
    for i, s in enumerate(pairs4):
        pose_ref, err_ref, st_ref, _ = oracle_align(s, 5, 0, 4, mode=0, trace=False)
        assert np.abs(canon(poses[i]) - canon(pose_ref)).max() <= 1e-5
        assert abs(err[i] - err_ref) <= 1e-4 * err_ref
        assert st[i] == st_ref


def test_batch_composition_and_repeat_invariance(pairs4):
    b, _ = gpu_batch(pairs4, 5, 0, 4)
    b.run()
    p_all, e_all, s_all = b.results()
    b.run()
    p_again, e_again, _ = b.results()
    assert np.array_equal(p_all, p_again) and np.array_equal(e_all, e_again)
    b1, _ = gpu_batch(pairs4[2:3], 5, 0, 4)
    b1.run()
    p1, e1, s1 = b1.results()
    assert np.array_equal(p1[0], p_all[2]) and np.array_equal(e1[0], e_all[2]) and s1[0] == s_all[2]


def test_align_edge_cases():
    s = synth.make_pair(n_features=100, null_point_fraction=0.3)
    # null-point features keep their slots (src/image_alignment.cpp:85-99)
    b, _ = gpu_batch([s], 5, 0, 2)
    b.run()
    p, e, st = b.results()
    pc, ec, stc, trc = oracle_align(s, 5, 0, 2, mode=1)
    assert np.abs(canon(p[0]) - canon(pc)).max() <= 1e-9 and st[0] == stc
    _check_traces(b.traces(0), trc, 0, 2, exact_levels={2})
    # every feature without a point: nothing visible -> NaN error, Small_Step_Size (dx = 0)
    s2 = synth.make_pair(n_features=40)
    s2.has_point[:] = 0
    b, _ = gpu_batch([s2], 5, 0, 2)
    b.run()
    p, e, st = b.results()
    pc, ec, stc, _ = oracle_align(s2, 5, 0, 2, mode=1)
    assert np.isnan(e[0]) and np.isnan(ec) and st[0] == stc == 3
    assert np.array_equal(canon(p[0]), canon(pc))
    # initial pose far away: the patches leave the current image
    s3 = synth.make_pair(n_features=60)
    far = s3.cur_init_pose.copy()
    far[4] += 50.0
    s3.cur_init_pose = far
    b, _ = gpu_batch([s3], 5, 0, 2)
    b.run()
    p, e, st = b.results()
    pc, ec, stc, _ = oracle_align(s3, 5, 0, 2, mode=1)
    assert st[0] == stc and (np.isnan(e[0]) == np.isnan(ec))
    assert np.abs(canon(p[0]) - canon(pc)).max() <= 1e-9


# Residual distributions where rank n/2 is the first element of its bin and the bin below is far away:
# the even-length median (largest of the lower bin + smallest of the bin) / 2 lies below the median's
# bin, and K2's MAD bracket must allow for that (found by a model search of K2's bracket; the first
# case gave MAD 13 instead of 9 before the fix).  Known answers: exact order statistics of the slots.
# The other cases drive K2's exact fallbacks: an overfull median bin (> kCandCap slots), overfull MAD
# candidate bins, the bin below an even-length median holding > kPrevCap slots, an odd length, and
# outliers past +-64 that clamp into the end bins (MAD 90: its distance bin clamps too).
FLAT_CASES = [({2: 7, 7: 4, 15: 5, 24: 6}, 11.0, 9.0),
              ({2: 7, -8: 7, -22: 12, -14: 2}, None, None),
              ({18: 4, -20: 1, -3: 6, -25: 14, 10: 5}, None, None),
              ({0: 90, 5: 30, -5: 30}, 0.0, 0.0),
              ({-3: 50, 3: 50, 0: 2}, 0.0, 3.0),
              ({1: 20, 4: 20}, 2.5, 1.5),
              ({1: 3, 2: 2}, 1.0, 0.0),
              ({-90: 3, 0: 4, 90: 3}, 0.0, 90.0)]


def _exact_med_mad(groups):
    v = np.sort(np.repeat(np.array(list(groups.keys()), float), [25 * c for c in groups.values()]))
    m = len(v) // 2
    even = len(v) % 2 == 0
    med = (v[m - 1] + v[m]) / 2 if even else v[m]
    d = np.sort(np.abs(v - med))
    return med, ((d[m - 1] + d[m]) / 2 if even else d[m])


@pytest.mark.parametrize("case", FLAT_CASES)
def test_align_scale_median_below_its_bin(case):
    groups, med_known, mad_known = case
    med_x, mad_x = _exact_med_mad(groups)
    if med_known is not None:
        assert (med_x, mad_x) == (med_known, mad_known)
    s = synth.make_flat_blocks(groups, width=640, height=192)
    _, _, _, tr_c = oracle_align(s, 5, 0, 0, mode=1)
    assert (tr_c[0].median, tr_c[0].mad) == (med_x, mad_x)
    b, _ = gpu_batch([s], 5, 0, 0)
    b.run()
    g = b.traces(0)[0]
    assert (g.n_vis, g.median, g.mad, g.sigma) == (tr_c[0].n_vis, med_x, mad_x, tr_c[0].sigma)


def test_align_no_ref_features():
    s = synth.make_pair(n_features=40)
    s.n_kf, s.n_ref = s.n_ref + s.n_kf, 0
    b, _ = gpu_batch([s], 5, 0, 2)
    b.run()
    p, e, st = b.results()
    assert e[0] == 0.0 and np.array_equal(p[0], s.cur_init_pose)  # align() returns 0 (src/image_alignment.cpp:27-28)


def test_class_surface_align():
    s = synth.make_pair(n_features=300)
    cam = svo_amd.PinholeCamera.kitti()
    kf = svo_amd.Frame(cam, s.kf_img, 5)
    kf.abs_pose[:] = s.kf_pose
    ref = svo_amd.Frame(cam, s.ref_img, 5, last_keyframe=kf)
    ref.abs_pose[:] = s.ref_pose
    cur = svo_amd.Frame(cam, s.cur_img, 5, last_keyframe=kf)
    cur.abs_pose[:] = s.cur_init_pose
    for i in range(len(s.px)):
        fr = ref if i < s.n_ref else kf
        f = svo_amd.Feature(fr, s.px[i], bearing=s.bearing[i], point=svo_amd.Point(s.point[i]))
        fr.add_feature(f)
    ia = svo_amd.ImageAlignment(5, 0, 4)  # default: the reference's median semantics
    err = ia.align(ref, cur)
    pc, ec, stc, _ = oracle_align(s, 5, 0, 4, mode=0)  # oracle mode 0 = the reference's nth_element
    assert np.abs(canon(cur.abs_pose) - canon(pc)).max() <= 1e-9
    assert abs(err - ec) <= 1e-9 * ec
    # a second call reuses the object's batch and repeats the first exactly
    first = cur.abs_pose.copy()
    cur.abs_pose[:] = s.cur_init_pose
    assert ia.align(ref, cur) == err and np.array_equal(cur.abs_pose, first)
    # the per-level traces of the last call (entry l: level l), read on first access
    tr = ia.last_traces
    assert tr is ia.last_traces and [t.level for t in tr] == [0, 1, 2, 3, 4]
    assert all(t.n_vis > 0 for t in tr)
    # exact order statistics on request
    cur.abs_pose[:] = s.cur_init_pose
    svo_amd.ImageAlignment(5, 0, 4, median_mode=svo_amd.MEDIAN_EXACT).align(ref, cur)
    px_, ex_, _, _ = oracle_align(s, 5, 0, 4, mode=1)
    assert np.abs(canon(cur.abs_pose) - canon(px_)).max() <= 1e-9
    # ImagePyramid getters (src/image_pyramid.cpp:54-124)
    assert np.array_equal(ref.image_pyramid.get_base_image(), s.ref_img)
    assert ref.image_pyramid.get_image_size_at_level(4) == (78, 24)
    assert ref.image_pyramid.get_image_size_at_level(5) == (0, 0)


@pytest.mark.parametrize("patch", [7, 8, 5])
def test_feature_align_bitexact(patch):
    s = synth.make_pair(n_features=2000, patch_size=patch)
    rng = np.random.default_rng(patch)
    ref_grad = O.build_pyramid(s.ref_img, 1)[1]
    cur_grad = O.build_pyramid(s.cur_img, 1)[1]
    n = 2000
    ref_px = s.px[:n].copy()
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    init[:5] = [[-3, 10], [2, 2], [1240.5, 100], [600, 375.9], [3.5, 3.5]]  # out-of-frame / border cases
    px_c, err_c, st_c = O.feature_align(s.camera, patch, ref_grad, cur_grad, ref_px, init)
    ps = svo_amd.PyramidSet(2, 1241, 376, 1)
    ps.upload(0, np.stack([s.ref_img, s.cur_img]))
    ps.build()
    px_g = init.copy()
    fa = svo_amd.FeatureAlignment(patch)
    err_g, st_g = fa.align_batch(ps, 0, ps, 1, ref_px, px_g, svo_amd.PinholeCamera.kitti())
    assert np.array_equal(px_g, px_c)
    assert np.array_equal(st_g, st_c)
    assert np.array_equal(np.isnan(err_g), np.isnan(err_c))
    ok = ~np.isnan(err_c)
    assert np.array_equal(err_g[ok], err_c[ok])


def test_feature_align_large_batch_pageable_staging():
    """200k candidates (11 MB of per-call data, past the context's 8 MB pinned staging block): the
    pageable staging path gives the same bit-exact answers."""
    s = synth.make_pair(n_features=2000, patch_size=7)
    rng = np.random.default_rng(11)
    reps = 100
    ref_px = np.tile(s.px[:2000], (reps, 1))
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    ref_grad = O.build_pyramid(s.ref_img, 1)[1]
    cur_grad = O.build_pyramid(s.cur_img, 1)[1]
    px_c, err_c, st_c = O.feature_align(s.camera, 7, ref_grad, cur_grad, ref_px, init)
    ps = svo_amd.PyramidSet(2, 1241, 376, 1)
    ps.upload(0, np.stack([s.ref_img, s.cur_img]))
    ps.build()
    px_g = np.ascontiguousarray(init.copy())
    err_g, st_g = svo_amd.FeatureAlignment(7).align_batch(ps, 0, ps, 1, ref_px, px_g, svo_amd.PinholeCamera.kitti())
    assert np.array_equal(px_g, px_c) and np.array_equal(st_g, st_c)


def test_pyramid_build_async_pipeline():
    """svo_pyramid_set_build_async (the prep stream): a set built asynchronously while a batch aligns on another
    set gives the oracle's bytes, and a batch handed the async-built set (set_pairs waits for the build) aligns
    exactly as one built synchronously (bench.py end_to_end_device_images pipelines batches this way)."""
    sc = make_pairs(2)
    cam = svo_amd.PinholeCamera.kitti()
    imgs = np.stack([im for s in sc for im in (s.ref_img, s.kf_img, s.cur_img)])
    A = svo_amd.PyramidSet(6, 1241, 376, 5)
    B = svo_amd.PyramidSet(6, 1241, 376, 5)
    A.upload(0, imgs)
    B.upload(0, imgs)
    A.build()
    b = svo_amd.AlignBatch(cam, 5, 0, 4, 2, 2000, median_mode=svo_amd.MEDIAN_REFERENCE)
    frames = np.arange(6, dtype=np.int32).reshape(2, 3)
    poses = np.stack([np.concatenate([s.ref_pose, s.kf_pose, s.cur_init_pose]) for s in sc])
    n_feat = np.array([[s.n_ref, s.n_kf] for s in sc], np.int32)
    cat = lambda f: np.concatenate([getattr(s, f) for s in sc])
    feats = (cat("px"), cat("bearing"), cat("point"), cat("has_point"))
    b.set_pairs(0, A, A, A, frames, poses, n_feat, *feats)
    B.build_async()  # overlaps the alignment queued next
    b.run()
    pa, ea, sa = b.results()
    for i, im in enumerate(imgs[:3]):
        oi, og = O.build_pyramid(im, 5)
        li, lg = O.unpack_levels(oi, 1241, 376, 5), O.unpack_levels(og, 1241, 376, 5)
        for l in range(5):
            assert np.array_equal(B.download(i, l, False), li[l]) and np.array_equal(B.download(i, l, True), lg[l])
    A.build_async()  # rebuild A while B serves the next batch
    b.set_pairs(0, B, B, B, frames, poses, n_feat, *feats)
    b.run()
    pb, eb, sb = b.results()
    assert np.array_equal(pa, pb) and np.array_equal(ea, eb) and np.array_equal(sa, sb)
    b.set_pairs(0, A, A, A, frames, poses, n_feat, *feats)  # waits for A's async build
    b.run()
    pc, _, _ = b.results()
    assert np.array_equal(pa, pc)


def test_build_async_consumers_wait_for_the_rebuild():
    """Every consumer of a set's planes waits for the set's pending svo_pyramid_set_build_async: the set
    first holds scene X's pyramids, then scene Y's base images are uploaded and rebuilt asynchronously, and the
    consumer is called straight away.  A consumer that did not wait would read X's (or half-built) gradient /
    levels.  The set is large and the frames read are the last ones built, so a missing wait shows.  Consumers: FeatureAlignment, feature detection, an alignment batch whose pairs were set
    before the rebuild (run joins it), and FeatureAlignment through a multi-set call."""
    sx, sy = synth.make_pair(seed=synth.SEED_BASE + 3), synth.make_pair(seed=synth.SEED_BASE + 9)
    # 1536 frames (~1.4 ms of build): on the box the round-4 library (no joins in these consumers) failed this test
    # at this size and passed it at 384 frames (profiles/r05_async_negative_control.log)
    N, W, H, L = int(os.environ.get("SVO_ASYNC_FRAMES", "1536")), 1241, 376, 5
    frames_of = lambda s: np.stack([s.ref_img, s.kf_img, s.cur_img] * (N // 3))
    X, Y = frames_of(sx), frames_of(sy)
    cam = svo_amd.PinholeCamera.kitti()
    ps = svo_amd.PyramidSet(N, W, H, L)
    ps.upload(0, X)
    ps.build()
    fr_ref, fr_kf, fr_cur = N - 3, N - 2, N - 1

    def rebuild(imgs):
        ps.upload(0, imgs)
        ps.build_async()

    # FeatureAlignment on Y's gradients
    rng = np.random.default_rng(5)
    ref_px = sy.px[:1500].copy()
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    gy_ref, gy_cur = O.build_pyramid(sy.ref_img, 1)[1], O.build_pyramid(sy.cur_img, 1)[1]
    px_c, err_c, st_c = O.feature_align(sy.camera, 7, gy_ref, gy_cur, ref_px, init)
    rebuild(Y)
    px_g = init.copy()
    svo_amd.FeatureAlignment(7).align_batch(ps, fr_ref, ps, fr_cur, ref_px, px_g, cam)
    assert np.array_equal(px_g, px_c)
    # feature detection on X's level-0 gradient (keys response << 24 | y * W + x, row-major)
    gx_cur = O.build_pyramid(sx.cur_img, 1)[1][:W * H]
    thr = 50
    idx = np.nonzero(gx_cur > thr)[0].astype(np.uint32)
    keys_c = (gx_cur[idx].astype(np.uint32) << 24) | idx
    rebuild(X)
    fs = svo_amd.FeatureSelection(W, H, 30)
    keys = np.zeros(W * H, np.uint32)
    n = ctypes.c_int32()
    check(lib().svo_feature_detect(fs.ctx.handle, ps.handle, fr_cur, thr, W * H,
                                                          keys.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)))
    assert np.array_equal(keys[:n.value], keys_c)
    # an alignment batch handed Y's pair while the set still holds X, then the set rebuilt with Y: run waits
    b = svo_amd.AlignBatch(cam, 5, 0, L - 1, 1, 2000, median_mode=svo_amd.MEDIAN_REFERENCE)
    frames = np.array([[fr_ref, fr_kf, fr_cur]], np.int32)
    poses = np.concatenate([sy.ref_pose, sy.kf_pose, sy.cur_init_pose])[None]
    b.set_pairs(0, ps, ps, ps, frames, poses, np.array([[sy.n_ref, sy.n_kf]], np.int32), sy.px, sy.bearing, sy.point,
                sy.has_point)
    rebuild(Y)
    b.run()
    pg, eg, sg = b.results()
    pc, ec, stc, _ = oracle_align(sy, 5, 0, L - 1, mode=0)
    assert np.abs(canon(pg[0]) - canon(pc)).max() <= 1e-9 and sg[0] == stc
    # FeatureAlignment with per-candidate sets (svo_feature_align_multi) after a rebuild with X
    gx_ref = O.build_pyramid(sx.ref_img, 1)[1]
    gx_cur2 = O.build_pyramid(sx.cur_img, 1)[1]
    ref_px = sx.px[:1000].copy()
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    px_c, _, _ = O.feature_align(sx.camera, 7, gx_ref, gx_cur2, ref_px, init)
    rebuild(X)
    px_g = np.ascontiguousarray(init.copy())
    err = np.zeros(len(ref_px))
    st = np.zeros(len(ref_px), np.int32)
    sets = (ctypes.c_void_p * len(ref_px))(*([ps.handle] * len(ref_px)))
    rf = np.full(len(ref_px), fr_ref, np.int32)
    check(lib().svo_feature_align_multi(
        ps.ctx.handle, ctypes.byref(cam.as_c()), 7, sets, rf.ctypes.data_as(ctypes.c_void_p), ps.handle, fr_cur,
        len(ref_px), np.ascontiguousarray(ref_px).ctypes.data_as(ctypes.c_void_p), px_g.ctypes.data_as(ctypes.c_void_p),
        err.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p)))
    assert np.array_equal(px_g, px_c)
