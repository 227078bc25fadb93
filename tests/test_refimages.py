"""The reference's own test images as parity inputs: image_1.png (1920 x 1080) and
camera/undistort_input.png (1280 x 960), converted to grey once by tests/golden/make_golden_refimages.py and
committed as tests/golden/refimages.npz.  Real textures with odd level sizes (1080 -> 540 -> 270 -> 135 -> 68,
960 -> ... -> 60), unlike the synthetic scenes of the other tests.

GPU against the oracle on the same bytes:
  * the 5-level intensity and gradient pyramids (src/image_pyramid.cpp:36-52) ........ byte-equal
  * FeatureAlignment p7 / p8 on the level-0 gradients (src/feature_alignment.cpp) ...... bit-exact
  * FeatureSelection gradientMagnitudeWithSSC / ByValue (src/feature_selection.cpp) ..... bit-exact
  * ImageAlignment (reference median semantics) on a real-texture pair ................. pose <= 1e-9, status exact
"""
import os
import types

import numpy as np
import pytest

import oracle as O
from common import canon, oracle_align

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "refimages.npz")
NAMES = ("image_1", "undistort_input")


def _img(name):
    with np.load(GOLDEN) as z:
        return np.ascontiguousarray(z[name])


def test_fixture_and_oracle_levels():
    """CPU: the fixtures and the oracle's level geometry ((w + 1) / 2, (h + 1) / 2 per level)."""
    a, b = _img("image_1"), _img("undistort_input")
    assert a.shape == (1080, 1920) and b.shape == (960, 1280) and a.dtype == np.uint8
    assert a.std() > 20 and b.std() > 20  # real texture
    w, h = 1920, 1080
    lv = O.unpack_levels(O.build_pyramid(a, 5)[0], w, h, 5)
    assert [x.shape for x in lv] == [(1080, 1920), (540, 960), (270, 480), (135, 240), (68, 120)]
    assert np.array_equal(lv[0], a)


def _texture_points(img, n, rng, border=24):
    """n distinct textured pixels (level-0 abs gradient sum >= 40) away from the border."""
    g = O.unpack_levels(O.build_pyramid(img, 1)[1], img.shape[1], img.shape[0], 1)[0]
    ys, xs = np.nonzero(g[border:-border, border:-border] >= 40)
    pick = rng.choice(len(xs), size=n, replace=False)
    return np.stack([xs[pick] + border, ys[pick] + border], axis=1).astype(np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_pyramid_bytes(name):
    import svo_amd
    img = _img(name)
    h, w = img.shape
    ps = svo_amd.PyramidSet(1, w, h, 5)
    ps.upload(0, img[None])
    ps.build()
    oi, og = O.build_pyramid(img, 5)
    li, lg = O.unpack_levels(oi, w, h, 5), O.unpack_levels(og, w, h, 5)
    for l in range(5):
        assert np.array_equal(ps.download(0, l, False), li[l]), (name, l, "image")
        assert np.array_equal(ps.download(0, l, True), lg[l]), (name, l, "gradient")


@pytest.mark.gpu
@pytest.mark.parametrize("patch", [7, 8])
def test_gpu_feature_align_bitexact(patch):
    import svo_amd
    img = _img("image_1")
    h, w = img.shape
    cur = np.ascontiguousarray(np.roll(img, (1, 2), axis=(0, 1)))  # the scene moved by (+2, +1) px
    rng = np.random.default_rng(patch)
    ref_px = _texture_points(img, 2000, rng)
    init = ref_px + [2.0, 1.0] + rng.uniform(-1.5, 1.5, ref_px.shape)
    init[:3] = [[-3.0, 10.0], [w - 0.5, 500.0], [3.5, 3.5]]  # out of frame / border
    cam = dict(fx=1000.0, fy=1000.0, cx=w / 2, cy=h / 2, width=w, height=h)
    rg = O.build_pyramid(img, 1)[1]
    cg = O.build_pyramid(cur, 1)[1]
    px_c, err_c, st_c = O.feature_align(cam, patch, rg, cg, ref_px, init)
    ps = svo_amd.PyramidSet(2, w, h, 1)
    ps.upload(0, np.stack([img, cur]))
    ps.build()
    px_g = init.copy()
    err_g, st_g = svo_amd.FeatureAlignment(patch).align_batch(ps, 0, ps, 1, ref_px, px_g,
                                                             svo_amd.PinholeCamera(w, h, 1000.0, 1000.0, w / 2, h / 2))
    assert np.array_equal(px_g, px_c) and np.array_equal(st_g, st_c)
    ok = ~np.isnan(err_c)
    assert np.array_equal(np.isnan(err_g), ~ok) and np.array_equal(err_g[ok], err_c[ok])
    assert (st_c[3:] >= 0).all()  # (a real run: the candidates moved)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_feature_selection_bitexact(name):
    import svo_amd
    img = _img(name)
    h, w = img.shape
    fr = svo_amd.Frame(svo_amd.PinholeCamera(w, h, 1000.0, 1000.0, w / 2, h / 2), img, 1)
    for thr, num, bucket in ((50, 200, True), (50, 2000, False), (30, 1000, True)):
        fr.features = []
        fs = svo_amd.FeatureSelection(w, h, 30)
        n = fs.gradient_magnitude_with_ssc(fr, thr, num, bucket)
        px, resp, occ, nk = O.feature_select_ssc(img, thr, num, bucket, 30)
        assert n == len(px) and fs.last_keypoints == nk, (thr, num, bucket)
        np.testing.assert_array_equal(np.array([f.pixel_position for f in fr.features]).reshape(-1, 2), px)
        np.testing.assert_array_equal([f.gradient_magnitude for f in fr.features], resp)
        np.testing.assert_array_equal(fs.occupancy_grid, occ)
    fr.features = []
    fs = svo_amd.FeatureSelection(w, h, 30)
    n = fs.gradient_magnitude_by_value(fr, 50)
    px, resp, _ = O.feature_select_by_value(img, 50, 30)
    assert n == len(px)
    np.testing.assert_array_equal(np.array([f.pixel_position for f in fr.features]).reshape(-1, 2), px)
    fr.image_pyramid.clear()


def _real_pair(img, n_feat=2000, seed=3):
    """An ImageAlignment problem on the real texture: ref = last keyframe = the image at the identity pose,
    2000 textured features on a slanted plane (depth 8 .. 12 m), cur = the same image, aligned from a perturbed
    initial pose (the true motion is the identity)."""
    h, w = img.shape
    rng = np.random.default_rng(seed)
    px = _texture_points(img, n_feat, rng)
    fx = fy = 1000.0
    cx, cy = w / 2, h / 2
    v = np.stack([(px[:, 0] - cx) / fx, (px[:, 1] - cy) / fy, np.ones(len(px))], axis=1)
    bearing = v / np.linalg.norm(v, axis=1, keepdims=True)
    depth = 8.0 + 4.0 * px[:, 1] / h
    point = v * depth[:, None]  # camera = world at the identity pose
    ident = np.array([0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
    a = 0.003
    init = np.array([np.sin(a / 2) * 0.6, np.sin(a / 2) * 0.8, 0.0, np.cos(a / 2), 0.02, -0.015, 0.03])
    return types.SimpleNamespace(
        camera=dict(fx=fx, fy=fy, cx=cx, cy=cy, width=w, height=h), ref_img=img, kf_img=img, cur_img=img,
        ref_pose=ident, kf_pose=ident, cur_init_pose=init, n_ref=n_feat // 2, n_kf=n_feat - n_feat // 2,
        px=np.ascontiguousarray(px), bearing=np.ascontiguousarray(bearing), point=np.ascontiguousarray(point),
        has_point=np.ones(n_feat, np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_image_alignment_real_texture(name):
    import svo_amd
    s = _real_pair(_img(name))
    c = s.camera
    cam = svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])
    ps = svo_amd.PyramidSet(3, c["width"], c["height"], 5)
    ps.upload(0, np.stack([s.ref_img, s.kf_img, s.cur_img]))
    ps.build()
    b = svo_amd.AlignBatch(cam, 5, 0, 4, 1, len(s.px), median_mode=svo_amd.MEDIAN_REFERENCE)
    b.set_pair(0, (ps, 0), (ps, 1), (ps, 2), s.ref_pose, s.kf_pose, s.cur_init_pose, s.n_ref, s.n_kf, s.px,
               s.bearing, s.point, s.has_point)
    b.run()
    poses, err, st = b.results()
    pc, ec, stc, tr = oracle_align(s, 5, 0, 4, mode=0)
    assert st[0] == stc
    assert np.abs(canon(poses[0]) - canon(pc)).max() <= 1e-9
    assert abs(err[0] - ec) <= 1e-9 * ec
    g = b.traces(0)
    for l in range(5):
        assert (g[l].n_vis, g[l].status) == (tr[l].n_vis, tr[l].status), l
    # the first (coarsest) level's robust scale is the reference's own, bit for bit
    assert g[4].median == tr[4].median and g[4].mad == tr[4].mad, (g[4].median, tr[4].median)
    assert [t.scale_kernel for t in g] == [svo_amd.SCALE_K2V] * 5
