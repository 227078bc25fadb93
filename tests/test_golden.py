"""Golden fixtures (tests/golden/, written by tests/golden/make_golden*.py): the oracle must keep
reproducing them exactly (CPU), and the HIP path must match them within the parity tolerances (GPU)."""
import os

import numpy as np
import pytest

import oracle as O
from common import canon

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, name)))


def cam_of(d):
    fx, fy, cx, cy, w, h = d["camera"]
    return dict(fx=fx, fy=fy, cx=cx, cy=cy, width=int(w), height=int(h))


def oracle_pair(d, levels):
    pl = [O.build_pyramid(d[k], levels)[0] for k in ("ref_img", "kf_img", "cur_img")]
    return O.make_pair(pl[0], pl[1], pl[2], d["ref_pose"], d["kf_pose"], int(d["n_ref"]), int(d["n_kf"]), d["px"],
                       d["bearing"], d["point"], d["has_point"])


def test_synth_reproduces_golden_inputs():
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    s = make_golden.mini_pair()
    d = load("align_small.npz")
    for k in ("kf_img", "ref_img", "cur_img", "px", "bearing", "point", "has_point", "cur_init_pose", "ref_pose"):
        assert np.array_equal(s[k], d[k]), k


@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_reproduces_golden_alignment(mode):
    d = load("align_small.npz")
    L = int(d["levels"])
    pose, err, st, tr = O.image_align(cam_of(d), int(d["patch"]), 0, L - 1, oracle_pair(d, L), d["cur_init_pose"],
                                      median_mode=mode, trace=True)
    assert np.array_equal(pose, d[f"m{mode}_pose"]) and err == d[f"m{mode}_err"] and st == d[f"m{mode}_status"]
    assert [t.n_vis for t in tr] == list(d[f"m{mode}_trace_n_vis"])
    assert [t.sigma for t in tr] == list(d[f"m{mode}_trace_sigma"])


def test_oracle_reproduces_golden_pyramids():
    d = load("pyramid_small.npz")
    for k in ("ref_img", "kf_img", "cur_img"):
        img = d[f"{k}_stack"][:320 * 96].reshape(96, 320)
        i, g = O.build_pyramid(img, 4)
        assert np.array_equal(i, d[f"{k}_stack"]) and np.array_equal(g, d[f"{k}_grad"])


def test_oracle_reproduces_golden_feature_alignment():
    d = load("feature_small.npz")
    a = load("align_small.npz")
    px, err, st = O.feature_align(cam_of(a), int(d["patch"]), d["ref_grad"], d["cur_grad"], d["ref_px"], d["init_px"])
    assert np.array_equal(px, d["px"]) and np.array_equal(st, d["status"])
    assert np.array_equal(np.isnan(err), np.isnan(d["err"]))
    ok = ~np.isnan(err)
    assert np.array_equal(err[ok], d["err"][ok])


@pytest.mark.gpu
def test_gpu_matches_golden():
    import svo_amd
    d = load("align_small.npz")
    L = int(d["levels"])
    c = cam_of(d)
    camera = svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])
    ps = svo_amd.PyramidSet(3, c["width"], c["height"], 4)
    ps.upload(0, np.stack([d["ref_img"], d["kf_img"], d["cur_img"]]))
    ps.build()
    g = load("pyramid_small.npz")
    for i, k in enumerate(("ref_img", "kf_img", "cur_img")):
        for l, (hh, ww, off) in enumerate(O.level_shapes(c["width"], c["height"], 4)):
            assert np.array_equal(ps.download(i, l).ravel(), g[f"{k}_stack"][off:off + hh * ww])
            assert np.array_equal(ps.download(i, l, True).ravel(), g[f"{k}_grad"][off:off + hh * ww])
    # golden m0 = the reference's nth_element semantics (SVO_MEDIAN_REFERENCE), m1 = exact order statistics
    for gpu_mode, m in ((svo_amd.MEDIAN_REFERENCE, "m0"), (svo_amd.MEDIAN_EXACT, "m1")):
        b = svo_amd.AlignBatch(camera, int(d["patch"]), 0, L - 1, 1, len(d["px"]), median_mode=gpu_mode)
        b.set_pair(0, (ps, 0), (ps, 1), (ps, 2), d["ref_pose"], d["kf_pose"], d["cur_init_pose"], int(d["n_ref"]),
                   int(d["n_kf"]), d["px"], d["bearing"], d["point"], d["has_point"])
        b.run()
        pose, err, st = b.results()
        assert np.abs(canon(pose[0]) - canon(d[f"{m}_pose"])).max() <= 1e-9
        assert np.abs(canon(pose[0]) - canon(d["m0_pose"])).max() <= 1e-5
        assert abs(err[0] - d[f"{m}_err"]) <= 1e-9 * d[f"{m}_err"] and st[0] == d[f"{m}_status"]
        tr = b.traces(0)
        assert [t.n_vis for t in tr] == list(d[f"{m}_trace_n_vis"])
        assert [t.n_ref_vis for t in tr] == list(d[f"{m}_trace_n_ref_vis"])
    fd = load("feature_small.npz")
    ps2 = svo_amd.PyramidSet(2, c["width"], c["height"], 1)
    ps2.upload(0, np.stack([d["ref_img"], d["cur_img"]]))
    ps2.build()
    px = np.ascontiguousarray(fd["init_px"].copy())
    err, st = svo_amd.FeatureAlignment(7).align_batch(ps2, 0, ps2, 1, fd["ref_px"], px, camera)
    assert np.array_equal(px, fd["px"]) and np.array_equal(st, fd["status"])


# ---------------------------------------------------------------- FeatureSelection / pose BA fixtures
# (tests/golden/make_golden_select_ba.py)
def _sel():
    return load("select_small.npz")


def _ba():
    return load("pose_ba_small.npz")


def test_oracle_reproduces_golden_feature_selection():
    d = _sel()
    for name, bucket in (("b", True), ("nb", False)):
        px, resp, occ, nk = O.feature_select_ssc(d["img"], 40, 60, bucket, 16, d["occ"])
        np.testing.assert_array_equal(px, d[f"ssc_{name}_px"])
        np.testing.assert_array_equal(resp, d[f"ssc_{name}_resp"])
        np.testing.assert_array_equal(occ, d[f"ssc_{name}_occ"])
        assert nk == int(d[f"ssc_{name}_nk"])
    px, resp, _ = O.feature_select_by_value(d["img"], 40, 16, d["occ"])
    np.testing.assert_array_equal(px, d["val_px"])
    np.testing.assert_array_equal(resp, d["val_resp"])


def test_oracle_reproduces_golden_pose_ba():
    d = _ba()
    p1, e1, s1, v1 = O.optimize_pose(d["bearing"], d["point"], d["has_point"], [], d["init"])
    assert np.isnan(e1) and np.isnan(d["err1"]) and s1 == d["status1"]
    np.testing.assert_array_equal(p1, d["pose1"])
    np.testing.assert_array_equal(v1, d["vis1"])
    p2, e2, s2, v2 = O.optimize_pose(d["bearing"], d["point"], d["has_point"], v1, p1)
    assert e2 == d["err2"] and s2 == d["status2"]
    np.testing.assert_array_equal(p2, d["pose2"])


@pytest.mark.gpu
def test_gpu_matches_golden_feature_selection_and_pose_ba():
    import svo_amd
    d = _sel()
    h, w = d["img"].shape
    cam = svo_amd.PinholeCamera(w, h, 100.0, 100.0, w / 2, h / 2)
    for name, bucket in (("b", True), ("nb", False)):
        fr = svo_amd.Frame(cam, d["img"], 1)
        fs = svo_amd.FeatureSelection(w, h, 16)
        fs.occupancy_grid[:] = d["occ"]
        fs.gradient_magnitude_with_ssc(fr, 40, 60, bucket)
        np.testing.assert_array_equal(np.array([f.pixel_position for f in fr.features]).reshape(-1, 2),
                                      d[f"ssc_{name}_px"])
        np.testing.assert_array_equal([f.gradient_magnitude for f in fr.features], d[f"ssc_{name}_resp"])
        np.testing.assert_array_equal(fs.occupancy_grid, d[f"ssc_{name}_occ"])
    fr = svo_amd.Frame(cam, d["img"], 1)
    fs = svo_amd.FeatureSelection(w, h, 16)
    fs.occupancy_grid[:] = d["occ"]
    fs.gradient_magnitude_by_value(fr, 40)
    np.testing.assert_array_equal(np.array([f.pixel_position for f in fr.features]).reshape(-1, 2), d["val_px"])
    b = _ba()
    n = len(b["has_point"])
    vis = np.zeros(n, np.uint8)
    poses = b["init"].reshape(1, 7).copy()
    err, st = svo_amd.pose_optimize_batch([0, n], b["bearing"], b["point"], b["has_point"], vis, poses)
    assert np.isnan(err[0]) and st[0] == b["status1"]
    np.testing.assert_array_equal(vis, b["vis1"])
    np.testing.assert_allclose(poses[0], b["pose1"], atol=1e-12)
    err, st = svo_amd.pose_optimize_batch([0, n], b["bearing"], b["point"], b["has_point"], vis, poses)
    assert st[0] == b["status2"] and abs(err[0] - b["err2"]) <= 1e-12 * b["err2"]
    np.testing.assert_allclose(poses[0], b["pose2"], atol=1e-12)
