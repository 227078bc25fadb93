"""Depth filter (BASELINE config 5): DepthEstimator::updateFilters (src/depth_estimator.cpp:192-309).

CPU: the oracle's pieces against independent restatements (uint8-mean ZSAD, least-squares triangulation,
the MixedGaussianFilter init), its behaviour on a scene with a known answer (a plane at depth 10), and the
golden fixture (tests/golden/depth_small.npz, tests/golden/make_golden_depth.py).
GPU: the HIP path (svo_depth_update) against the oracle.  Tolerances: outcomes, survivor order and
candidate order bit-exact (the epipolar argmin is integer-exact); seed state and points 1e-12 relative
(acos / sin / exp of the device math library vs glibc may differ in the last bit).
"""
import os

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import oracle as O
import svo_amd.synth as synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "depth_small.npz")
FIELDS = ("a", "b", "mu", "sigma", "var", "max_depth", "px", "bearing", "kf", "valid")


def test_seed_init_formula():
    # src/mixed_gaussian_filter.cpp:7-24
    a, b, mu, sigma, var, md = O.depth_seed_init(12.5, 3.0)
    assert (a, b) == (10, 10) and mu == 1 / 12.5 and md == 1 / 3.0
    assert sigma == (1 / 3.0) / 6 and var == sigma * sigma


def np_zsad(ref, cur):
    """computeScore (src/algorithm.cpp:396-410) with Eigen's uint8 mean: (sum mod 256) / n in uint8."""
    n = len(ref)
    mr = (int(ref.astype(np.int64).sum()) % 256) // n
    mc = (int(cur.astype(np.int64).sum()) % 256) // n
    return float(np.abs((ref.astype(np.int64) - mr) - (cur.astype(np.int64) - mc)).sum())


def test_zsad_uint8_mean_quirk():
    ref = np.full(49, 200, np.uint8)   # sum 9800 = 72 mod 256 -> "mean" 1, not 200
    cur = np.full(49, 100, np.uint8)   # sum 4900 = 36 mod 256 -> "mean" 0
    assert O.zsad(ref, cur) == 49 * ((200 - 1) - (100 - 0))
    rng = np.random.default_rng(5)
    for _ in range(50):
        r, c = rng.integers(0, 256, 49, dtype=np.uint8), rng.integers(0, 256, 49, dtype=np.uint8)
        assert O.zsad(r, c) == np_zsad(r, c)


def test_triangulation_matches_least_squares():
    # depthFromTriangulation solves [R f_ref, -f_cur] (d1, d2) = -t in the least-squares sense
    rng = np.random.default_rng(9)
    for _ in range(40):
        q = Rotation.from_rotvec(rng.normal(0, 0.05, 3)).as_quat()  # x y z w
        t = rng.normal(0, 0.5, 3)
        P = np.array([rng.uniform(-3, 3), rng.uniform(-2, 2), rng.uniform(4, 30)])
        fr = P / np.linalg.norm(P)
        R = Rotation.from_quat(q).as_matrix()
        Pc = R @ P + t
        fc = Pc / np.linalg.norm(Pc) + rng.normal(0, 1e-4, 3)
        fc /= np.linalg.norm(fc)
        ok, d = O.depth_triangulate(np.concatenate([q, t]), fr, fc)
        A = np.stack([R @ fr, -fc], 1)
        sol = np.linalg.lstsq(A, -t, rcond=None)[0]
        assert ok and d == pytest.approx(abs(sol[0]), rel=1e-9)
    ok, _ = O.depth_triangulate(np.array([0, 0, 0, 1, 0, 0, 0.0]), np.array([0, 0, 1.0]), np.array([0, 0, 1.0]))
    assert not ok  # parallel rays: det(A^T A) = 0 < 1e-6


def test_plane_seeds_converge_to_the_plane():
    p = synth.make_shifted_plane()
    seeds = O.make_seeds(p.px, p.bearing, p.depth_mean, p.depth_min)
    surv, outcome, pts, cs = O.depth_update(p.camera, [p.kf_img], p.kf_pose[None], p.cur_img, p.cur_pose, seeds)
    assert np.all(outcome == 3) and len(surv) == 0
    assert list(cs) == list(range(len(seeds) - 1, -1, -1))  # candidates in the update loop's order
    assert np.abs(pts[:, 2] - 10.0).max() < 0.3             # within a scan step of the plane


def golden():
    d = dict(np.load(GOLD))
    fx, fy, cx, cy, w, h = d["camera"]
    cam = dict(fx=fx, fy=fy, cx=cx, cy=cy, width=int(w), height=int(h))

    def seeds(prefix):
        n = len(d[f"{prefix}_a"])
        s = np.zeros(n, O.DEPTH_SEED)
        for k in FIELDS:
            s[k] = d[f"{prefix}_{k}"]
        return s
    return d, cam, seeds("in"), seeds("out")


def test_oracle_reproduces_golden():
    d, cam, sin, sout = golden()
    surv, outcome, pts, cs = O.depth_update(cam, [d["kf_img"]], d["kf_pose"][None], d["cur_img"], d["cur_pose"], sin)
    assert set(np.unique(outcome)) >= {0, 1, 3}
    assert np.array_equal(outcome, d["outcome"]) and np.array_equal(cs, d["cand_seed"])
    assert np.array_equal(pts, d["cand_points"])
    for k in FIELDS:
        assert np.array_equal(surv[k], sout[k]), k


# ---------------------------------------------------------------- GPU parity
def gpu_update(cam, kf_img, kf_pose, cur_img, cur_pose, seeds):
    import svo_amd
    camera = svo_amd.PinholeCamera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"])
    ps = svo_amd.PyramidSet(2, cam["width"], cam["height"], 1)
    ps.upload(0, np.stack([kf_img, cur_img]))
    ps.build()
    s = np.zeros(len(seeds), svo_amd.DEPTH_SEED)
    for k in FIELDS:
        s[k] = seeds[k]
    return svo_amd.depth_update(camera, [(ps, 0, kf_pose)], (ps, 1), cur_pose, s)


def check_same(g, c):
    sg, og, pg, cg = g
    sc, oc, pc, cc = c
    assert np.array_equal(og, oc)
    assert np.array_equal(cg, cc)
    assert len(sg) == len(sc)
    for k in ("px", "bearing", "kf", "valid"):
        assert np.array_equal(sg[k], sc[k]), k
    for k in ("a", "b", "mu", "sigma", "var", "max_depth"):
        assert np.allclose(sg[k], sc[k], rtol=1e-12, atol=0), k
    assert np.allclose(pg, pc, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_gpu_matches_golden():
    d, cam, sin, _ = golden()
    g = gpu_update(cam, d["kf_img"], d["kf_pose"], d["cur_img"], d["cur_pose"], sin)
    c = O.depth_update(cam, [d["kf_img"]], d["kf_pose"][None], d["cur_img"], d["cur_pose"], sin)
    check_same(g, c)


@pytest.mark.gpu
def test_gpu_matches_oracle_config5():
    p = synth.make_depth_problem(n_seeds=2000)
    seeds = O.make_seeds(p.px, p.bearing, p.depth_mean, p.depth_min)
    g = gpu_update(p.camera, p.kf_img, p.kf_pose, p.cur_img, p.cur_pose, seeds)
    c = O.depth_update(p.camera, [p.kf_img], p.kf_pose[None], p.cur_img, p.cur_pose, seeds)
    check_same(g, c)
    # a wide prior: long epipolar scans (depth_min 10x smaller)
    seeds = O.make_seeds(p.px, p.bearing, p.depth_mean, p.depth_min / 10)
    g = gpu_update(p.camera, p.kf_img, p.kf_pose, p.cur_img, p.cur_pose, seeds)
    c = O.depth_update(p.camera, [p.kf_img], p.kf_pose[None], p.cur_img, p.cur_pose, seeds)
    check_same(g, c)


@pytest.mark.gpu
def test_gpu_depth_estimator_class_surface():
    import svo_amd
    p = synth.make_shifted_plane()
    cam = svo_amd.PinholeCamera(p.camera["width"], p.camera["height"], p.camera["fx"], p.camera["fy"], p.camera["cx"],
                                p.camera["cy"])
    kf = svo_amd.Frame(cam, p.kf_img, 1)
    kf.abs_pose[:] = p.kf_pose
    for i in range(len(p.px)):
        kf.add_feature(svo_amd.Feature(kf, p.px[i], bearing=p.bearing[i]))
    cur = svo_amd.Frame(cam, p.cur_img, 1)
    cur.abs_pose[:] = p.cur_pose
    de = svo_amd.DepthEstimator()
    de.add_keyframe(kf, p.depth_mean, p.depth_min)
    assert de.number_filters() == len(p.px)
    new = de.update_filters(cur)
    assert len(new) == len(p.px) and de.number_filters() == 0
    assert all(abs(pt.position[2] - 10.0) < 0.3 for _, pt in new)


@pytest.mark.gpu
@pytest.mark.parametrize("problem", ["config5", "plane"])
def test_gpu_cpp_mirror_depth_estimator(problem, tmp_path):
    """host/svo.hpp DepthEstimator (libsvo_host.so via build/svo_host_check depth): addKeyframe +
    updateFilters against the oracle: surviving filter count, candidate points in the reference's order
    (1e-12 relative, the device acos / sin / exp)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    p = synth.make_depth_problem(n_seeds=2000) if problem == "config5" else synth.make_shifted_plane()
    c = p.camera
    hdr = [c["fx"], c["fy"], c["cx"], c["cy"], c["width"], c["height"], *p.kf_pose, *p.cur_pose, p.depth_mean,
           p.depth_min, len(p.px)]
    data = np.concatenate([np.array(hdr, np.float64), np.concatenate([p.px, p.bearing], axis=1).ravel()])
    (tmp_path / "d.bin").write_bytes(data.astype(np.float64).tobytes())
    (tmp_path / "kf.raw").write_bytes(np.ascontiguousarray(p.kf_img).tobytes())
    (tmp_path / "cur.raw").write_bytes(np.ascontiguousarray(p.cur_img).tobytes())
    out = subprocess.run([exe, "depth", str(tmp_path / "d.bin"), str(tmp_path / "kf.raw"), str(tmp_path / "cur.raw")],
                         capture_output=True, text=True, timeout=60, check=True).stdout.splitlines()
    seeds = O.make_seeds(p.px, p.bearing, p.depth_mean, p.depth_min)
    surv, outc, pts, cs = O.depth_update(c, [p.kf_img], p.kf_pose[None], p.cur_img, p.cur_pose, seeds)
    assert out[0] == f"filters {len(surv)}"
    got = np.array([[float(v) for v in line.split()[1:]] for line in out[1:]]).reshape(-1, 3)
    assert got.shape == pts.shape
    np.testing.assert_allclose(got, pts, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_gpu_large_seed_set_pageable_staging():
    """80k seeds (10 MB of per-call data, past the context's 8 MB pinned staging block): the pageable
    staging path gives the oracle's answers."""
    p = synth.make_depth_problem(n_seeds=2000)
    seeds = O.make_seeds(p.px, p.bearing, p.depth_mean, p.depth_min)
    seeds = np.concatenate([seeds] * 40)
    g = gpu_update(p.camera, p.kf_img, p.kf_pose, p.cur_img, p.cur_pose, seeds)
    c = O.depth_update(p.camera, [p.kf_img], p.kf_pose[None], p.cur_img, p.cur_pose, seeds)
    check_same(g, c)
