"""Trajectory / feature-dump text formats: System::writeInFile
(src/system.cpp:635-640) and utils::write*/read* (src/utils.cpp:54-117).

The oracle streams through std::ostream with std::setprecision(6) and Eigen's IOFormat restated
(oracle/svo_oracle.cpp oracle_kitti_line / oracle_stream_g6): exactly the reference's output path.  The
product writes the same bytes through the C ABI (svo_format_kitti_pose), the Python mirror
(svo_amd.trajectory) and the C++ mirror (host/svo.hpp utils::writeInFile, driven by build/svo_host_check).
No GPU needed: these are host entry points of libsvo_hip.so.
"""
import io
import os
import subprocess

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import oracle as O
import svo_amd
from svo_amd import trajectory as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_CHECK = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "svo_host_check")


def poses(n, seed=0):
    rng = np.random.default_rng(seed)
    out = [np.array([0, 0, 0, 1, 0, 0, 0.0]), np.array([0, 0, 0, 1, 1e-9, -2.5e-7, 123456.789]),
           np.array([0, 0, 0, -1, -0.0, 0.0, 0.5])]
    for i in range(n):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        t = rng.normal(size=3) * 10.0 ** rng.integers(-8, 6)
        out.append(np.concatenate([q, t]))
    return out


def test_kitti_line_matches_oracle_stream():
    for p in poses(300):
        assert T.kitti_line(p) == O.kitti_line(p)


def test_matrix3x4_is_camera_to_world():
    for p in poses(50, seed=1):
        m = T.pose_matrix3x4_inverse(p)
        R = Rotation.from_quat(p[:4]).as_matrix()
        np.testing.assert_allclose(m[:, :3], R.T, atol=1e-14)
        np.testing.assert_allclose(m[:, 3], -R.T @ p[4:], rtol=1e-12, atol=1e-12 * max(1.0, np.abs(p[4:]).max()))


def test_g6_matches_ostream():
    rng = np.random.default_rng(2)
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 1e-5, 1e-4, 123456.5, 1234567.0, 999999.5, 0.1 + 0.2, float("inf"),
            float("-inf"), 2.0 ** -1074, 1.7976931348623157e308]
    vals += list(rng.normal(size=200) * 10.0 ** rng.integers(-12, 12, 200))
    vals += list(rng.integers(-5000, 5000, 50) / 2.0)
    for v in vals:
        assert T._g6(v) == O.stream_g6(v), v


def test_trajectory_round_trip_and_failed_lines():
    class F:
        pass
    buf = io.StringIO()
    ps = poses(20, seed=3)
    for i, p in enumerate(ps):
        if i % 7 == 3:
            T.write_failed(buf)
        f = F()
        f.abs_pose = p
        T.write_in_file(f, buf)
    lines = buf.getvalue().splitlines()
    assert lines.count("Failed") == 3
    back = T.read_trajectory(io.StringIO(buf.getvalue()))
    mats = [m for m in back if m is not None]
    assert len(mats) == len(ps) and back[3] is None
    for m, p in zip(mats, ps):
        want = T.pose_matrix3x4_inverse(p)
        np.testing.assert_allclose(m, want, rtol=5e-6, atol=1e-300)


def test_cpp_mirror_writes_the_same_lines():
    ps = poses(40, seed=4)
    stdin = "\n".join(" ".join(repr(float(x)) for x in p) for p in ps) + "\n"
    out = subprocess.run([HOST_CHECK, "io"], input=stdin, capture_output=True, text=True, check=True).stdout
    assert out.splitlines() == [O.kitti_line(p) for p in ps]


def test_feature_dump_format_and_reader_quirk():
    class Fr:
        def __init__(self):
            self.features = []

    class Ft:
        def __init__(self, px, point=None):
            self.pixel_position = np.asarray(px, np.float64)
            self.point = point

    rng = np.random.default_rng(5)
    ref, cur = Fr(), Fr()
    for i in range(25):
        pt = svo_amd.Point(rng.normal(size=3) * 20)
        ref.features.append(Ft(rng.uniform(0, 1241, 2), pt))
        cur.features.append(Ft(rng.uniform(0, 1241, 2)))
    a, b = io.StringIO(), io.StringIO()
    T.write_all_info_file(ref, cur, a)
    T.write_features_info_file(ref, cur, b)
    for i, line in enumerate(a.getvalue().splitlines()):
        r, c, p = ref.features[i].pixel_position, cur.features[i].pixel_position, ref.features[i].point.position
        assert line == " ".join(O.stream_g6(v) for v in (*r, *c, *p))
    assert [l.split()[:4] for l in a.getvalue().splitlines()] == [l.split() for l in b.getvalue().splitlines()]
    rp, cp, pts = T.read_all_info(io.StringIO(a.getvalue()))
    np.testing.assert_allclose(rp, [f.pixel_position for f in ref.features], rtol=5e-6)
    np.testing.assert_allclose(pts, [f.point.position for f in ref.features], rtol=5e-6)
    # readAllFromFile / readFeaturesFromFile clear first and then read numberObservation() == 0 lines
    T.read_all_from_file(ref, cur, io.StringIO(a.getvalue()))
    assert ref.features == [] and cur.features == []
    T.read_features_from_file(ref, cur, io.StringIO(b.getvalue()))
    assert ref.features == [] and cur.features == []


def test_errors_are_codes():
    with pytest.raises(svo_amd.SvoError):
        p = np.zeros(7)
        import ctypes
        from svo_amd._capi import check, lib, ptr
        check(lib().svo_format_kitti_pose(ptr(p), ctypes.create_string_buffer(8), 8))


@pytest.mark.gpu
def test_trajectory_row_on_gpu_box():
    """The same checks inside the GPU tier (the driver's -m gpu run on the MI355X box), so this §8(f) row is
    exercised with the GPU build of libsvo_hip.so / svo_host_check as the box loads it."""
    test_kitti_line_matches_oracle_stream()
    test_matrix3x4_is_camera_to_world()
    test_g6_matches_ostream()
    test_cpp_mirror_writes_the_same_lines()
    test_feature_dump_format_and_reader_quirk()
    test_errors_are_codes()
