"""Pins the CPU oracle (oracle/svo_oracle.cpp) to known answers.

The reference cannot be built here, so the oracle is pinned by
  * the reference's own known-answer test of the projection (tests/test_camera.cpp:94-95) and its image
    pyramid structure tests (tests/test_image_pyramid.cpp:27-60), and
  * independent restatements of the third-party arithmetic it relies on: numpy integer pyrDown /
    abs-gradient (OpenCV, Simd), scipy rotations / matrix exponential (Sophus), numpy.linalg.solve
    (Eigen LDLT), finite differences of the projection (the 2x6 image Jacobian of python/symbol.py:50-60),
    sorted order statistics (std::nth_element).
"""
import numpy as np
import pytest
from scipy.linalg import expm
from scipy.spatial.transform import Rotation

import oracle as O


def test_project2d_reference_kat():
    # tests/test_camera.cpp:84-95: fx=30.3 fy=40.4 cx=325.5 cy=248.8, point (17.7, 28.8, 39.9)
    cam = dict(fx=30.3, fy=40.4, cx=325.5, cy=248.8, width=640, height=480)
    uv = O.project2d(cam, [17.7, 28.8, 39.9])
    assert uv[0] == pytest.approx(338.9413533834586466165, rel=4e-16, abs=0)
    assert uv[1] == pytest.approx(277.9609022556390977443, rel=4e-16, abs=0)


def np_pyr_down(img):
    """cv::pyrDown restated in numpy: 5x5 binomial, BORDER_REFLECT_101, (s + 128) >> 8."""
    h, w = img.shape
    k = np.array([1, 4, 6, 4, 1], np.int64)
    p = np.pad(img.astype(np.int64), 2, mode="reflect")  # numpy 'reflect' == OpenCV REFLECT_101
    rows = sum(k[i] * p[i:i + h, :] for i in range(5))
    full = sum(k[j] * rows[:, j:j + w] for j in range(5))
    return ((full[::2, ::2] + 128) >> 8).astype(np.uint8)


def np_abs_grad(img):
    g = np.zeros_like(img)
    i = img.astype(np.int32)
    dx = np.abs(i[1:-1, 2:] - i[1:-1, :-2])
    dy = np.abs(i[2:, 1:-1] - i[:-2, 1:-1])
    g[1:-1, 1:-1] = np.minimum(dx + dy, 255)
    return g


@pytest.mark.parametrize("shape", [(376, 1241), (37, 101), (64, 64), (11, 6), (480, 640)])
def test_pyramid_vs_numpy(shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    levels = 4 if min(shape) > 16 else 2
    oi, og = O.build_pyramid(img, levels)
    li = O.unpack_levels(oi, shape[1], shape[0], levels)
    lg = O.unpack_levels(og, shape[1], shape[0], levels)
    ref_i, ref_g = img, np_abs_grad(img)
    for l in range(levels):
        assert np.array_equal(li[l], ref_i), ("image", l)
        assert np.array_equal(lg[l], ref_g), ("gradient", l)
        ref_i, ref_g = np_pyr_down(ref_i), np_pyr_down(ref_g)


def test_pyramid_structure_reference_tests():
    # tests/test_image_pyramid.cpp:27-60 on a random 640x480 image: level count, base image equality, sizes
    img = np.random.default_rng(0).integers(0, 256, (480, 640), dtype=np.uint8)
    oi, _ = O.build_pyramid(img, 4)
    levels = O.unpack_levels(oi, 640, 480, 4)
    assert len(levels) == 4
    assert np.array_equal(levels[0], img)
    assert [l.shape for l in levels] == [(480, 640), (240, 320), (120, 160), (60, 80)]


def se3_matrix(p):
    T = np.eye(4)
    T[:3, :3] = Rotation.from_quat(p[:4]).as_matrix()
    T[:3, 3] = p[4:]
    return T


def hat6(a):
    v, w = a[:3], a[3:]
    X = np.zeros((4, 4))
    X[:3, :3] = [[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]
    X[:3, 3] = v
    return X


@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e-7, 1e-12, 0.0])
def test_se3_exp_vs_expm(scale):
    rng = np.random.default_rng(3)
    for _ in range(20):
        a = rng.normal(size=6) * scale
        p = O.se3_exp(a)
        assert abs(np.linalg.norm(p[:4]) - 1.0) < 1e-15
        assert np.allclose(se3_matrix(p), expm(hat6(a)), atol=1e-14, rtol=0)
        if scale > 0:
            q = Rotation.from_rotvec(a[3:]).as_quat()
            q = q if np.dot(q, p[:4]) >= 0 else -q
            assert np.allclose(p[:4], q, atol=1e-15)


def test_se3_compose_vs_matrices():
    rng = np.random.default_rng(4)
    for _ in range(20):
        a, b = O.se3_exp(rng.normal(size=6)), O.se3_exp(rng.normal(size=6))
        c = O.se3_compose(a, b)
        assert np.allclose(se3_matrix(c), se3_matrix(a) @ se3_matrix(b), atol=1e-14)


@pytest.mark.parametrize("n", [6, 3])
def test_ldlt_vs_numpy(n):
    rng = np.random.default_rng(n)
    for _ in range(50):
        A = rng.normal(size=(3 * n, n))
        H = A.T @ A + 1e-3 * np.eye(n)
        b = rng.normal(size=n)
        x = O.ldlt_solve(H, b)
        assert np.allclose(x, np.linalg.solve(H, b), rtol=1e-9, atol=1e-12)
    assert np.array_equal(O.ldlt_solve(np.zeros((n, n)), np.ones(n)), np.zeros(n))  # H = 0 -> D^+ = 0 -> dx = 0


def test_ldlt_reads_lower_triangle_only():
    rng = np.random.default_rng(9)
    A = rng.normal(size=(12, 6))
    H = A.T @ A + np.eye(6)
    b = rng.normal(size=6)
    Hu = H.copy()
    Hu[np.triu_indices(6, 1)] = 1e9  # garbage above the diagonal
    assert np.array_equal(O.ldlt_solve(Hu, b), O.ldlt_solve(H, b))


def test_image_jacobian_finite_difference():
    # d/dxi pi(exp(xi) X) at xi = 0 (left perturbation), the 2x6 of python/symbol.py:50-60
    fx, fy = 721.5377, 700.0
    X = np.array([1.3, -0.7, 9.0])
    J = O.image_jac(X, fx, fy)
    proj = lambda P: np.array([fx * P[0] / P[2], fy * P[1] / P[2]])
    eps = 1e-6
    for k in range(6):
        d = np.zeros(6)
        d[k] = eps
        num = (proj((expm(hat6(d)) @ np.append(X, 1))[:3]) - proj((expm(hat6(-d)) @ np.append(X, 1))[:3])) / (2 * eps)
        assert np.allclose(J[:, k], num, rtol=1e-6, atol=1e-6), k


def test_median_semantics():
    rng = np.random.default_rng(5)
    DMAX = np.finfo(np.float64).max
    for M in (49, 50, 1001, 1000):
        for _ in range(20):
            v = rng.normal(0, 8, M)
            inv = rng.random(M) < 0.2
            v[inv] = DMAX
            n = int((~inv).sum())
            s = np.sort(v)
            mid = n // 2
            exact = s[mid] if M % 2 else (s[mid - 1] + s[mid]) / 2
            assert O.median(v, n, mode=1) == exact
            ref = O.median(v, n, mode=0)  # libstdc++: v[mid] exact, v[mid-1] any element <= v[mid]
            if M % 2:
                assert ref == s[mid]
            else:
                assert s[0] <= 2 * ref - s[mid] <= s[mid] + 1e-12
    assert O.median(np.full(10, DMAX), 0, 1) == DMAX  # nothing visible (mid == 0): vec[mid]


def test_bilinear_known_answers():
    img = np.array([[10, 20, 30], [40, 50, 60], [70, 80, 90]], np.uint8)
    assert O.bilinear_d(img, 1.0, 1.0) == 50.0
    assert O.bilinear_d(img, 0.5, 0.0) == 15.0
    assert O.bilinear_d(img, 0.25, 0.75) == 0.75 * (0.75 * 40 + 0.25 * 50) + 0.25 * (0.75 * 10 + 0.25 * 20)
    x, y = 0.1234567891, 1.3333333333
    a = np.float32((1 - x) * 40 + x * 50)
    b = np.float32((1 - x) * 70 + x * 80)
    want = np.float32((2 - y) * np.float64(a) + (y - 1) * np.float64(b))
    assert O.bilinear_f(img, x, y) == want  # float-rounded row blends (src/algorithm.cpp:885-894)


def test_oracle_robust_scale_on_flat_blocks():
    """Exact integer residuals (flat squares, synth.make_flat_blocks): the oracle's level trace holds the
    exact order statistics, including the even-length median that lies below its histogram bin."""
    import svo_amd.synth as synth
    from common import oracle_align
    for groups, med, mad in [({2: 7, 7: 4, 15: 5, 24: 6}, 11.0, 9.0), ({-5: 3, 5: 3}, 0.0, 5.0)]:
        s = synth.make_flat_blocks(groups)
        _, _, _, tr = oracle_align(s, 5, 0, 0, mode=1)
        assert (tr[0].n_vis, tr[0].median, tr[0].mad) == (25 * sum(groups.values()), med, mad)


def test_image_jac_vs_reference_sympy():
    """The oracle's 2x6 image Jacobian against the reference's own sympy derivation (python/symbol.py:50-60,
    `final = first * second`, lambdified by tests/golden/make_golden_symbol.py into symbol_jac.npz) and the
    reference formula (src/image_alignment.cpp:235-247): equal to within 2 ulp (sympy's expression tree
    orders some products differently: fx + fx*x**2/z2 vs (fx*x2)/z2 + fx)."""
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "symbol_jac.npz"))
    for (fx, fy, x, y, z), ref in zip(d["inputs"], d["jac"]):
        got = O.image_jac([x, y, z], fx, fy)
        assert got[0, 1] == 0.0 and got[1, 0] == 0.0 and ref[0, 1] == 0.0 and ref[1, 0] == 0.0
        scale = np.maximum(np.abs(ref), 1e-300)
        assert (np.abs(got - ref) / scale).max() <= 2 * np.finfo(np.float64).eps, (fx, fy, x, y, z)


def test_inverse_projection_round_trip():
    """tests/test_camera.cpp:97-102: inverse projection of the projected KAT point recovers the point within
    testMaxError = 1e-12 (:8).  The test is written against an older z-normalised invProject2d; the current
    PinholeCamera::inverseProject2d (src/pinhole_camera.cpp:81-101) returns the unit bearing, so the point is
    the bearing scaled by |P| (and the z-normalised form bearing / bearing.z * z)."""
    cam = dict(fx=30.3, fy=40.4, cx=325.5, cy=248.8, width=640, height=480)
    P = np.array([17.7, 28.8, 39.9])
    b = O.inverse_project2d(cam, O.project2d(cam, P))
    assert abs(np.linalg.norm(b) - 1.0) <= 1e-15
    np.testing.assert_allclose(b * np.linalg.norm(P), P, rtol=0, atol=1e-12)
    np.testing.assert_allclose(b / b[2] * P[2], P, rtol=0, atol=1e-12)
