"""FeatureSelection: gradientMagnitudeWithSSC / gradientMagnitudeByValue
(src/feature_selection.cpp:19-287).

CPU: the oracle restatement (oracle/feature_selection_oracle.cpp) against independent pure-Python
restatements of each step — threshold in row-major order, SSC's binary search (:166-248), the bucketing
(:60-76) and the per-cell first maximum (:91-143) — with the keypoint order taken from libstdc++'s
std::sort (oracle.sort_responses: the toolchain function itself, like std::nth_element for the median).
GPU: svo_amd.FeatureSelection (device detection + host sort/SSC, device per-cell maxima) against the
oracle: the same features (pixel, response) in the same addFeature order, the same occupancy grid after.
"""
import math

import numpy as np
import pytest

import oracle as O
import svo_amd.synth as synth


# ---------------------------------------------------------------- independent restatements
def py_ssc(xs, ys, num_ret, cols, rows, tolerance=0.1):
    """FeatureSelection::SSC (src/feature_selection.cpp:166-248), written from the reference text."""
    f32 = np.float32
    exp1 = rows + cols + 2 * num_ret
    exp2 = 4 * cols + 4 * num_ret + 4 * rows * num_ret + rows * rows + cols * cols - 2 * rows * cols + \
        4 * rows * cols * num_ret
    exp3 = math.sqrt(float(exp2))
    exp4 = float(2 * (num_ret - 1))
    sol1 = -float(round_half_away((exp1 + exp3) / exp4))
    sol2 = -float(round_half_away((exp1 - exp3) / exp4))
    high = int(sol1) if sol1 > sol2 else int(sol2)
    low = int(math.sqrt(len(xs) / num_ret))
    K = f32(num_ret)
    kmin = int(round_half_away(float(f32(K - f32(K * f32(tolerance))))))
    kmax = int(round_half_away(float(f32(K + f32(K * f32(tolerance))))))
    prev_w, result = -1, []
    while True:
        width = low + (high - low) // 2
        if width == prev_w or low > high or width <= 0:
            return result
        res = []
        c = width / 2.0
        ncc, ncr = int(cols / c), int(rows / c)
        covered = np.zeros((ncr + 1, ncc + 1), bool)
        k = int(width / c)
        for i in range(len(xs)):
            row, col = int(float(f32(ys[i])) / c), int(float(f32(xs[i])) / c)
            if not covered[row, col]:
                res.append(i)
                covered[max(row - k, 0):min(row + k, ncr) + 1, max(col - k, 0):min(col + k, ncc) + 1] = True
        result = res
        if kmin <= len(res) <= kmax:
            return res
        if len(res) < kmin:
            high = width - 1
        else:
            low = width + 1
        prev_w = width


def round_half_away(x):  # std::round
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def abs_gradient(img):
    g = np.zeros(img.shape, np.int32)
    i = img.astype(np.int32)
    g[1:-1, 1:-1] = np.abs(i[1:-1, 2:] - i[1:-1, :-2]) + np.abs(i[2:, 1:-1] - i[:-2, 1:-1])
    return np.minimum(g, 255).astype(np.uint8)


def py_select_ssc(img, thr, num, bucketing, cell, occ):
    mag = abs_gradient(img)
    h, w = img.shape
    ys, xs = np.nonzero(mag > thr)  # row-major (:38-50)
    resp = mag[ys, xs]
    perm = O.sort_responses(resp)
    assert np.all(np.diff(resp[perm].astype(int)) <= 0)
    xs, ys, resp = xs[perm], ys[perm], resp[perm]
    sel = py_ssc(xs, ys, num, w, h)
    occ = occ.copy()
    px, out = [], []
    for i in sel:
        if bucketing:
            r, c = ys[i] // cell, xs[i] // cell
            if occ[r, c]:
                continue
            occ[r, c] = 1
        px.append((xs[i], ys[i]))
        out.append(resp[i])
    if bucketing:
        occ[:] = 0
    return np.array(px, np.float64).reshape(-1, 2), np.array(out, np.float64), occ, len(xs)


def py_by_value(img, thr, cell, occ):
    mag = abs_gradient(img)
    h, w = img.shape
    px, resp = [], []
    for r in range(h // cell + 1):
        for c in range(w // cell + 1):
            if occ[r, c]:
                continue
            blk = mag[r * cell:min((r + 1) * cell, h), c * cell:min((c + 1) * cell, w)]
            if blk.size == 0 or blk.max() <= thr:
                continue
            i, j = np.unravel_index(int(np.argmax(blk)), blk.shape)  # first maximum, row-major
            px.append((c * cell + j, r * cell + i))
            resp.append(blk[i, j])
    return np.array(px, np.float64).reshape(-1, 2), np.array(resp, np.float64)


def textured(seed, w, h, frac_flat=0.0):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (h // 4 + 1, w // 4 + 1)).astype(np.uint8)
    img = np.kron(img, np.ones((4, 4), np.uint8))[:h, :w]
    img = (img.astype(np.int32) + rng.integers(-6, 7, (h, w))).clip(0, 255).astype(np.uint8)
    if frac_flat:
        img[:, : int(w * frac_flat)] = 90
    return np.ascontiguousarray(img)


# ---------------------------------------------------------------- CPU: oracle pinned
def test_oracle_gradient_matches_pyramid_gradient():
    img = textured(1, 97, 61)
    np.testing.assert_array_equal(abs_gradient(img), O.build_pyramid(img, 1)[1][: 97 * 61].reshape(61, 97))


@pytest.mark.parametrize("seed,n,num,cols,rows", [(0, 500, 50, 200, 120), (1, 3000, 200, 1241, 376),
                                                  (2, 40, 30, 64, 48), (3, 5, 200, 100, 100), (4, 0, 10, 50, 50),
                                                  (5, 2000, 2, 320, 96)])
def test_ssc_matches_python_restatement(seed, n, num, cols, rows):
    rng = np.random.default_rng(seed)
    xs = rng.integers(0, cols, n).astype(np.float32)
    ys = rng.integers(0, rows, n).astype(np.float32)
    np.testing.assert_array_equal(O.ssc(xs, ys, num, cols, rows), np.array(py_ssc(xs, ys, num, cols, rows), np.int32))


def test_ssc_known_answer():
    # 4 points far apart: radius search ends with every point kept (fewer than Kmin = 9 at num 10)
    xs = np.array([0, 90, 0, 90], np.float32)
    ys = np.array([0, 0, 90, 90], np.float32)
    assert list(O.ssc(xs, ys, 10, 100, 100)) == [0, 1, 2, 3]
    # the same pixel twice: the second is always covered by the first
    assert list(O.ssc(np.array([5, 5], np.float32), np.array([5, 5], np.float32), 2, 100, 100)) == [0]


@pytest.mark.parametrize("seed,w,h,thr,num,bucket,cell", [(0, 160, 96, 50, 60, True, 16), (1, 160, 96, 50, 60, False, 16),
                                                          (2, 97, 61, 30, 20, True, 30), (3, 128, 64, 254, 10, True, 8),
                                                          (4, 200, 80, 80, 200, True, 30)])
def test_oracle_select_ssc_matches_python(seed, w, h, thr, num, bucket, cell):
    img = textured(seed, w, h, frac_flat=0.3)
    occ = np.zeros((h // cell + 1, w // cell + 1), np.uint8)
    occ[0, 0] = occ[-1, -1] = 1  # setExistingFeatures
    got = O.feature_select_ssc(img, thr, num, bucket, cell, occ)
    want = py_select_ssc(img, thr, num, bucket, cell, occ)
    for g, e in zip(got, want):
        np.testing.assert_array_equal(g, e)


@pytest.mark.parametrize("seed,w,h,thr,cell", [(0, 160, 96, 50, 16), (1, 97, 61, 30, 30), (2, 120, 60, 40, 30),
                                               (3, 64, 64, 255, 8)])
def test_oracle_by_value_matches_python(seed, w, h, thr, cell):
    img = textured(seed, w, h, frac_flat=0.4)
    occ = np.zeros((h // cell + 1, w // cell + 1), np.uint8)
    occ[1, 1] = 1
    px, resp, occ_after = O.feature_select_by_value(img, thr, cell, occ)
    epx, eresp = py_by_value(img, thr, cell, occ)
    np.testing.assert_array_equal(px, epx)
    np.testing.assert_array_equal(resp, eresp)
    assert not occ_after.any()


# ---------------------------------------------------------------- GPU parity
def _frame(img, ctx=None):
    import svo_amd
    h, w = img.shape
    cam = svo_amd.PinholeCamera(w, h, 300.0, 300.0, w / 2, h / 2)
    return svo_amd.Frame(cam, img, 1, ctx=ctx)


def _kitti_images(n):
    return [synth.make_pair(seed=synth.SEED_BASE + i, n_features=10).ref_img for i in range(n)]


@pytest.mark.gpu
def test_gpu_detect_keys_row_major():
    import svo_amd
    for img in [textured(7, 1241, 376), textured(8, 97, 61), textured(9, 17, 5)]:
        fr = _frame(img)
        fs = svo_amd.FeatureSelection(img.shape[1], img.shape[0], 30)
        for thr in (0, 50, 254, 255):
            keys = fs.detect(fr, thr)
            mag = abs_gradient(img).ravel()
            idx = np.nonzero(mag > thr)[0]
            want = (mag[idx].astype(np.uint32) << 24) | idx.astype(np.uint32)
            np.testing.assert_array_equal(keys, want)


@pytest.mark.gpu
@pytest.mark.parametrize("thr,num,bucket", [(50, 200, True), (50, 200, False), (30, 1000, True), (254, 200, True),
                                            (255, 200, True), (50, 2, False)])
def test_gpu_select_ssc_matches_oracle(thr, num, bucket):
    import svo_amd
    for img in _kitti_images(2) + [textured(11, 1241, 376, 0.5)]:
        fr = _frame(img)
        fs = svo_amd.FeatureSelection(1241, 376, 30)
        existing = [svo_amd.Feature(fr, np.array([15.5, 20.0])), svo_amd.Feature(fr, np.array([1240.0, 375.0]))]
        fs.set_existing_features(existing)
        occ0 = fs.occupancy_grid.copy()
        n = fs.gradient_magnitude_with_ssc(fr, thr, num, bucket)
        px, resp, occ, nk = O.feature_select_ssc(img, thr, num, bucket, 30, occ0)
        assert n == len(px) and fs.last_keypoints == nk
        got = np.array([f.pixel_position for f in fr.features]).reshape(-1, 2)
        np.testing.assert_array_equal(got, px)
        np.testing.assert_array_equal([f.gradient_magnitude for f in fr.features], resp)
        np.testing.assert_array_equal(fs.occupancy_grid, occ)


@pytest.mark.gpu
@pytest.mark.parametrize("thr,cell", [(50, 30), (0, 16), (120, 7), (255, 30)])
def test_gpu_by_value_matches_oracle(thr, cell):
    import svo_amd
    for img in _kitti_images(1) + [textured(12, 1241, 376, 0.3), textured(13, 90, 60)]:
        h, w = img.shape
        fr = _frame(img)
        fs = svo_amd.FeatureSelection(w, h, cell)
        fs.set_cell_in_grid_occupancy((cell * 1.5, 0.0))
        occ0 = fs.occupancy_grid.copy()
        n = fs.gradient_magnitude_by_value(fr, thr)
        px, resp, occ = O.feature_select_by_value(img, thr, cell, occ0)
        got = np.array([f.pixel_position for f in fr.features]).reshape(-1, 2)
        assert n == len(px)
        np.testing.assert_array_equal(got, px)
        np.testing.assert_array_equal([f.gradient_magnitude for f in fr.features], resp)
        assert not fs.occupancy_grid.any()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fs", "fv"])
def test_gpu_cpp_mirror_matches_oracle(mode, tmp_path):
    """host/svo.hpp FeatureSelection (libsvo_host.so, via build/svo_host_check) against the oracle."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    img = _kitti_images(1)[0]
    raw = tmp_path / "img.raw"
    raw.write_bytes(img.tobytes())
    h, w = img.shape
    if mode == "fs":
        args = [exe, "fs", str(w), str(h), "30", "50", "200", "1", str(raw), "15.5", "20", "600", "200"]
        occ = np.zeros((h // 30 + 1, w // 30 + 1), np.uint8)
        occ[0, 0] = occ[200 // 30, 600 // 30] = 1
        px, resp, _, _ = O.feature_select_ssc(img, 50, 200, True, 30, occ)
    else:
        args = [exe, "fv", str(w), str(h), "30", "50", str(raw)]
        px, resp, _ = O.feature_select_by_value(img, 50, 30)
    out = subprocess.run(args, capture_output=True, text=True, timeout=60, check=True).stdout
    got = np.array([[float(v) for v in line.split()] for line in out.splitlines()]).reshape(-1, 3)
    np.testing.assert_array_equal(got[:, :2], px)
    np.testing.assert_array_equal(got[:, 2], resp)


def test_host_sort_is_libstdcxx_std_sort(tmp_path):
    """svo::feature_sort_keys (a threaded restatement of libstdc++'s introsort + a counting pass for its
    stable final insertion sort) gives std::sort's exact permutation: tests/cpp/sort_check.cpp, 112 inputs
    (ties, sorted, reversed, all equal; sizes 0 - 150000, past the threading threshold)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    build = os.path.join(root, "semi-direct-visual-odometry_amd", "build")
    exe = str(tmp_path / "sort_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(root, "tests", "cpp", "sort_check.cpp"),
                    "-L" + build, "-lsvo_hip", "-Wl,-rpath," + build], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
