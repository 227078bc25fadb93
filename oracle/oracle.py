"""ctypes wrapper for the CPU oracle (oracle/svo_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / CPU baseline.  The product path never imports this module.

Parity status: partially pinned.  The reference cannot be compiled here (OpenCV, Eigen, Sophus, g2o
and the prebuilt Simd/CHOLMOD libraries are absent), so the restatement is pinned by
(i) the reference's own known-answer test for the projection (tests/test_camera.cpp:94-95) and its
pyramid structure tests (tests/test_image_pyramid.cpp:27-60), and (ii) independent restatements of the
third-party arithmetic (numpy pyrDown / abs-gradient, scipy rotations for SE3 exp, numpy solve for
LDLT, real libstdc++ nth_element) — see tests/test_oracle_kats.py.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsvo_oracle.so")
_lib = None


class OcCamera(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_double), ("fy", ctypes.c_double), ("cx", ctypes.c_double), ("cy", ctypes.c_double),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32)]


class OcPair(ctypes.Structure):
    _fields_ = [("ref_pyr", ctypes.c_void_p), ("kf_pyr", ctypes.c_void_p), ("cur_pyr", ctypes.c_void_p),
                ("ref_pose", ctypes.c_double * 7), ("kf_pose", ctypes.c_double * 7),
                ("n_ref", ctypes.c_int32), ("n_kf", ctypes.c_int32),
                ("px", ctypes.c_void_p), ("bearing", ctypes.c_void_p), ("point", ctypes.c_void_p),
                ("has_point", ctypes.c_void_p)]


class LevelTrace(ctypes.Structure):
    _fields_ = [("level", ctypes.c_int32), ("n_ref_vis", ctypes.c_int32), ("n_vis", ctypes.c_int32),
                ("status", ctypes.c_int32), ("median", ctypes.c_double), ("mad", ctypes.c_double),
                ("sigma", ctypes.c_double), ("chi2", ctypes.c_double), ("lambda_", ctypes.c_double),
                ("err", ctypes.c_double), ("H", ctypes.c_double * 36), ("g", ctypes.c_double * 6),
                ("dx", ctypes.c_double * 6)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_NATIVE_PATH = os.path.join(_HERE, "build", "native", "libsvo_oracle.so")
_native = None


def native_lib(timeout=300):
    """The same restatement built for this host's CPU (make native: -O3 -DNDEBUG -march=native, FMA contraction
    allowed): the CPU BASELINE build (BASELINE.md's Release flags), built on first use.  Only bench.py's
    cpu_baseline times it; the parity checker stays the contraction-free lib().  None if it cannot be built."""
    global _native
    if _native is None:
        try:
            subprocess.run(["make", "-s", "-C", _HERE, "native"], check=True, timeout=timeout,
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            _native = _load(_NATIVE_PATH)
        except (OSError, subprocess.SubprocessError):
            return None
    return _native


def _load(path):
    L = ctypes.CDLL(path)
    L.oracle_pyramid_bytes.restype = ctypes.c_int64
    L.oracle_image_align.restype = ctypes.c_double
    L.oracle_median.restype = ctypes.c_double
    L.oracle_median.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32]
    assert L.oracle_level_trace_size() == ctypes.sizeof(LevelTrace)
    return L


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_pyramid_bytes.restype = ctypes.c_int64
        L.oracle_image_align.restype = ctypes.c_double
        L.oracle_median.restype = ctypes.c_double
        L.oracle_median.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32]
        L.oracle_bilinear_d.restype = ctypes.c_double
        L.oracle_bilinear_d.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double]
        L.oracle_bilinear_f.restype = ctypes.c_float
        L.oracle_bilinear_f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double]
        assert L.oracle_level_trace_size() == ctypes.sizeof(LevelTrace)
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def camera(cam):
    return OcCamera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["width"], cam["height"])


def pyramid_bytes(w, h, levels):
    return lib().oracle_pyramid_bytes(w, h, levels)


def build_pyramid(img, levels):
    """ImagePyramid::createImagePyramid -> (packed image stack, packed gradient stack)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    n = pyramid_bytes(w, h, levels)
    out_i = np.zeros(n, np.uint8)
    out_g = np.zeros(n, np.uint8)
    lib().oracle_build_pyramid(_p(img), w, h, levels, _p(out_i), _p(out_g))
    return out_i, out_g


def level_shapes(w, h, levels):
    shapes, off = [], 0
    for _ in range(levels):
        shapes.append((h, w, off))
        off += w * h
        w, h = (w + 1) // 2, (h + 1) // 2
    return shapes


def unpack_levels(packed, w, h, levels):
    return [packed[o:o + hh * ww].reshape(hh, ww) for hh, ww, o in level_shapes(w, h, levels)]


def project2d(cam, p3):
    out = np.zeros(2)
    p3 = np.ascontiguousarray(p3, dtype=np.float64)
    lib().oracle_project2d(ctypes.byref(camera(cam)), _p(p3), _p(out))
    return out


def inverse_project2d(cam, uv):
    out = np.zeros(3)
    uv = np.ascontiguousarray(uv, dtype=np.float64)
    lib().oracle_inverse_project2d(ctypes.byref(camera(cam)), _p(uv), _p(out))
    return out


def se3_exp(tangent):
    t = np.ascontiguousarray(tangent, dtype=np.float64)
    out = np.zeros(7)
    lib().oracle_se3_exp(_p(t), _p(out))
    return out


def se3_compose(a, b):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    out = np.zeros(7)
    lib().oracle_se3_compose(_p(a), _p(b), _p(out))
    return out


def ldlt_solve(H, b):
    H = np.ascontiguousarray(H, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(len(b))
    lib().oracle_ldlt_solve(len(b), _p(H), _p(b), _p(x))
    return x


def image_jac(p3, fx, fy):
    p3 = np.ascontiguousarray(p3, dtype=np.float64)
    out = np.zeros((2, 6))
    lib().oracle_image_jac(_p(p3), ctypes.c_double(fx), ctypes.c_double(fy), _p(out))
    return out


def median(v, n_valid, mode=0):
    v = np.ascontiguousarray(v, dtype=np.float64)
    return lib().oracle_median(_p(v), len(v), n_valid, mode)


def bilinear_d(img, x, y):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return lib().oracle_bilinear_d(_p(img), img.shape[1], img.shape[0], x, y)


def bilinear_f(img, x, y):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return lib().oracle_bilinear_f(_p(img), img.shape[1], img.shape[0], x, y)


class _PairKeep:
    """Keeps numpy buffers alive while an OcPair points into them."""

    def __init__(self, pair, keep):
        self.pair = pair
        self.keep = keep


def make_pair(ref_pyr, kf_pyr, cur_pyr, ref_pose, kf_pose, n_ref, n_kf, px, bearing, point, has_point):
    keep = [np.ascontiguousarray(a) for a in (ref_pyr, kf_pyr, cur_pyr)]
    feats = [np.ascontiguousarray(px, np.float64), np.ascontiguousarray(bearing, np.float64),
             np.ascontiguousarray(point, np.float64), np.ascontiguousarray(has_point, np.uint8)]
    P = OcPair()
    P.ref_pyr, P.kf_pyr, P.cur_pyr = (_p(a).value for a in keep)
    P.ref_pose[:] = list(ref_pose)
    P.kf_pose[:] = list(kf_pose)
    P.n_ref, P.n_kf = int(n_ref), int(n_kf)
    P.px, P.bearing, P.point, P.has_point = (_p(a).value for a in feats)
    return _PairKeep(P, keep + feats)


def image_align(cam, patch, min_level, max_level, pair, cur_pose, median_mode=0, trace=False, L=None):
    """ImageAlignment::align.  Returns (pose[7], err, status, traces or None).  L: another build of the
    oracle library (native_lib()), default lib()."""
    pose = np.ascontiguousarray(cur_pose, dtype=np.float64).copy()
    st = ctypes.c_int32()
    traces = (LevelTrace * (max_level + 1))() if trace else None
    err = (L or lib()).oracle_image_align(ctypes.byref(camera(cam)), patch, min_level, max_level, median_mode,
                                   ctypes.byref(pair.pair), _p(pose), ctypes.byref(st),
                                   ctypes.cast(traces, ctypes.c_void_p) if trace else None)
    return pose, err, st.value, traces


def image_align_vectors(cam, patch, min_level, max_level, pair, cur_pose, median_mode=0):
    """image_align that also returns every level's residual vector (coarsest first) and its n_valid: the vectors the
    reference's computeMedian / computeMAD run on (tools/k2v_round_table.py)."""
    pose = np.ascontiguousarray(cur_pose, dtype=np.float64).copy()
    st = ctypes.c_int32()
    M = (pair.pair.n_ref + pair.pair.n_kf) * patch * patch
    out = np.zeros(M * (max_level - min_level + 1))
    nv = np.zeros(max_level - min_level + 1, np.uint32)
    f = lib().oracle_image_align_vectors
    f.restype = ctypes.c_int32
    n = f(ctypes.byref(camera(cam)), patch, min_level, max_level, median_mode, ctypes.byref(pair.pair), _p(pose),
          ctypes.byref(st), _p(out), ctypes.c_int64(len(out)), nv.ctypes.data_as(ctypes.c_void_p))
    return [out[i * M:(i + 1) * M] for i in range(n)], [int(x) for x in nv[:n]]


def image_align_batch(cam, patch, min_level, max_level, pairs, cur_poses, median_mode=0, nthreads=1, L=None):
    n = len(pairs)
    arr = (OcPair * n)(*[p.pair for p in pairs])
    poses = np.ascontiguousarray(cur_poses, dtype=np.float64).copy()
    err = np.zeros(n)
    st = np.zeros(n, np.int32)
    (L or lib()).oracle_image_align_batch(ctypes.byref(camera(cam)), patch, min_level, max_level, median_mode, n, arr,
                                   _p(poses), _p(err), _p(st), nthreads)
    return poses, err, st


def feature_align(cam, patch, ref_grad, cur_grad, ref_px, px_init):
    """FeatureAlignment::align for n candidates.  Returns (px[n,2], err[n], status[n])."""
    ref_grad = np.ascontiguousarray(ref_grad, np.uint8)
    cur_grad = np.ascontiguousarray(cur_grad, np.uint8)
    ref_px = np.ascontiguousarray(ref_px, np.float64)
    px = np.ascontiguousarray(px_init, np.float64).copy()
    n = len(px)
    err = np.zeros(n)
    st = np.zeros(n, np.int32)
    lib().oracle_feature_align(ctypes.byref(camera(cam)), patch, _p(ref_grad), _p(cur_grad), n, _p(ref_px), _p(px),
                               _p(err), _p(st))
    return px, err, st


# ---------------------------------------------------------------- depth filter (config 5)
DEPTH_SEED = np.dtype([("a", "f8"), ("b", "f8"), ("mu", "f8"), ("sigma", "f8"), ("var", "f8"), ("max_depth", "f8"),
                       ("px", "f8", 2), ("bearing", "f8", 3), ("kf", "i4"), ("valid", "i4")])


def depth_seed_init(depth_mean, depth_min):
    """MixedGaussianFilter(feature, depthMean, depthMin): (a, b, mu, sigma, var, max_depth)."""
    out = np.zeros(6)
    lib().oracle_depth_seed_init(ctypes.c_double(depth_mean), ctypes.c_double(depth_min), _p(out))
    return out


def make_seeds(px, bearing, depth_mean, depth_min, kf=0):
    """Seeds for features (px, bearing) of keyframe `kf` (DepthEstimator::initializeFilters)."""
    n = len(px)
    s = np.zeros(n, DEPTH_SEED)
    a, b, mu, sigma, var, md = depth_seed_init(depth_mean, depth_min)
    s["a"], s["b"], s["mu"], s["sigma"], s["var"], s["max_depth"] = a, b, mu, sigma, var, md
    s["px"], s["bearing"], s["kf"], s["valid"] = px, bearing, kf, 1
    return s


def depth_update(cam, kf_imgs, kf_poses, cur_img, cur_pose, seeds):
    """DepthEstimator::updateFilters.  Returns (survivors, outcome[n], cand_points[m,3], cand_seed[m])."""
    assert lib().oracle_depth_seed_size() == DEPTH_SEED.itemsize
    seeds = np.ascontiguousarray(seeds, DEPTH_SEED).copy()
    n = len(seeds)
    imgs = [np.ascontiguousarray(i, np.uint8) for i in kf_imgs]
    ptrs = (ctypes.c_void_p * max(len(imgs), 1))(*[_p(i).value for i in imgs])
    kp = np.ascontiguousarray(kf_poses, np.float64).reshape(-1, 7)
    cur = np.ascontiguousarray(cur_img, np.uint8)
    cp = np.ascontiguousarray(cur_pose, np.float64)
    outc = np.zeros(n, np.int32)
    pts = np.zeros((max(n, 1), 3))
    cs = np.zeros(max(n, 1), np.int32)
    n_out, n_cand = ctypes.c_int32(), ctypes.c_int32()
    lib().oracle_depth_update(ctypes.byref(camera(cam)), len(imgs), ptrs, _p(kp), _p(cur), _p(cp), n, _p(seeds),
                              ctypes.byref(n_out), _p(outc), _p(pts), _p(cs), ctypes.byref(n_cand))
    return seeds[:n_out.value].copy(), outc, pts[:n_cand.value].copy(), cs[:n_cand.value].copy()


def zsad(ref, cur):
    ref = np.ascontiguousarray(ref, np.uint8)
    cur = np.ascontiguousarray(cur, np.uint8)
    L = lib()
    L.oracle_zsad.restype = ctypes.c_double
    return L.oracle_zsad(_p(ref), _p(cur), len(ref))


def depth_triangulate(rel_pose, f_ref, f_cur):
    """(ok, depth) of algorithm::depthFromTriangulation."""
    d = ctypes.c_double()
    r, a, b = (np.ascontiguousarray(x, np.float64) for x in (rel_pose, f_ref, f_cur))
    ok = lib().oracle_depth_triangulate(_p(r), _p(a), _p(b), ctypes.byref(d))
    return bool(ok), d.value


def reproject_map(cam, cell_size, cell_order, cur_pose, cur_id, cur_grad, kf_grads, kf_feat_off, feat_px, feat_point,
                  point_pos, point_type, point_succ, point_last, cell_visited):
    """Map::reprojectMap (src/map.cpp:260-570) restated with one FeatureAlignment call per accepted candidate.
    point_type / point_succ / point_last / cell_visited are updated in place.  Returns (overlap, new_px,
    new_point, new_feat, matches, trials)."""
    n_kf = len(kf_grads)
    grads = [np.ascontiguousarray(g, np.uint8) for g in kf_grads]
    gp = (ctypes.c_void_p * n_kf)(*[g.ctypes.data for g in grads])
    cg = np.ascontiguousarray(cur_grad, np.uint8)
    n_cells = len(cell_order)
    overlap = np.zeros(n_kf, np.int32)
    new_px = np.zeros((n_cells, 2))
    new_point = np.zeros(n_cells, np.int32)
    new_feat = np.zeros(n_cells, np.int32)
    nn, m, t = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    c = camera(cam)
    args = [np.ascontiguousarray(a, dt) for a, dt in ((cell_order, np.int32), (cur_pose, np.float64),
                                                     (kf_feat_off, np.int32), (feat_px, np.float64),
                                                     (feat_point, np.int32), (point_pos, np.float64))]
    for a, dt in ((point_type, np.uint32), (point_succ, np.uint32), (point_last, np.uint64), (cell_visited, np.uint8)):
        assert a.dtype == dt and a.flags.c_contiguous
    lib().oracle_reproject_map(ctypes.byref(c), int(cell_size), _p(args[0]), _p(args[1]), ctypes.c_uint64(cur_id),
                               _p(cg), n_kf, gp, _p(args[2]), _p(args[3]), _p(args[4]), _p(args[5]),
                               _p(point_type), _p(point_succ), _p(point_last), _p(cell_visited), _p(overlap),
                               ctypes.byref(nn), _p(new_px), _p(new_point), _p(new_feat), ctypes.byref(m),
                               ctypes.byref(t))
    k = nn.value
    return overlap, new_px[:k], new_point[:k], new_feat[:k], m.value, t.value


def add_candidates(cam, cell_size, cell_visited, cur_pose, cur_grad, cand_grads, cand_px, cand_point_pos):
    """Map::addCandidateToFrame (src/map.cpp:595-627) restated sequentially.  cell_visited is updated in
    place.  Returns (matched, new_px)."""
    n = len(cand_grads)
    grads = [np.ascontiguousarray(g, np.uint8) for g in cand_grads]
    gp = (ctypes.c_void_p * max(n, 1))(*[g.ctypes.data for g in grads])
    matched = np.zeros(max(n, 1), np.uint8)
    new_px = np.zeros((max(n, 1), 2))
    assert cell_visited.dtype == np.uint8 and cell_visited.flags.c_contiguous
    c = camera(cam)
    cpx = np.ascontiguousarray(cand_px, np.float64)
    cpp = np.ascontiguousarray(cand_point_pos, np.float64)
    lib().oracle_add_candidates(ctypes.byref(c), int(cell_size), _p(cell_visited),
                                _p(np.ascontiguousarray(cur_pose, np.float64)), _p(np.ascontiguousarray(cur_grad, np.uint8)),
                                n, gp, _p(cpx), _p(cpp), _p(matched), _p(new_px))
    return matched[:n].astype(bool), new_px[:n]


# ---------------------------------------------------------------- FeatureSelection (feature_selection_oracle.cpp)
def grid_shape(w, h, cell):
    return h // cell + 1, w // cell + 1


def ssc(x, y, num_ret, cols, rows, tolerance=0.1):
    """FeatureSelection::SSC on keypoints already in sorted order; returns the selected indices."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    out = np.zeros(max(len(x), 1), np.int32)
    n = lib().oracle_ssc(_p(x), _p(y), ctypes.c_int32(len(x)), ctypes.c_int32(num_ret), ctypes.c_float(tolerance),
                         ctypes.c_int32(cols), ctypes.c_int32(rows), _p(out))
    return out[:n]


def feature_select_ssc(img, threshold, num_candidates, use_bucketing, cell_size, occupancy=None):
    """gradientMagnitudeWithSSC on a base image: (px (n, 2), response (n,), occupancy after, n_keypoints)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    occ = np.zeros(grid_shape(w, h, cell_size), np.uint8) if occupancy is None else np.array(occupancy, np.uint8)
    cap = w * h
    px = np.zeros((cap, 2))
    resp = np.zeros(cap)
    nk = ctypes.c_int32()
    n = lib().oracle_feature_select_ssc(_p(img), w, h, threshold, num_candidates, int(bool(use_bucketing)), cell_size,
                                        _p(occ), cap, _p(px), _p(resp), ctypes.byref(nk))
    assert n >= 0
    return px[:n], resp[:n], occ, nk.value


def feature_select_by_value(img, threshold, cell_size, occupancy=None):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    occ = np.zeros(grid_shape(w, h, cell_size), np.uint8) if occupancy is None else np.array(occupancy, np.uint8)
    cap = occ.size
    px = np.zeros((cap, 2))
    resp = np.zeros(cap)
    n = lib().oracle_feature_select_by_value(_p(img), w, h, threshold, cell_size, _p(occ), cap, _p(px), _p(resp))
    assert n >= 0
    return px[:n], resp[:n], occ



def sort_responses(resp):
    """libstdc++ std::sort's keypoint order for u8 responses (reference comparator, :53-54)."""
    resp = np.ascontiguousarray(resp, np.uint8)
    perm = np.zeros(max(len(resp), 1), np.int32)
    lib().oracle_sort_responses(_p(resp), len(resp), _p(perm))
    return perm[:len(resp)]


# ---------------------------------------------------------------- trajectory / feature dump text
def kitti_line(pose):
    """System::writeInFile's line for a world->camera pose (Sophus params)."""
    pose = np.ascontiguousarray(pose, np.float64)
    buf = ctypes.create_string_buffer(512)
    n = lib().oracle_kitti_line(_p(pose), buf, 512)
    assert n >= 0
    return buf.value.decode()


def stream_g6(v):
    """`std::ostream << std::setprecision(6) << v` for one double."""
    buf = ctypes.create_string_buffer(64)
    lib().oracle_stream_g6.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_int32]
    n = lib().oracle_stream_g6(float(v), buf, 64)
    assert n >= 0
    return buf.value.decode()


# ---------------------------------------------------------------- pose-only bundle adjustment
def optimize_pose(bearing, point, has_point, vis_in, pose, median_mode=1):
    """BundleAdjustment::optimizePose on one frame: (pose, err, status, vis_out); vis_in is the object's
    m_refVisibility before the call (any length: resized like the member)."""
    n = len(has_point)
    bearing = np.ascontiguousarray(bearing, np.float64).reshape(-1, 3)
    point = np.ascontiguousarray(point, np.float64).reshape(-1, 3)
    has_point = np.ascontiguousarray(has_point, np.uint8)
    vis = np.zeros(max(n, len(vis_in), 1), np.uint8)
    vis[:len(vis_in)] = vis_in
    pose = np.ascontiguousarray(pose, np.float64).copy()
    err = ctypes.c_double()
    st = ctypes.c_int32()
    rc = lib().oracle_optimize_pose(n, _p(bearing), _p(point), _p(has_point), len(vis_in), _p(vis), _p(pose),
                                    median_mode, ctypes.byref(err), ctypes.byref(st))
    if rc != 0:
        raise ValueError("stale visible flag on a feature without a point")
    return pose, err.value, st.value, (vis[:n].copy() if n else np.array(vis_in, np.uint8))
