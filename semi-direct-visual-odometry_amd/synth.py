"""Deterministic synthetic KITTI-shaped frame pairs (host/svo_synth.cpp through ctypes).

Inputs for benchmarks and parity tests only: seeds follow SURVEY.md §8(d) (seed = 0x5EED0000 + pair).
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _paths

SEED_BASE = 0x5EED0000
_lib = None


class SynthConfig(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("fx", ctypes.c_double),
                ("fy", ctypes.c_double), ("cx", ctypes.c_double), ("cy", ctypes.c_double),
                ("n_features", ctypes.c_int32), ("patch_size", ctypes.c_int32),
                ("null_point_fraction", ctypes.c_double), ("init_trans_err", ctypes.c_double),
                ("init_rot_err_deg", ctypes.c_double), ("nthreads", ctypes.c_int32),
                ("cell_order", ctypes.c_int32)]


def lib():
    global _lib
    if _lib is None:
        path = _paths.lib_path("libsvo_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C semi-direct-visual-odometry_amd` (or __graft_entry__.build())")
        _lib = ctypes.CDLL(path)
        _lib.svo_synth_pair.restype = ctypes.c_int32
        _lib.svo_synth_gradient_fraction.restype = ctypes.c_double
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class SynthPair:
    camera: dict
    kf_img: np.ndarray
    ref_img: np.ndarray
    cur_img: np.ndarray
    kf_pose: np.ndarray
    ref_pose: np.ndarray
    cur_true_pose: np.ndarray
    cur_init_pose: np.ndarray
    n_ref: int
    n_kf: int
    px: np.ndarray
    bearing: np.ndarray
    point: np.ndarray
    has_point: np.ndarray


def default_config(**kw):
    c = SynthConfig()
    lib().svo_synth_default_config(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def make_pair(seed=SEED_BASE, n_features=2000, patch_size=5, width=1241, height=376, null_point_fraction=0.0,
              init_trans_err=0.02, init_rot_err_deg=0.2, nthreads=8, cell_order=0):
    """cell_order: 0 shuffled features; c > 0 the reference detector's order (c-px cells row by row)."""
    c = default_config(n_features=n_features, patch_size=patch_size, width=width, height=height,
                       null_point_fraction=null_point_fraction, init_trans_err=init_trans_err,
                       init_rot_err_deg=init_rot_err_deg, nthreads=nthreads, cell_order=cell_order)
    H, W, N = c.height, c.width, c.n_features
    imgs = [np.zeros((H, W), np.uint8) for _ in range(3)]
    poses = [np.zeros(7) for _ in range(4)]
    px, br, pt = np.zeros((N, 2)), np.zeros((N, 3)), np.zeros((N, 3))
    hp = np.zeros(N, np.uint8)
    nr, nk = ctypes.c_int32(), ctypes.c_int32()
    n = lib().svo_synth_pair(ctypes.byref(c), ctypes.c_uint64(seed), *[_p(i) for i in imgs], *[_p(p) for p in poses],
                             ctypes.byref(nr), ctypes.byref(nk), _p(px), _p(br), _p(pt), _p(hp))
    cam = dict(fx=c.fx, fy=c.fy, cx=c.cx, cy=c.cy, width=W, height=H)
    return SynthPair(cam, imgs[0], imgs[1], imgs[2], *poses, nr.value, nk.value, px[:n], br[:n], pt[:n], hp[:n])


def make_flat_blocks(groups, width=320, height=96, block=12, base=100, fx=300.0):
    """A pair whose level-0 residuals are chosen exactly: feature i sits on a flat block-by-block square of
    the ref image (intensity `base`) and of the cur image (intensity base + r_i); identity poses, so every
    slot of feature i has residual r_i (an integer, bilinear of a flat square).  groups: {r: n_features}.
    For the robust-scale edge cases of K2 (tests/test_gpu_parity.py); align it on level 0 only."""
    r = np.repeat(np.array(list(groups.keys()), np.int64), list(groups.values()))
    n, cols = len(r), width // block - 2
    assert n <= cols * (height // block - 2) and 0 <= base + r.min() and base + r.max() <= 255
    ref = np.full((height, width), 60, np.uint8)
    cur = ref.copy()
    px = np.zeros((n, 2))
    for i in range(n):
        y0, x0 = block * (1 + i // cols), block * (1 + i % cols)
        ref[y0:y0 + block, x0:x0 + block] = base
        cur[y0:y0 + block, x0:x0 + block] = base + r[i]
        px[i] = (x0 + block / 2 - 0.2, y0 + block / 2 - 0.3)
    cam = dict(fx=fx, fy=fx, cx=width / 2, cy=height / 2, width=width, height=height)
    b = np.stack([(px[:, 0] - cam["cx"]) / fx, (px[:, 1] - cam["cy"]) / fx, np.ones(n)], 1)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    ident = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    return SynthPair(cam, ref.copy(), ref, cur, ident.copy(), ident.copy(), ident.copy(), ident.copy(), n, 0, px, b,
                     10.0 * b, np.ones(n, np.uint8))


def gradient_fraction(img, thr=50):
    img = np.ascontiguousarray(img, np.uint8)
    return lib().svo_synth_gradient_fraction(_p(img), img.shape[1], img.shape[0], thr)


@dataclass
class DepthProblem:
    """Config 5: seeds on the keyframe's features (no point yet) refined against cur."""
    camera: dict
    kf_img: np.ndarray
    cur_img: np.ndarray
    kf_pose: np.ndarray
    cur_pose: np.ndarray
    px: np.ndarray        # (n, 2) keyframe pixel of each seed's feature
    bearing: np.ndarray   # (n, 3)
    depth: np.ndarray     # (n,) true distance along the bearing (for checks only)
    depth_mean: float     # initialisation like src/system.cpp:259 / :433: median depth, 0.5 * min depth
    depth_min: float


def make_depth_problem(seed=SEED_BASE, n_seeds=2000, nthreads=8):
    """The lastKF of a synthetic pair is the keyframe, the pair's cur frame (true pose) the new frame."""
    s = make_pair(seed=seed, n_features=2 * n_seeds, nthreads=nthreads)
    sl = slice(s.n_ref, s.n_ref + min(s.n_kf, n_seeds))
    kf = s.kf_pose
    # keyframe centre C = -R^T t; distance along the bearing = |P - C|
    q, t = kf[:4], kf[4:]
    x, y, z, w = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    C = -R.T @ t
    d = np.linalg.norm(s.point[sl] - C, axis=1)
    return DepthProblem(s.camera, s.kf_img, s.cur_img, s.kf_pose.copy(), s.cur_true_pose.copy(), s.px[sl].copy(),
                        s.bearing[sl].copy(), d, float(np.median(d)), float(0.5 * d.min()))


def make_shifted_plane(seed=7, width=320, height=120, fx=300.0, depth=10.0, disparity=48, n_seeds=64,
                       depth_min=1.5):
    """A fronto-parallel textured plane at `depth` seen from the keyframe (identity pose) and from a
    camera moved sideways by depth * disparity / fx: the cur image is the keyframe image shifted left by
    `disparity` pixels, so the epipolar search must find every seed `disparity` px to the left.  The
    small depth_min gives a wide inverse-depth range (mu +- var), so the search scans ~10 steps."""
    rng = np.random.default_rng(seed)
    coarse = rng.uniform(0, 255, ((height + disparity) // 4 + 3, (width + disparity) // 4 + 3))
    yy, xx = np.mgrid[0:height + disparity, 0:width + disparity] / 4.0
    y0, x0 = np.floor(yy).astype(int), np.floor(xx).astype(int)
    fy_, fx_ = yy - y0, xx - x0
    tex = ((1 - fy_) * ((1 - fx_) * coarse[y0, x0] + fx_ * coarse[y0, x0 + 1]) +
           fy_ * ((1 - fx_) * coarse[y0 + 1, x0] + fx_ * coarse[y0 + 1, x0 + 1]))
    tex = np.clip(tex, 0, 255).astype(np.uint8)
    kf_img = np.ascontiguousarray(tex[:height, :width])
    cur_img = np.ascontiguousarray(tex[:height, disparity:disparity + width])
    cam = dict(fx=fx, fy=fx, cx=width / 2.0, cy=height / 2.0, width=width, height=height)
    base = depth * disparity / fx
    cur_pose = np.array([0, 0, 0, 1, -base, 0, 0], np.float64)  # camera centre at (+base, 0, 0)
    us = rng.uniform(disparity + 30, width - 30, n_seeds)
    vs = rng.uniform(20, height - 20, n_seeds)
    px = np.stack([us, vs], 1)
    b = np.stack([(us - cam["cx"]) / fx, (vs - cam["cy"]) / fx, np.ones(n_seeds)], 1)
    bearing = b / np.linalg.norm(b, axis=1, keepdims=True)
    d = depth / bearing[:, 2]  # distance along the bearing to the plane z = depth
    return DepthProblem(cam, kf_img, cur_img, np.array([0, 0, 0, 1, 0, 0, 0], np.float64), cur_pose, px, bearing, d,
                        float(np.median(d) * 1.03), float(depth_min))


@dataclass
class MapProblem:
    """A map for Map::reprojectMap / addCandidateToFrame, from a config-2 scene:
    the ref frame's and its last keyframe's features observe points; some lastKF features share a ref
    feature's point (so the per-frame projection flag matters), point types are mixed (DELETED cells are
    skipped), success counters sit around the promotion threshold, and lastKF features without a point
    become depth-filter candidates for addCandidateToFrame."""
    camera: dict
    ref_img: np.ndarray
    kf_img: np.ndarray
    cur_img: np.ndarray
    ref_pose: np.ndarray
    kf_pose: np.ndarray
    cur_pose: np.ndarray
    n_ref: int
    n_kf: int
    feat_px: np.ndarray      # (n_ref + n_kf, 2): ref features, then lastKF features
    feat_point: np.ndarray   # (n,) point index or -1
    point_pos: np.ndarray    # (n_points, 3)
    point_type: np.ndarray   # (n_points,) uint32 Point::PointType
    point_succ: np.ndarray   # (n_points,) uint32 m_succeededProjection
    cand_feat: np.ndarray    # (n_cand,) feature indices (lastKF features without a point)
    cand_pos: np.ndarray     # (n_cand, 3) their converged points
    cell_size: int = 30      # config "cell_pixel_size"


def make_map_problem(seed=SEED_BASE, n_features=2000, share=0.2, cand_frac=0.15, nthreads=8):
    s = make_pair(seed=seed, n_features=n_features, nthreads=nthreads, cell_order=30)
    rng = np.random.default_rng(seed ^ 0x3A9)
    n = s.n_ref + s.n_kf
    feat_point = np.full(n, -1, np.int32)
    pos = []
    for f in range(n):
        if s.has_point[f]:
            feat_point[f] = len(pos)
            pos.append(s.point[f])
    pos = np.array(pos)
    kf_idx = np.arange(s.n_ref, n)
    cand = rng.choice(kf_idx, size=int(cand_frac * s.n_kf), replace=False)
    cand.sort()
    cand_pos = pos[feat_point[cand]].copy()
    feat_point[cand] = -1
    rest = np.setdiff1d(kf_idx, cand)
    shared = rng.choice(rest, size=int(share * len(rest)), replace=False)
    feat_point[shared] = rng.integers(0, s.n_ref, size=len(shared))  # ref features' points (index = ref feature)
    npt = len(pos)
    ptype = rng.choice(np.array([0, 1, 2, 3], np.uint32), size=npt, p=[0.2, 0.1, 0.2, 0.5]).astype(np.uint32)
    psucc = rng.integers(0, 13, size=npt).astype(np.uint32)
    return MapProblem(s.camera, s.ref_img, s.kf_img, s.cur_img, s.ref_pose, s.kf_pose, s.cur_true_pose, s.n_ref, s.n_kf,
                      s.px.copy(), feat_point, pos, ptype, psucc, cand, cand_pos)


def map_objects(p, levels=1, ctx=None, seed=0):
    """The svo_amd object graph of a MapProblem: (map, ref frame, last keyframe, cur frame, points)."""
    import svo_amd
    c = p.camera
    cam = svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])
    kf = svo_amd.Frame(cam, p.kf_img, levels, ctx=ctx)
    kf.abs_pose[:] = p.kf_pose
    ref = svo_amd.Frame(cam, p.ref_img, levels, last_keyframe=kf, ctx=ctx)
    ref.abs_pose[:] = p.ref_pose
    cur = svo_amd.Frame(cam, p.cur_img, levels, last_keyframe=kf, ctx=ctx)
    cur.abs_pose[:] = p.cur_pose
    points = []
    for i in range(len(p.point_pos)):
        pt = svo_amd.Point(p.point_pos[i])
        pt.type = int(p.point_type[i])
        pt.succeeded_projection = int(p.point_succ[i])
        points.append(pt)
    feats = []
    for f in range(p.n_ref + p.n_kf):
        fr = ref if f < p.n_ref else kf
        ft = svo_amd.Feature(fr, p.feat_px[f], 0, point=points[p.feat_point[f]] if p.feat_point[f] >= 0 else None)
        fr.add_feature(ft)
        feats.append(ft)
    m = svo_amd.Map(cam, p.cell_size, seed=seed, ctx=ctx)
    for i, f in enumerate(p.cand_feat):
        m.add_new_candidate(feats[f], svo_amd.Point(p.cand_pos[i]))
    return m, ref, kf, cur, points, feats


def write_align_problem(s, directory):
    """Files for build/svo_host_check align (the C++ mirror's ImageAlignment): align.bin (the camera, the three
    poses, n_ref, n_kf, then one 9-double row per feature: px, bearing, point, has_point) and the three base
    images.  Returns the four paths."""
    c = s.camera
    hdr = [c["fx"], c["fy"], c["cx"], c["cy"], c["width"], c["height"], *s.ref_pose, *s.kf_pose, *s.cur_init_pose,
           s.n_ref, s.n_kf]
    rows = np.concatenate([s.px, s.bearing, s.point, s.has_point.reshape(-1, 1).astype(np.float64)], axis=1)
    data = os.path.join(directory, "align.bin")
    np.concatenate([np.array(hdr, np.float64), rows.ravel()]).tofile(data)
    paths = [data]
    for k, img in (("ref", s.ref_img), ("kf", s.kf_img), ("cur", s.cur_img)):
        path = os.path.join(directory, f"{k}.raw")
        np.ascontiguousarray(img, np.uint8).tofile(path)
        paths.append(path)
    return paths


def write_map_problem(p, directory, cell_order):
    """Files for build/svo_host_check map (the C++ mirror's Map): DATA.bin (doubles, layout in
    host/svo_host_check.cpp) and the three base images.  Returns the four paths."""
    import os
    c = p.camera
    parts = [[c["fx"], c["fy"], c["cx"], c["cy"], c["width"], c["height"], p.cell_size], p.ref_pose, p.kf_pose,
             p.cur_pose, [p.n_ref, p.n_kf, len(p.point_pos), len(p.cand_feat), len(cell_order)], p.feat_px.ravel(),
             p.feat_point, p.point_pos.ravel(), p.point_type, p.point_succ, p.cand_feat, p.cand_pos.ravel(),
             cell_order]
    data = np.concatenate([np.asarray(x, np.float64).ravel() for x in parts])
    paths = [os.path.join(directory, n) for n in ("map.bin", "ref.raw", "kf.raw", "cur.raw")]
    with open(paths[0], "wb") as f:
        f.write(data.tobytes())
    for path, img in zip(paths[1:], (p.ref_img, p.kf_img, p.cur_img)):
        with open(path, "wb") as f:
            f.write(np.ascontiguousarray(img, np.uint8).tobytes())
    return paths
