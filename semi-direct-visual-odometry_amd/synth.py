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
                ("init_rot_err_deg", ctypes.c_double), ("nthreads", ctypes.c_int32)]


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
              init_trans_err=0.02, init_rot_err_deg=0.2, nthreads=8):
    c = default_config(n_features=n_features, patch_size=patch_size, width=width, height=height,
                       null_point_fraction=null_point_fraction, init_trans_err=init_trans_err,
                       init_rot_err_deg=init_rot_err_deg, nthreads=nthreads)
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


def gradient_fraction(img, thr=50):
    img = np.ascontiguousarray(img, np.uint8)
    return lib().svo_synth_gradient_fraction(_p(img), img.shape[1], img.shape[0], thr)
