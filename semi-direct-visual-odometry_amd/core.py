"""Python mirror of the reference's class surface for the alignment hot path, over the C ABI.

Names, argument meaning and error behaviour follow the reference:
  PinholeCamera      include/pinhole_camera.hpp:16 (undistorted path, src/pinhole_camera.cpp:50-101)
  ImagePyramid       include/image_pyramid.hpp:23-149          (device resident; getters download)
  Frame / Feature / Point   include/frame.hpp:70-208, include/feature.hpp:14, include/point.hpp:14
  ImageAlignment     include/image_alignment.hpp:15-73         (align(ref, cur) -> error, cur pose in place)
  FeatureAlignment   include/feature_alignment.hpp:15-43       (align(feature, cur, px) -> error, px in place)
plus the batched forms the GPU is built for (AlignBatch, FeatureAlignment.align_batch).
"""
import ctypes
import math
import operator
import time

import numpy as np

from . import _capi
from ._capi import check, lib, ptr

_default_ctx = {}


class Context:
    """One HIP stream on one GPU (svo_ctx)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().svo_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = int(device)

    @property
    def stream(self):
        return lib().svo_ctx_stream(self.handle)

    def synchronize(self):
        check(lib().svo_ctx_synchronize(self.handle))

    def record(self, slot):
        """hipEventRecord(slot) on this context's stream."""
        check(lib().svo_ctx_event_record(self.handle, int(slot)))

    def elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        check(lib().svo_ctx_event_elapsed(self.handle, int(a), int(b), ctypes.byref(ms)))
        return ms.value

    def close(self):
        if self.handle:
            lib().svo_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_context(device=0):
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def device_count():
    n = ctypes.c_int32()
    check(lib().svo_device_count(ctypes.byref(n)))
    return n.value


class PinholeCamera:
    def __init__(self, width, height, fx, fy, cx, cy):
        self.width, self.height = int(width), int(height)
        self.fx, self.fy, self.cx, self.cy = float(fx), float(fy), float(cx), float(cy)

    @classmethod
    def kitti(cls):  # resource/kitti.yaml:7-8, config/config.json:10-11
        return cls(1241, 376, 721.5377, 721.5377, 609.5593, 172.8540)

    def as_c(self):
        return _capi.SvoCamera(self.fx, self.fy, self.cx, self.cy, self.width, self.height)

    def as_dict(self):
        return dict(fx=self.fx, fy=self.fy, cx=self.cx, cy=self.cy, width=self.width, height=self.height)

    def project2d(self, p):  # src/pinhole_camera.cpp:53-57
        return np.array([self.fx * (p[0] / p[2]) + self.cx, self.fy * (p[1] / p[2]) + self.cy])

    def inverse_project2d(self, px):  # src/pinhole_camera.cpp:84-100
        v = np.array([(px[0] - self.cx) / self.fx, (px[1] - self.cy) / self.fy, 1.0])
        return v * (1.0 / math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]))

    def is_in_frame(self, p, boundary=0.0):  # src/pinhole_camera.cpp:163-168
        return p[0] >= boundary and p[1] >= boundary and p[0] < self.width - boundary and p[1] < self.height - boundary


class PyramidSet:
    """n_frames device-resident (image, gradient) stacks of equal geometry (svo_pyramid_set)."""

    def __init__(self, n_frames, width, height, levels, ctx=None):
        self.ctx = ctx or default_context()
        self.n_frames, self.width, self.height, self.levels = int(n_frames), int(width), int(height), int(levels)
        h = ctypes.c_void_p()
        check(lib().svo_pyramid_set_create(self.ctx.handle, self.n_frames, self.width, self.height, self.levels,
                                           ctypes.byref(h)))
        self.handle = h

    def upload(self, first, images):
        imgs = np.ascontiguousarray(images, dtype=np.uint8)
        count = imgs.shape[0] if imgs.ndim == 3 else 1
        if imgs.shape[-2:] != (self.height, self.width):
            raise ValueError(f"image shape {imgs.shape[-2:]} != ({self.height}, {self.width})")
        check(lib().svo_pyramid_set_upload(self.handle, int(first), count, ptr(imgs)))
        self.ctx.synchronize()  # the host buffer may die after return

    def build(self, first=0, count=None):
        count = self.n_frames - first if count is None else count
        check(lib().svo_pyramid_set_build(self.handle, int(first), int(count)))

    def build_async(self, first=0, count=None):
        """build() on the context's prep stream, overlapping work queued after it (svo_pyramid_set_build_async):
        every later use of the set through the library waits for it."""
        count = self.n_frames - first if count is None else count
        check(lib().svo_pyramid_set_build_async(self.handle, int(first), int(count)))

    def level_size(self, level):
        w, h = ctypes.c_int32(), ctypes.c_int32()
        check(lib().svo_pyramid_level_size(self.handle, int(level), ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    def download(self, frame, level, gradient=False):
        w, h = self.level_size(level)
        out = np.empty((h, w), np.uint8)
        check(lib().svo_pyramid_set_download(self.handle, int(frame), int(level), 1 if gradient else 0, ptr(out)))
        return out

    def close(self):
        # only while the owning context lives: objects kept alive by reference cycles (Frame <-> Feature)
        # may be finalized after their context at interpreter exit
        if getattr(self, "handle", None) and getattr(self.ctx, "handle", None):
            lib().svo_pyramid_set_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ImagePyramid:
    """ImagePyramid(baseImage, maxPyramidLevel) — device resident (src/image_pyramid.cpp:14-52)."""

    def __init__(self, base_image=None, levels=4, ctx=None):
        self.ctx = ctx or default_context()
        self.levels = int(levels)
        self.set = None
        if base_image is not None:
            self.create_image_pyramid(base_image, levels)

    def create_image_pyramid(self, base_image, levels):
        img = np.ascontiguousarray(base_image, dtype=np.uint8)
        if img.ndim != 2:
            raise ValueError("ImagePyramid expects one 8-bit grey image")
        self.levels = int(levels)
        self.set = PyramidSet(1, img.shape[1], img.shape[0], self.levels, self.ctx)
        self.set.upload(0, img[None])
        self.set.build(0, 1)

    def get_size_image_pyramid(self):
        return 0 if self.set is None else self.levels

    def get_image_at_level(self, level):
        return self.set.download(0, level, False)

    def get_gradient_at_level(self, level):
        return self.set.download(0, level, True)

    def get_base_image(self):
        return self.get_image_at_level(0)

    def get_base_gradient_image(self):
        return self.get_gradient_at_level(0)

    def get_image_size_at_level(self, level):
        if self.set is None or level >= self.levels:
            return (0, 0)
        return self.set.level_size(level)

    def get_base_image_size(self):
        return self.get_image_size_at_level(0)

    def clear(self):
        if self.set is not None:
            self.set.close()
        self.set = None


def _frozen(v):
    """A read-only float64 copy of v (the per-frame SoA caches rely on positions changing only by assignment)."""
    a = np.array(v, dtype=np.float64)
    a.flags.writeable = False
    return a


class PointType:  # Point::PointType (include/point.hpp:18-24)
    GOOD, DELETED, CANDIDATE, UNKNOWN = 0, 1, 2, 3


class _PointTable:
    """The state of every live Point as arrays (position, type, m_lastProjectedKFId, the projection counters), one
    row per point: Map.reproject_map gathers these fields of ~2000 points and writes the projection ids back as
    array operations instead of walking the objects.  Rows of collected points are reused."""

    def __init__(self, cap=4096):
        self.pos = np.zeros((cap, 3))
        self.type = np.zeros(cap, np.uint32)
        self.last = np.zeros(cap, np.uint64)
        self.succ = np.zeros(cap, np.int64)
        self.fail = np.zeros(cap, np.int64)
        self.n = 0
        self.free = []

    def alloc(self):
        if self.free:
            return self.free.pop()
        if self.n == len(self.type):
            for k in ("pos", "type", "last", "succ", "fail"):
                a = getattr(self, k)
                b = np.zeros((2 * len(a),) + a.shape[1:], a.dtype)
                b[:len(a)] = a
                setattr(self, k, b)
        self.n += 1
        return self.n - 1


_PT = _PointTable()


class Point:
    """Point(position) (src/point.cpp:6-18): position, type, the observing features and the
    reprojection bookkeeping the Map reads (include/point.hpp:28-40).  The fields live in a row of _PT."""
    NO_FRAME = 2 ** 64 - 1  # m_lastProjectedKFId(-1) on a uint64

    def __init__(self, position):
        i = _PT.alloc()
        self._i = i
        _PT.pos[i] = np.asarray(position, np.float64).reshape(3)  # (a new point is in no frame's cached arrays yet)
        _PT.type[i] = PointType.UNKNOWN
        _PT.last[i] = Point.NO_FRAME
        _PT.succ[i] = 0
        _PT.fail[i] = 0
        self.features = []

    def __del__(self):
        try:
            _PT.free.append(self._i)
        except Exception:  # (interpreter shutdown)
            pass

    # copies own a fresh row: copying _i would alias one row between two Points and put it on the free list twice
    # 
    def _state(self):
        i = self._i
        return (_PT.pos[i].copy(), int(_PT.type[i]), int(_PT.last[i]), int(_PT.succ[i]), int(_PT.fail[i]))

    def __copy__(self):
        return _point_from_state(self._state(), self.features)

    def __deepcopy__(self, memo):
        import copy
        p = _point_from_state(self._state(), ())
        memo[id(self)] = p
        p.features = copy.deepcopy(self.features, memo)
        return p

    def __reduce__(self):
        return (_point_from_state, (self._state(), self.features))

    type = property(lambda self: int(_PT.type[self._i]), lambda self, v: _PT.type.__setitem__(self._i, v))
    last_projected_kf_id = property(lambda self: int(_PT.last[self._i]),
                                    lambda self, v: _PT.last.__setitem__(self._i, v))
    succeeded_projection = property(lambda self: int(_PT.succ[self._i]),
                                    lambda self, v: _PT.succ.__setitem__(self._i, v))
    failed_projection = property(lambda self: int(_PT.fail[self._i]), lambda self, v: _PT.fail.__setitem__(self._i, v))

    def add_feature(self, feature):  # src/point.cpp:35-38
        self.features.append(feature)

    def find_frame(self, frame):  # src/point.cpp: any observing feature in `frame`
        return any(f.frame is frame for f in self.features)

    # a read-only float64 copy of the row (an in-place edit would not reach the table, so it raises instead).
    # Assigning it bumps a global version that invalidates every Frame's cached point array (a point is not told
    # which frames' features hold it).
    _ver = 0

    @property
    def position(self):
        return _frozen(_PT.pos[self._i])

    @position.setter
    def position(self, v):
        _PT.pos[self._i] = np.asarray(v, np.float64).reshape(3)
        Point._ver += 1


def _point_from_state(state, features):
    """A Point on a row of its own holding `state` (Point._state()) and observed by `features` (copy / pickle)."""
    p = Point(state[0])
    i = p._i
    _PT.type[i], _PT.last[i], _PT.succ[i], _PT.fail[i] = state[1:]
    p.features = list(features)
    return p


class Feature:
    """Feature(frame, pixelPosition, level) — bearing from the frame's camera (src/feature.cpp:14)."""

    # Feature::FeatureType (include/feature.hpp:19-23)
    EDGE, CORNER = 0, 1

    def __init__(self, frame, pixel_position, level=0, point=None, bearing=None, gradient_magnitude=1.0,
                 gradient_orientation=0.0, feature_type=EDGE):
        self._frame = frame
        self._px = _frozen(pixel_position)
        self.level = level
        self.gradient_magnitude = gradient_magnitude      # m_gradientMagnitude (src/feature.cpp:15,34)
        self.gradient_orientation = gradient_orientation  # m_gradientOrientation
        self.type = feature_type
        self._bearing = None if bearing is None else np.asarray(bearing, np.float64)
        self._point = point
        self._pi = -1 if point is None else point._i  # the point's _PT row (-1: none), read by the array gathers
        self._touch()

    @classmethod
    def _many(cls, frame, px, level=0, points=None, gradient_magnitude=None, feature_type=EDGE):
        """Features at the rows of px (n, 2) on `frame` without the per-object property path (the Map and
        FeatureSelection surfaces create hundreds per call): each pixel position is a read-only row of one frozen
        copy of px, points / gradient magnitudes per feature (None: none / 1.0).  Not added to the frame."""
        pxf = _frozen(px)
        n = len(pxf)
        pts = points if points is not None else [None] * n
        gm = gradient_magnitude if gradient_magnitude is not None else [1.0] * n
        out = []
        new = object.__new__
        for i in range(n):
            f = new(cls)
            p = pts[i]
            f.__dict__ = {"_frame": frame, "_px": pxf[i], "level": level, "gradient_magnitude": gm[i],
                          "gradient_orientation": 0.0, "type": feature_type, "_bearing": None, "_point": p,
                          "_pi": -1 if p is None else p._i}
            out.append(f)
        return out

    def _touch(self):  # the owning frame's cached feature arrays are stale
        fr = getattr(self, "_frame", None)
        cell = getattr(fr, "_feat_ver", None)
        if cell is not None:
            cell[0] += 1

    @property
    def frame(self):
        return self._frame

    @frame.setter
    def frame(self, fr):  # both the old and the new frame's cached arrays are stale
        self._touch()
        self._frame = fr
        self._touch()

    # always a read-only float64 array (_feature_arrays joins the raw bytes); assignments invalidate the frame's
    # cached arrays, in-place edits raise (they would leave the cache stale)
    @property
    def pixel_position(self):
        return self._px

    @pixel_position.setter
    def pixel_position(self, v):
        self._px = _frozen(v)
        self._touch()

    @property
    def point(self):
        return self._point

    @point.setter
    def point(self, p):
        self._point = p
        self._pi = -1 if p is None else p._i
        self._touch()

    @property
    def bearing_vec(self):  # formed on first use (the map creates many features that never need it)
        if self._bearing is None:
            self._bearing = np.asarray(self.frame.camera.inverse_project2d(self._px), dtype=np.float64)
        return self._bearing

    def set_point(self, point):
        self.point = point


class _FeatureList(list):
    """Frame.features: a list whose mutations bump the frame's feature version (the cached SoA arrays of
    _feature_arrays are rebuilt only after a change)."""
    __slots__ = ("_cell",)

    def __init__(self, items=(), cell=None):
        super().__init__(items)
        self._cell = cell

    def _bump(self):
        if self._cell is not None:
            self._cell[0] += 1


def _mutator(name):
    base = getattr(list, name)

    def f(self, *a, **k):
        r = base(self, *a, **k)
        self._bump()
        return r if name != "__iadd__" else self
    f.__name__ = name
    return f


for _m in ("append", "extend", "insert", "remove", "pop", "clear", "sort", "reverse", "__setitem__", "__delitem__",
           "__iadd__", "__imul__"):
    setattr(_FeatureList, _m, _mutator(_m))


class Frame:
    """Frame(camera, img, maxImagePyramid, timestamp, lastKeyframe) (src/frame.cpp:6-27)."""

    _frame_counter = 0  # Frame::m_frameCounter

    def __init__(self, camera, image, max_image_pyramid, timestamp=0, last_keyframe=None, ctx=None):
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2 or img.shape != (camera.height, camera.width):
            raise RuntimeError("Image Corrupted")  # src/frame.cpp:20-24
        self.camera = camera
        self.abs_pose = np.array([0, 0, 0, 1, 0, 0, 0], dtype=np.float64)  # identity (src/frame.cpp:13)
        self.image_pyramid = ImagePyramid(img, max_image_pyramid, ctx)
        self._feat_ver = [0]  # bumped by any change to the features (list or Feature attributes)
        self._soa = None      # (key, px, bearing, point, has_point) of the current features
        self.features = []
        self.last_keyframe = last_keyframe
        self.timestamp = timestamp
        self.id = Frame._frame_counter
        Frame._frame_counter += 1

    def world2image(self, points):
        """Frame::world2image (src/frame.cpp:83-92) for an (n, 3) array (or one point)."""
        pts = np.ascontiguousarray(np.atleast_2d(points), dtype=np.float64)
        out = np.zeros((pts.shape[0], 2))
        cam = self.camera.as_c()
        check(lib().svo_world2image(ctypes.byref(cam), ptr(np.ascontiguousarray(self.abs_pose, np.float64)),
                                    pts.shape[0], ptr(pts), ptr(out)))
        return out if np.ndim(points) == 2 else out[0]

    @property
    def features(self):
        return self._features

    @features.setter
    def features(self, v):
        self._features = _FeatureList(v, self._feat_ver)
        self._feat_ver[0] += 1

    def add_feature(self, feature):
        self.features.append(feature)

    def number_observation(self):
        return len(self.features)

    def feature_arrays(self):
        """This frame's features as SoA arrays (px, bearing, point, has_point), cached until the features change
        (list mutations, Feature.pixel_position / point assignments, any Point.position assignment)."""
        key = (self._feat_ver[0], Point._ver)
        c = self._soa
        if c is None or c[0] != key:
            if c is not None and c[0][0] == key[0]:  # only point positions moved: regather them (same rows)
                self._soa = (key, c[1], c[2], _gather_points(c[5]), c[4], c[5])
            else:
                self._soa = (key, *_feature_soa(self.features))
        return self._soa[1:5]


def _rows(vals, width):
    """float64 arrays of `width` values each -> an (n, width) array.  One join of their raw bytes is ~2x faster
    than np.array over the list (the per-frame gather of ~2000 features is most of align()'s host time).  Feature
    and Point keep these attributes float64 arrays (their setters convert); a duck-typed feature's rows that are
    not all float64 arrays of `width` values (checked per row and by the total length) take np.array's
    conversion."""
    n = len(vals)
    try:
        buf = b"".join([v.tobytes() for v in vals])
        if len(buf) == 8 * width * n and all(v.dtype == np.float64 for v in vals):
            return np.frombuffer(buf, dtype=np.float64).reshape(n, width)
    except AttributeError:
        pass
    return np.array(vals, dtype=np.float64).reshape(n, width)


_get_pi = operator.attrgetter("_pi")


def _point_rows(feats):
    """The _PT rows of the features' points (-1: no point).  A live point's row is never reused (the feature
    holds the point), so each Feature keeps it in _pi."""
    return np.fromiter(map(_get_pi, feats), np.int64, count=len(feats))


def _gather_points(idx):
    out = _PT.pos[np.maximum(idx, 0)]
    out[idx < 0] = 0.0
    return out


def _points_of(feats):
    return _gather_points(_point_rows(feats)) if feats else np.zeros((0, 3))


def _feature_soa(feats):
    """(px, bearing, point, has_point, point rows) of the features."""
    n = len(feats)
    if n == 0:
        return np.zeros((0, 2)), np.zeros((0, 3)), np.zeros((0, 3)), np.zeros(0, np.uint8), np.zeros(0, np.int64)
    px = _rows([f.pixel_position for f in feats], 2)
    br = _rows([f.bearing_vec for f in feats], 3)
    idx = _point_rows(feats)
    return px, br, _gather_points(idx), (idx >= 0).astype(np.uint8), idx


def _feature_arrays(frames):
    """The frames' features as SoA arrays (px, bearing, point, has_point), in frame then feature order (each
    frame's arrays cached by Frame.feature_arrays, so a frame that serves as ref or keyframe again costs no
    per-feature gather)."""
    parts = [fr.feature_arrays() for fr in frames]
    if sum(len(p[0]) for p in parts) == 0:
        return np.zeros((1, 2)), np.zeros((1, 3)), np.zeros((1, 3)), np.zeros(1, np.uint8)
    return tuple(np.concatenate([p[i] for p in parts]) for i in range(4))


MEDIAN_EXACT, MEDIAN_REFERENCE = 0, 1  # include/svo_c.h SVO_MEDIAN_*
REF_MAX_SLOTS = 524288  # include/svo_c.h SVO_REF_MAX_SLOTS


class AlignBatch:
    """n_pairs independent ImageAlignment::align problems on one GPU (svo_align_batch).

    median_mode: MEDIAN_REFERENCE (default) reproduces the reference's robust scale bit for bit (libstdc++
    nth_element post-state, src/algorithm.cpp:834-853); MEDIAN_EXACT uses true order statistics (faster,
    not the reference's numbers: DESIGN.md)."""

    def __init__(self, camera, patch_size, min_level, max_level, n_pairs, max_features, ctx=None,
                 median_mode=MEDIAN_REFERENCE):
        self.ctx = ctx or default_context()
        self.camera = camera
        self.n_pairs = int(n_pairs)
        self.max_level = int(max_level)
        self.median_mode = int(median_mode)
        self._c_cam = camera.as_c()
        self._c_prm = _capi.SvoAlignParams(int(patch_size), int(min_level), int(max_level), self.median_mode)
        h = ctypes.c_void_p()
        check(lib().svo_align_batch_create(self.ctx.handle, ctypes.byref(self._c_cam), ctypes.byref(self._c_prm),
                                           self.n_pairs, int(max_features), ctypes.byref(h)))
        self.handle = h
        self._keep = {}

    def set_pair(self, pair, ref, kf, cur, ref_pose, kf_pose, cur_pose, n_ref, n_kf, px, bearing, point, has_point):
        """ref/kf/cur: (PyramidSet, frame index)."""
        arr = lambda a, dt: np.ascontiguousarray(a, dtype=dt)
        px, bearing, point, has_point = arr(px, np.float64), arr(bearing, np.float64), arr(point, np.float64), \
            arr(has_point, np.uint8)
        poses = [arr(p, np.float64) for p in (ref_pose, kf_pose, cur_pose)]
        check(lib().svo_align_batch_set_pair(self.handle, int(pair), ref[0].handle, int(ref[1]), kf[0].handle,
                                             int(kf[1]), cur[0].handle, int(cur[1]), *[ptr(p) for p in poses],
                                             int(n_ref), int(n_kf), ptr(px), ptr(bearing), ptr(point), ptr(has_point)))
        self._keep[pair] = (ref[0], kf[0], cur[0])

    def set_pairs(self, first, ref_set, kf_set, cur_set, frames, poses, n_feat, px, bearing, point, has_point):
        """Bulk set_pair (svo_align_batch_set_pairs) for pairs [first, first + len(frames)): frames (count, 3)
        (ref, kf, cur) indices into the three PyramidSets, poses (count, 3, 7), n_feat (count, 2) = (n_ref,
        n_kf), feature rows packed pair after pair.  Feature arrays may be numpy (host) or CUDA tensors
        (device pointers, copied on the device)."""
        frames = np.ascontiguousarray(frames, dtype=np.int32).reshape(-1, 3)
        count = frames.shape[0]
        poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(count, 21)
        n_feat = np.ascontiguousarray(n_feat, dtype=np.int32).reshape(count, 2)
        arrs = (px, bearing, point, has_point)
        cuda = [hasattr(a, "data_ptr") and getattr(a, "is_cuda", False) for a in arrs]
        on_dev = all(cuda)
        if any(cuda) and not on_dev:
            raise ValueError("set_pairs: the feature arrays must be all host arrays or all CUDA tensors")
        if on_dev:
            import torch
            T = int(n_feat.astype(np.int64).sum())
            for name, a, per, dt in (("px", px, 2, (torch.float64,)), ("bearing", bearing, 3, (torch.float64,)),
                                     ("point", point, 3, (torch.float64,)),
                                     ("has_point", has_point, 1, (torch.uint8, torch.int8, torch.bool))):
                if a.dtype not in dt:
                    raise TypeError(f"set_pairs: {name} is {a.dtype}, expected {' / '.join(map(str, dt))}")
                if not a.is_contiguous():
                    raise ValueError(f"set_pairs: {name} must be contiguous")
                if a.device.index != self.ctx.device:
                    raise ValueError(f"set_pairs: {name} is on {a.device}, the batch on cuda:{self.ctx.device}")
                if a.numel() != per * T:
                    raise ValueError(f"set_pairs: {name} has {a.numel()} elements, expected {per} x {T} rows")
            # the scatter runs on the library's streams: whatever torch queued to produce the tensors goes first
            for d in {a.device for a in arrs}:
                torch.cuda.current_stream(d).synchronize()
            ptrs = [ctypes.c_void_p(a.data_ptr()) for a in (px, bearing, point, has_point)]
            keep = (px, bearing, point, has_point)
        else:
            keep = (np.ascontiguousarray(px, dtype=np.float64), np.ascontiguousarray(bearing, dtype=np.float64),
                    np.ascontiguousarray(point, dtype=np.float64), np.ascontiguousarray(has_point, dtype=np.uint8))
            ptrs = [ptr(a) for a in keep]
        check(lib().svo_align_batch_set_pairs(self.handle, int(first), int(count), ref_set.handle, kf_set.handle,
                                              cur_set.handle, ptr(frames), ptr(poses), ptr(n_feat), *ptrs, int(on_dev)))
        for i in range(count):
            self._keep[int(first) + i] = (ref_set, kf_set, cur_set)
        del keep

    def set_initial_poses(self, poses):
        poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(self.n_pairs, 7)
        check(lib().svo_align_batch_set_initial_poses(self.handle, ptr(poses)))

    def run(self):
        check(lib().svo_align_batch_run(self.handle))

    STAGES = ("init", "residual", "scale", "weights", "solve")

    def profile(self):
        """One synchronous run with events between launches: device ms per stage, summed over levels."""
        ms = (ctypes.c_float * 5)()
        check(lib().svo_align_batch_profile(self.handle, ms))
        return {k: float(v) for k, v in zip(self.STAGES, ms)}

    def results(self):
        poses = np.zeros((self.n_pairs, 7))
        err = np.zeros(self.n_pairs)
        st = np.zeros(self.n_pairs, np.int32)
        check(lib().svo_align_batch_results(self.handle, ptr(poses), ptr(err), ptr(st)))
        return poses, err, st

    def traces(self, pair):
        out = (_capi.SvoLevelTrace * (self.max_level + 1))()
        check(lib().svo_align_batch_traces(self.handle, int(pair), ctypes.cast(out, ctypes.c_void_p)))
        return out

    def close(self):
        if getattr(self, "handle", None) and getattr(self.ctx, "handle", None):
            lib().svo_align_batch_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ImageAlignment:
    """ImageAlignment(patchSize, minLevel, maxLevel, numParameters) (src/image_alignment.cpp:15-67)."""

    def __init__(self, patch_size, min_level, max_level, num_parameters=6, ctx=None, median_mode=MEDIAN_REFERENCE):
        if num_parameters != 6:
            raise ValueError("ImageAlignment estimates SE(3): numParameters must be 6")
        self.patch_size, self.min_level, self.max_level = int(patch_size), int(min_level), int(max_level)
        self.ctx = ctx or default_context()
        self.median_mode = int(median_mode)
        self.last_status = None
        self._traces = None  # the last align()'s per-level traces, fetched on first access (last_traces)
        self._batch = None  # grow-only single-pair batch, reused across align() calls
        self._batch_key = None

    @property
    def last_traces(self):
        """Per-level traces of the last align() (SvoLevelTrace array), or None."""
        if isinstance(self._traces, AlignBatch):
            self._traces = self._traces.traces(0)
        return self._traces

    def align(self, ref_frame, cur_frame):
        """Aligns cur_frame.abs_pose in place; returns the finest level's RMSE (0 if ref has no features)."""
        self._traces = None
        if ref_frame.number_observation() == 0:
            return 0.0
        kf = ref_frame.last_keyframe
        if kf is None:
            raise ValueError("ref_frame.last_keyframe is required (src/image_alignment.cpp:30-31)")
        px, br, pt, hp = _feature_arrays([ref_frame, kf])
        nf = ref_frame.number_observation() + kf.number_observation()
        cam = ref_frame.camera
        key = (cam.width, cam.height, cam.fx, cam.fy, cam.cx, cam.cy)
        if self._batch is None or self._batch_key != key or self._batch_cap < nf:
            if self._batch is not None:
                self._batch.close()
            grow = 1 if self._batch is None else 2 * self._batch_cap
            if self.median_mode == MEDIAN_REFERENCE:  # doubling must not cross the reference-mode limit
                grow = min(grow, REF_MAX_SLOTS // (self.patch_size * self.patch_size))
            cap = max(nf, grow)
            self._batch = AlignBatch(cam, self.patch_size, self.min_level, self.max_level, 1, cap, self.ctx,
                                     median_mode=self.median_mode)
            self._batch_key, self._batch_cap = key, cap
        b = self._batch
        s = lambda fr: (fr.image_pyramid.set, 0)
        b.set_pair(0, s(ref_frame), s(kf), s(cur_frame), ref_frame.abs_pose, kf.abs_pose, cur_frame.abs_pose,
                   ref_frame.number_observation(), kf.number_observation(), px, br, pt, hp)
        b.run()
        poses, err, st = b.results()
        self._traces = b  # (a device read only when someone asks: not on the per-frame path)
        cur_frame.abs_pose[:] = poses[0]
        self.last_status = int(st[0])
        return float(err[0])


class FeatureAlignment:
    """FeatureAlignment(patchSize, level, numParameters) (src/feature_alignment.cpp:15-62)."""

    def __init__(self, patch_size, level=0, num_parameters=3, ctx=None):
        if num_parameters != 3:
            raise ValueError("FeatureAlignment estimates (u, v, bias): numParameters must be 3")
        self.patch_size, self.level = int(patch_size), int(level)
        self.ctx = ctx or default_context()
        self.last_status = None

    def align(self, ref_feature, cur_frame, pixel_pos):
        """pixel_pos (numpy float64[2]) is updated in place; returns the RMSE (NaN if out of frame)."""
        px = np.ascontiguousarray(pixel_pos, dtype=np.float64).reshape(1, 2).copy()
        err, st = self.align_batch(ref_feature.frame.image_pyramid.set, [0], cur_frame.image_pyramid.set, 0,
                                   ref_feature.pixel_position.reshape(1, 2), px, cur_frame.camera)
        pixel_pos[0], pixel_pos[1] = px[0, 0], px[0, 1]
        self.last_status = int(st[0])
        return float(err[0])

    def align_batch(self, ref_set, ref_frames, cur_set, cur_frame, ref_px, px_inout, camera):
        ref_px = np.ascontiguousarray(ref_px, dtype=np.float64)
        n = ref_px.shape[0]
        if px_inout.dtype != np.float64 or not px_inout.flags.c_contiguous or px_inout.shape != (n, 2):
            raise ValueError("px_inout must be a C-contiguous float64 (n, 2) array")
        rf = np.ascontiguousarray(np.broadcast_to(np.asarray(ref_frames, np.int32), (n,)))
        err = np.zeros(n)
        st = np.zeros(n, np.int32)
        cam = camera.as_c()
        check(lib().svo_feature_align(self.ctx.handle, ctypes.byref(cam), self.patch_size, ref_set.handle, ptr(rf), 0,
                                      cur_set.handle, int(cur_frame), n, ptr(ref_px), ptr(px_inout), ptr(err), ptr(st)))
        return err, st


    def align_many(self, ref_features, cur_frame, px_inout):
        """align() for every (ref_features[i], px_inout[i]) against cur_frame in one launch; each
        reference feature reads the gradient of its own frame (svo_feature_align_multi)."""
        n = len(ref_features)
        if px_inout.dtype != np.float64 or not px_inout.flags.c_contiguous or px_inout.shape != (n, 2):
            raise ValueError("px_inout must be a C-contiguous float64 (n, 2) array")
        err = np.zeros(n)
        st = np.zeros(n, np.int32)
        if n == 0:
            return err, st
        sets = (ctypes.c_void_p * n)(*[f.frame.image_pyramid.set.handle.value for f in ref_features])
        frames = np.zeros(n, np.int32)
        ref_px = np.ascontiguousarray([f.pixel_position for f in ref_features], dtype=np.float64)
        cam = cur_frame.camera.as_c()
        check(lib().svo_feature_align_multi(self.ctx.handle, ctypes.byref(cam), self.patch_size, sets, ptr(frames),
                                            cur_frame.image_pyramid.set.handle, 0, n, ptr(ref_px), ptr(px_inout),
                                            ptr(err), ptr(st)))
        return err, st


# ---------------------------------------------------------------- map reprojection
class Map:
    """Map(camera, cellSize) (src/map.cpp:15-19; grid :222-248): the reprojection half of the reference's
    map, reprojectMap (:260-478) with reprojectPoint (:481-492) and reprojectCell (:495-570),
    addNewCandidate (:586-593), addCandidateToFrame (:595-627) and removeMatchedCandidate (:629-634).

    The reference aligns candidates one FeatureAlignment(7, 0, 3) call at a time; here every alignment of
    a call runs in one launch (svo_feature_align_multi) and the decisions are replayed in the reference's
    order: reprojectCell accepts the first non-deleted candidate of a cell whatever its error, so the
    aligned set is fixed before the alignment (svo_map_reproject_plan); addCandidateToFrame aligns every
    candidate whose cell is free and then lets the first match of each cell win.  The cell order is a
    seeded permutation (the reference shuffles it with an unseeded std::random_device, :243-247)."""

    MAX_MATCHES = 150  # :474

    def __init__(self, camera, cell_size, seed=0, ctx=None):
        self.camera = camera
        self.cell_size = int(cell_size)
        self.grid_cols = int(math.ceil(camera.width / self.cell_size))
        self.grid_rows = int(math.ceil(camera.height / self.cell_size))
        n = self.grid_cols * self.grid_rows
        self.cell_orders = np.random.default_rng(seed).permutation(n).astype(np.int32)
        self.cell_visited = np.zeros(n, bool)  # never cleared by the reference (resetGrid :250-258)
        self.matches = 0
        self.trials = 0
        self.candidates = []  # [feature, point, matched]
        self.alignment = FeatureAlignment(7, 0, 3, ctx)
        self.key_frames = []
        self.native_seconds = 0.0  # time inside the C ABI calls (plan, projection, batched alignment)

    def cell_of(self, px):
        return int(px[1]) // self.cell_size * self.grid_cols + int(px[0]) // self.cell_size

    def reproject_map(self, ref_frame, cur_frame, overlap_keyframes):
        if ref_frame.last_keyframe is None:
            raise ValueError("reprojectMap needs refFrame->m_lastKeyframe")
        kfs = [ref_frame, ref_frame.last_keyframe]
        nfs = [len(kf.features) for kf in kfs]
        off = np.cumsum([0] + nfs).astype(np.int32)
        # the distinct points (their _PT rows) in first-seen order and each feature's index among them (-1: none)
        rows = np.concatenate([_point_rows(kf.features) for kf in kfs])
        valid = rows >= 0
        u, first, inv = np.unique(rows[valid], return_index=True, return_inverse=True)
        order = np.argsort(first, kind="stable")
        prow = u[order]
        rank = np.empty(len(u), np.int32)
        rank[order] = np.arange(len(u), dtype=np.int32)
        feat_point = np.full(max(len(rows), 1), -1, np.int32)
        feat_point[np.nonzero(valid)[0]] = rank[inv.reshape(-1)]
        npt = len(prow)
        pos = np.ascontiguousarray(_PT.pos[prow]) if npt else np.zeros((1, 3))
        ptype = _PT.type[prow] if npt else np.zeros(1, np.uint32)
        plast = _PT.last[prow] if npt else np.zeros(1, np.uint64)
        n_cells = len(self.cell_orders)
        overlap = np.zeros(len(kfs), np.int32)
        sel_feat = np.zeros(n_cells, np.int32)
        sel_cell = np.zeros(n_cells, np.int32)
        sel_px = np.zeros((n_cells, 2))
        n_sel, m, t = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        cam = self.camera.as_c()
        t0 = time.perf_counter()
        check(lib().svo_map_reproject_plan(ctypes.byref(cam), self.cell_size, n_cells, ptr(self.cell_orders),
                                           ptr(np.ascontiguousarray(cur_frame.abs_pose, np.float64)),
                                           ctypes.c_uint64(cur_frame.id), len(kfs), ptr(off), ptr(feat_point), npt,
                                           ptr(pos), ptr(ptype), ptr(plast), ptr(overlap), ctypes.byref(n_sel),
                                           ptr(sel_feat), ptr(sel_cell), ptr(sel_px), ctypes.byref(m),
                                           ctypes.byref(t)))
        self.native_seconds += time.perf_counter() - t0
        _PT.last[prow] = plast[:npt]
        for k, kf in enumerate(kfs):
            overlap_keyframes.append((kf, int(overlap[k])))
        self.matches, self.trials = m.value, t.value
        ns = n_sel.value
        f0, f1 = kfs[0].features, kfs[1].features
        n0 = nfs[0]
        chosen = [f0[i] if i < n0 else f1[i - n0] for i in sel_feat[:ns].tolist()]
        px = np.ascontiguousarray(sel_px[:ns])
        t0 = time.perf_counter()
        self.alignment.align_many(chosen, cur_frame, px)
        self.native_seconds += time.perf_counter() - t0
        pts = [f._point for f in chosen]
        new = Feature._many(cur_frame, px, 0, points=pts)
        # :558-569 (m_succeededProjection++, UNKNOWN -> GOOD past 10) on the points' rows; a point is planned at most
        # once per call (m_lastProjectedKFId), and the end state would be the same for repeats
        srow = np.fromiter((p._i for p in pts), np.int64, count=ns)
        np.add.at(_PT.succ, srow, 1)
        up = (_PT.type[srow] == PointType.UNKNOWN) & (_PT.succ[srow] > 10)
        _PT.type[srow[up]] = PointType.GOOD
        for point, feature in zip(pts, new):
            point.features.append(feature)
        cur_frame.features.extend(new)
        self.cell_visited[sel_cell[:ns]] = True

    def add_new_candidate(self, feature, point, matched=False):
        point.type = PointType.CANDIDATE
        self.candidates.append([feature, point, matched])

    def add_candidate_to_frame(self, frame):
        if not self.candidates:
            return
        rows = np.fromiter((c[1]._i for c in self.candidates), np.int64, count=len(self.candidates))
        pos = np.ascontiguousarray(_PT.pos[rows])
        t0 = time.perf_counter()
        px0 = frame.world2image(pos)
        self.native_seconds += time.perf_counter() - t0
        w, h = frame.camera.width, frame.camera.height
        # inside the 3-px border (isInFrame(px, 3)), cell not visited yet (:600-606); cell_of truncates like int()
        inside = (px0[:, 0] >= 3) & (px0[:, 1] >= 3) & (px0[:, 0] < w - 3) & (px0[:, 1] < h - 3)
        cell = np.zeros(len(px0), np.int64)
        cell[inside] = (px0[inside, 1].astype(np.int64) // self.cell_size * self.grid_cols
                        + px0[inside, 0].astype(np.int64) // self.cell_size)
        elig = np.nonzero(inside)[0]
        elig = elig[~self.cell_visited[cell[elig]]]
        cells = cell[elig].tolist()
        px = np.ascontiguousarray(px0[elig])
        cands = [self.candidates[i][0] for i in elig.tolist()]
        t0 = time.perf_counter()
        err, _ = self.alignment.align_many(cands, frame, px)
        self.native_seconds += time.perf_counter() - t0
        ok = (err < 50.0).tolist()
        acc = []
        for j, i in enumerate(elig.tolist()):  # the reference's order: a cell taken earlier in this loop is skipped
            if not ok[j] or self.cell_visited[cells[j]]:
                continue
            self.cell_visited[cells[j]] = True
            acc.append((j, i))
        if acc:
            pts = [self.candidates[i][1] for _, i in acc]
            new = Feature._many(frame, px[[j for j, _ in acc]], 0, points=pts)
            frame.features.extend(new)
            for (_, i), point, feature in zip(acc, pts, new):
                feat = self.candidates[i][0]
                point.features.append(feat)
                point.features.append(feature)
                feat.set_point(point)
                self.candidates[i][2] = True
        self.candidates = [c for c in self.candidates if not c[2]]  # removeMatchedCandidate


# ---------------------------------------------------------------- depth filter
DEPTH_SEED = np.dtype([("a", "f8"), ("b", "f8"), ("mu", "f8"), ("sigma", "f8"), ("var", "f8"), ("max_depth", "f8"),
                       ("px", "f8", 2), ("bearing", "f8", 3), ("kf", "i4"), ("valid", "i4")])  # svo_depth_seed


def depth_seeds(px, bearing, depth_mean, depth_min, kf=0):
    """MixedGaussianFilter(feature, depthMean, depthMin) for each feature (src/mixed_gaussian_filter.cpp:7-24)."""
    n = len(px)
    s = np.zeros(n, DEPTH_SEED)
    one = _capi.SvoDepthSeed()
    check(lib().svo_depth_seed_init(float(depth_mean), float(depth_min), ctypes.byref(one)))
    for k in ("a", "b", "mu", "sigma", "var", "max_depth"):
        s[k] = getattr(one, k)
    s["px"], s["bearing"], s["kf"], s["valid"] = px, bearing, kf, 1
    return s


def depth_update(camera, keyframes, cur, cur_pose, seeds, ctx=None):
    """DepthEstimator::updateFilters for `seeds` (DEPTH_SEED array) against the current frame.

    keyframes: list of (PyramidSet, frame index, pose[7]); seed["kf"] indexes it.  cur: (PyramidSet, frame).
    Returns (survivors, outcome[n], cand_points[m, 3], cand_seed[m]) in the reference's orders."""
    ctx = ctx or default_context()
    seeds = np.ascontiguousarray(seeds, DEPTH_SEED).copy()
    n = len(seeds)
    nk = len(keyframes)
    sets = (ctypes.c_void_p * max(nk, 1))(*[k[0].handle.value for k in keyframes])
    frames = np.array([k[1] for k in keyframes] or [0], np.int32)
    poses = np.ascontiguousarray(np.array([k[2] for k in keyframes] or [np.zeros(7)], np.float64))
    cp = np.ascontiguousarray(cur_pose, np.float64)
    outcome = np.zeros(max(n, 1), np.int32)
    pts = np.zeros((max(n, 1), 3))
    cs = np.zeros(max(n, 1), np.int32)
    n_out, n_cand = ctypes.c_int32(), ctypes.c_int32()
    cam = camera.as_c()
    check(lib().svo_depth_update(ctx.handle, ctypes.byref(cam), nk, ctypes.cast(sets, ctypes.c_void_p), ptr(frames),
                                 ptr(poses), cur[0].handle, int(cur[1]), ptr(cp), n, ptr(seeds), ctypes.byref(n_out),
                                 ptr(outcome), ptr(pts), ptr(cs), ctypes.byref(n_cand)))
    return seeds[:n_out.value].copy(), outcome[:n], pts[:n_cand.value].copy(), cs[:n_cand.value].copy()


class DepthEstimator:
    """DepthEstimator (include/depth_estimator.hpp, src/depth_estimator.cpp) without its worker thread:
    add_keyframe = initializeFilters (:175-190) for the keyframe's features without a point,
    update_filters = updateFilters (:192-309).  Converged seeds become candidates (Map::addNewCandidate,
    src/map.cpp:586-593): (feature, Point) pairs in the reference's order."""

    def __init__(self, ctx=None):
        self.ctx = ctx or default_context()
        self.keyframes = []   # Frame objects; seed["kf"] indexes this list
        self.features = []    # the Feature behind every seed, same order as self.seeds
        self.seeds = np.zeros(0, DEPTH_SEED)
        self.candidates = []

    def add_keyframe(self, frame, depth_mean, depth_min):
        feats = [f for f in frame.features if f.point is None]
        kf = len(self.keyframes)
        self.keyframes.append(frame)
        if feats:
            px = np.array([f.pixel_position for f in feats])
            br = np.array([f.bearing_vec for f in feats])
            self.seeds = np.concatenate([self.seeds, depth_seeds(px, br, depth_mean, depth_min, kf)])
            self.features += feats

    def number_filters(self):
        return len(self.seeds)

    def update_filters(self, frame):
        if len(self.seeds) == 0:
            return []
        kfs = [(k.image_pyramid.set, 0, k.abs_pose) for k in self.keyframes]
        surv, outcome, pts, cs = depth_update(frame.camera, kfs, (frame.image_pyramid.set, 0), frame.abs_pose,
                                              self.seeds, self.ctx)
        new = [(self.features[i], Point(p)) for i, p in zip(cs, pts)]
        self.candidates += new
        keep = [i for i in range(len(self.seeds)) if outcome[i] in (1, 2) and self.seeds[i]["valid"]]  # still seeds
        self.features = [self.features[i] for i in keep]
        self.seeds = surv
        return new


# ---------------------------------------------------------------- feature selection
class FeatureSelection:
    """FeatureSelection(width, height, cellSize) (src/feature_selection.cpp:19-287).

    The occupancy grid ((height // cellSize + 1) x (width // cellSize + 1) cells) lives here on the host
    like the reference's member; detection reads the frame's device-resident level-0 gradient plane."""

    def __init__(self, width, height, cell_size, ctx=None):
        self.ctx = ctx or default_context()
        r, c = ctypes.c_int32(), ctypes.c_int32()
        check(lib().svo_feature_grid_size(int(width), int(height), int(cell_size), ctypes.byref(r), ctypes.byref(c)))
        self.width, self.height, self.cell_size = int(width), int(height), int(cell_size)
        self.grid_rows, self.grid_cols = r.value, c.value
        self.occupancy_grid = np.zeros((self.grid_rows, self.grid_cols), np.uint8)
        self.last_keypoints = 0

    def set_existing_features(self, features):  # :268-274
        for f in features:
            self.set_cell_in_grid_occupancy(f.pixel_position)

    def set_cell_in_grid_occupancy(self, location):  # :276-282 (uint32 truncation of the division)
        self.occupancy_grid[int(location[1] / self.cell_size), int(location[0] / self.cell_size)] = 1

    def reset_grid_occupancy(self):  # :284-287
        self.occupancy_grid[:] = 0

    def _emit(self, frame, px, resp, n):
        frame.features.extend(Feature._many(frame, px[:n], 0, gradient_magnitude=resp[:n].tolist(),
                                            feature_type=Feature.EDGE))
        return n

    def detect(self, frame, detection_threshold):
        """The device step alone: keys (response << 24 | y * width + x) above the threshold, row-major."""
        cap = self.width * self.height
        keys = np.zeros(cap, np.uint32)
        n = ctypes.c_int32()
        check(lib().svo_feature_detect(self.ctx.handle, frame.image_pyramid.set.handle, 0, int(detection_threshold),
                                       cap, ptr(keys), ctypes.byref(n)))
        return keys[:n.value]

    def gradient_magnitude_with_ssc(self, frame, detection_threshold, number_candidate, use_bucketing):
        """:27-89 — adds the selected features to `frame` (EDGE, level 0); returns how many."""
        cap = self.grid_rows * self.grid_cols if use_bucketing else max(4 * int(number_candidate), 1024)
        while True:
            px = np.zeros((cap, 2))
            resp = np.zeros(cap)
            n, nk = ctypes.c_int32(), ctypes.c_int32()
            occ = self.occupancy_grid.copy()
            rc = lib().svo_feature_select_ssc(self.ctx.handle, frame.image_pyramid.set.handle, 0,
                                              int(detection_threshold), int(number_candidate), int(bool(use_bucketing)),
                                              self.cell_size, ptr(occ), cap, ptr(px), ptr(resp), ctypes.byref(n),
                                              ctypes.byref(nk))
            if rc == _capi.SVO_ERR_ARG and not use_bucketing and cap < self.width * self.height:
                cap = self.width * self.height  # SSC kept more than the first guess
                continue
            check(rc)
            break
        self.occupancy_grid[:] = occ
        self.last_keypoints = nk.value
        return self._emit(frame, px, resp, n.value)

    def gradient_magnitude_by_value(self, frame, detection_threshold, use_bucketing=True):
        """:91-143 — bucketing branch (the reference's other branch reads the 8-bit magnitude as float)."""
        if not use_bucketing:
            raise ValueError("gradientMagnitudeByValue without bucketing reads the u8 magnitude as float "
                             "(src/feature_selection.cpp:150); not supported")
        cap = self.grid_rows * self.grid_cols
        px = np.zeros((cap, 2))
        resp = np.zeros(cap)
        n = ctypes.c_int32()
        occ = self.occupancy_grid.copy()
        check(lib().svo_feature_select_by_value(self.ctx.handle, frame.image_pyramid.set.handle, 0,
                                                int(detection_threshold), self.cell_size, ptr(occ), cap, ptr(px),
                                                ptr(resp), ctypes.byref(n)))
        self.occupancy_grid[:] = occ
        return self._emit(frame, px, resp, n.value)


SCALE_AUTO, SCALE_K2R, SCALE_K2V, SCALE_K2 = 0, 1, 2, 3  # include/svo_c.h SVO_SCALE_*


def robust_scale_capacity(impl):
    """Largest residual vector (features x patch^2) the kernel `impl` takes (svo_robust_scale_capacity)."""
    v = ctypes.c_int64()
    check(lib().svo_robust_scale_capacity(int(impl), ctypes.byref(v)))
    return int(v.value)
SCALE_K2V_MAX_SLOTS = 128 * 512             # K2V holds the vector in registers (align_refv.hip LayC)
SCALE_K2V_LAYB_SLOTS = 118 * 512            # (LayB)
SCALE_K2V_LAYA_SLOTS = 98 * 512             # (LayA: the faster layout, the config-2 shape)


def debug_robust_scale(values, n_valid, ctx=None, impl=SCALE_AUTO, diagnostics=False):
    """svo_debug_robust_scale: algorithm::computeMAD(values, n_valid) with the reference's libstdc++
    nth_element post-state (MEDIAN_REFERENCE), on the device with kernel `impl` (SCALE_*); returns (median,
    mad), or (median, mad, diagnostics) with diagnostics=True (the 204 doubles after them, see
    include/svo_c.h).  values: the full residual vector, invisible slots = DBL_MAX (src/optimizer.cpp:387-396)."""
    ctx = ctx or default_context()
    v = np.ascontiguousarray(values, np.float64)
    # without diagnostics only med / mad come back, and K2V runs the product kernel's own code path (svo_c.h)
    out = np.zeros(206 if diagnostics else 2)
    check(lib().svo_debug_robust_scale(ctx.handle, ptr(v), len(v), int(n_valid), int(impl), ptr(out), len(out)))
    if diagnostics:
        return float(out[0]), float(out[1]), out[2:].copy()
    return float(out[0]), float(out[1])


# ---------------------------------------------------------------- pose-only bundle adjustment
def pose_optimize_batch(feat_off, bearing, point, has_point, vis, poses, ctx=None):
    """svo_pose_optimize over arrays: frame f owns rows feat_off[f]:feat_off[f+1].  vis (uint8, in/out) and
    poses ((F, 7), in/out) are updated in place; returns (err, status)."""
    ctx = ctx or default_context()
    feat_off = np.ascontiguousarray(feat_off, np.int32)
    F = len(feat_off) - 1
    for a, dt in ((vis, np.uint8), (poses, np.float64)):
        if a.dtype != dt or not a.flags.c_contiguous:
            raise ValueError("vis must be C-contiguous uint8 and poses C-contiguous float64")
    bearing = np.ascontiguousarray(bearing, np.float64)
    point = np.ascontiguousarray(point, np.float64)
    has_point = np.ascontiguousarray(has_point, np.uint8)
    err = np.zeros(F)
    st = np.zeros(F, np.int32)
    check(lib().svo_pose_optimize(ctx.handle, F, ptr(feat_off), ptr(bearing), ptr(point), ptr(has_point), ptr(vis),
                                  ptr(poses), ptr(err), ptr(st)))
    return err, st


class BundleAdjustment:
    """BundleAdjustment(camera, level, numParameters) — optimizePose (src/bundle_adjustment.cpp:30-166).

    ref_visibility is the member m_refVisibility: optimizePose's residual step reads the flags the
    previous call left (a fresh object returns NaN and moves nothing), see include/svo_c.h."""

    def __init__(self, camera, level=0, num_parameters=6, ctx=None):
        self.camera, self.level = camera, int(level)
        self.ctx = ctx or default_context()
        self.ref_visibility = np.zeros(0, np.uint8)
        self.last_status = None

    def optimize_pose(self, frame):
        n = len(frame.features)
        if n == 0:  # :37-38
            return 0.0
        vis = np.zeros(n, np.uint8)
        k = min(n, len(self.ref_visibility))
        vis[:k] = self.ref_visibility[:k]  # m_refVisibility.resize(n, false)
        bearing = np.array([f.bearing_vec for f in frame.features], np.float64).reshape(n, 3)
        has = np.array([f.point is not None for f in frame.features], np.uint8)
        point = np.array([f.point.position if f.point is not None else (0.0, 0.0, 0.0) for f in frame.features],
                         np.float64).reshape(n, 3)
        poses = np.ascontiguousarray(frame.abs_pose, np.float64).reshape(1, 7).copy()
        err, st = pose_optimize_batch([0, n], bearing, point, has, vis, poses, self.ctx)
        self.ref_visibility = vis
        frame.abs_pose = poses[0].copy()
        self.last_status = int(st[0])
        return float(err[0])
