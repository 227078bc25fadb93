"""CPU: Frame.feature_arrays caches the SoA gather of a frame's features (align() no longer
re-gathers 2000 Feature objects per call).  Every change the reference's code makes between two align() calls on
the same frames -- features appended / removed / replaced, a feature's pixel position or point reassigned, a
point moved -- must invalidate the cache, and the cached arrays must equal the plain per-call gather."""
import numpy as np

import svo_amd
from svo_amd import core


class _Cam:
    def inverse_project2d(self, px):  # a stand-in bearing (the cache only moves the numbers)
        return np.array([px[0] * 1e-3, px[1] * 1e-3, 1.0])


def _frame():
    # Frame without a device pyramid (Frame.__init__ builds one on the GPU): only the feature bookkeeping
    fr = core.Frame.__new__(core.Frame)
    fr.camera = _Cam()
    fr._feat_ver = [0]
    fr._soa = None
    fr.features = []
    return fr


def _plain(frames):
    feats = [f for fr in frames for f in fr.features]
    px = np.array([f.pixel_position for f in feats], np.float64).reshape(-1, 2)
    br = np.array([f.bearing_vec for f in feats], np.float64).reshape(-1, 3)
    pt = np.array([f.point.position if f.point is not None else np.zeros(3) for f in feats], np.float64).reshape(-1, 3)
    hp = np.array([f.point is not None for f in feats], np.uint8)
    return px, br, pt, hp


def _same(frames):
    got = core._feature_arrays(frames)
    want = _plain(frames)
    if len(want[0]) == 0:
        return got[0].shape == (1, 2)
    return all(np.array_equal(g, w) and g.dtype == w.dtype for g, w in zip(got, want))


def test_cache_follows_every_change():
    rng = np.random.default_rng(5)
    ref, kf = _frame(), _frame()
    for fr, n in ((ref, 300), (kf, 200)):
        for i in range(n):
            p = svo_amd.Point(rng.normal(size=3)) if i % 7 else None
            fr.add_feature(svo_amd.Feature(fr, rng.uniform(0, 1000, 2), point=p))
    assert _same([ref, kf])
    a1 = ref.feature_arrays()
    assert ref.feature_arrays()[0] is a1[0]  # cached: the same arrays come back
    # a feature's pixel position / point reassigned
    ref.features[3].pixel_position = [1.5, 2.5]
    assert ref.feature_arrays()[0] is not a1[0] and _same([ref, kf])
    ref.features[0].point = None
    assert _same([ref, kf])
    kf.features[1].set_point(svo_amd.Point([9.0, 8.0, 7.0]))
    assert _same([ref, kf])
    # a point moved (any frame's features may hold it)
    q = next(f.point for f in kf.features if f.point is not None)
    before = kf.feature_arrays()
    q.position = [1.0, 2.0, 3.0]
    after = kf.feature_arrays()
    assert after[0] is before[0] and after[2] is not before[2] and _same([ref, kf])
    # list mutations: append, pop, remove, slice assignment, clear, +=, reassignment of the list
    ref.add_feature(svo_amd.Feature(ref, [5.0, 6.0], point=svo_amd.Point([1, 1, 1])))
    assert _same([ref, kf])
    ref.features.pop(10)
    assert _same([ref, kf])
    ref.features.remove(ref.features[20])
    assert _same([ref, kf])
    ref.features[5:9] = [svo_amd.Feature(ref, [1.0, 1.0])]
    assert _same([ref, kf])
    del ref.features[0]
    assert _same([ref, kf])
    ref.features += [svo_amd.Feature(ref, [2.0, 2.0], point=svo_amd.Point([0, 0, 5]))]
    assert isinstance(ref.features, core._FeatureList) and _same([ref, kf])
    ref.features.reverse()
    assert _same([ref, kf])
    kf.features = kf.features[:50]
    assert isinstance(kf.features, core._FeatureList) and _same([ref, kf])
    kf.features.clear()
    assert _same([ref, kf]) and _same([kf])


def test_rows_rejects_mixed_dtypes():
    """a duck-typed row that is not float64 (int64 has the same byte length) must be converted, not
    reinterpreted."""
    vals = [np.array([1.0, 2.0]), np.array([3, 4], np.int64)]
    assert np.array_equal(core._rows(vals, 2), [[1.0, 2.0], [3.0, 4.0]])


def test_positions_read_only_and_point_construction_keeps_caches():
    """in-place edits of a cached position raise instead of leaving the cache stale; constructing a
    Point (in no frame yet) does not invalidate other frames' cached point arrays; reassigning Feature.frame
    invalidates both frames."""
    import pytest
    fr, other = _frame(), _frame()
    p = svo_amd.Point([1.0, 2.0, 3.0])
    f = svo_amd.Feature(fr, np.array([10.0, 20.0]), point=p)
    fr.add_feature(f)
    with pytest.raises(ValueError):
        f.pixel_position[0] = 5.0
    with pytest.raises(ValueError):
        p.position += 1.0
    src = np.array([1.0, 1.0])
    g = svo_amd.Feature(fr, src)
    assert src.flags.writeable  # the caller's array is copied, not frozen
    fr.add_feature(g)
    a = fr.feature_arrays()
    svo_amd.Point([4.0, 5.0, 6.0])  # a new point: no frame holds it
    assert fr.feature_arrays()[2] is a[2]
    other.add_feature(g)
    b = other.feature_arrays()
    g.frame = other
    assert fr.feature_arrays()[0] is not a[0] and other.feature_arrays()[0] is not b[0]
    assert _same([fr]) and _same([other])


def test_point_copies_own_their_row():
    """copy.copy / deepcopy / pickle of a Point allocate a row of their own (copying the row index would
    alias one row between two Points and free it twice)."""
    import copy
    import pickle
    p = svo_amd.Point([1.0, 2.0, 3.0])
    p.type = svo_amd.PointType.GOOD
    p.last_projected_kf_id = 7
    p.succeeded_projection = 3
    for q in (copy.copy(p), copy.deepcopy(p), pickle.loads(pickle.dumps(p))):
        assert q._i != p._i
        assert np.array_equal(q.position, p.position) and q.type == p.type
        assert q.last_projected_kf_id == 7 and q.succeeded_projection == 3 and q.failed_projection == 0
        q.position = [9.0, 9.0, 9.0]  # the copy's row is its own
        assert np.array_equal(p.position, [1.0, 2.0, 3.0])
    free0 = len(core._PT.free)
    del q
    import gc
    gc.collect()
    assert len(set(core._PT.free)) == len(core._PT.free) >= free0  # no row on the free list twice
