"""The reference's robust scale bit for bit: median_mode SVO_MEDIAN_REFERENCE (K2V, csrc/align_refv.hip, for
vectors of <= 60 416 slots in two register layouts; K2R, csrc/align_ref.hip, for any size).

algorithm::computeMedian (src/algorithm.cpp:834-853) runs std::nth_element on the full residual vector and
reads vec[n/2 - 1] from libstdc++'s post-partition state.  K2R re-runs that introselect on the device.

CPU: tests/cpp/introselect_model.cpp — the round formulation K2R uses (counts, prefix sums, the crossing
     max-min) against the real std::nth_element, whole final arrays, including inputs that exhaust the
     depth limit (heap select).
GPU: svo_debug_robust_scale (the K2V and K2R selections on arbitrary vectors) and whole alignments in
     MEDIAN_REFERENCE mode against the oracle's std::nth_element (oracle median_mode 0):
       median / MAD / sigma of every vector ............. bit-exact
       per-level n_vis, status; first-level median / MAD / sigma ... bit-exact
       final pose ........................................ 1e-9 (Sophus params, sign-canonical)
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle as O
import svo_amd
import svo_amd.synth as synth
from common import canon, gpu_batch, make_pairs, oracle_align

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBL_MAX = np.finfo(np.float64).max


def test_introselect_model_matches_std_nth_element(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "imodel"
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "introselect_model.cpp")])
    r = subprocess.run([str(exe), "1500"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout


def oracle_med_mad(v, n):
    """computeMAD with the reference's nth_element (oracle median_mode 0)."""
    med = O.median(v, n, 0)
    d = np.abs(v - med)
    d[v >= DBL_MAX] = DBL_MAX
    return med, O.median(d, n, 0)


def residual_vectors():
    rng = np.random.default_rng(5)
    out = []
    for n_feat in (1, 2, 3, 7, 40, 333, 2000):
        for p_vis in (1.0, 0.8, 0.3):
            v = rng.normal(0, 8, n_feat * 25)
            vis = np.repeat(rng.random(n_feat) < p_vis, 25)
            if not vis.any():
                vis[:25] = True
            v[~vis] = DBL_MAX
            out.append((f"normal n={n_feat} vis={p_vis}", v))
    v = np.round(rng.normal(0, 6, 50000))  # heavy ties (integer residuals)
    v[np.repeat(rng.random(2000) < 0.25, 25)] = DBL_MAX
    out.append(("integers", v))
    v = rng.integers(-2, 3, 50000) * 0.5 + rng.integers(0, 2, 50000) * 2.384185791015625e-07 / 3  # same-cell ties
    out.append(("same-key cells", v))
    v = rng.normal(0, 8, 49999)
    out.append(("odd length", v))
    v = np.clip(rng.standard_cauchy(60000) * 20, -255, 255)
    out.append(("cauchy, clamped", v))
    v = np.full(1000, 3.0)
    out.append(("constant", v))
    for n in (4, 5, 6, 17):
        out.append((f"tiny {n}", rng.normal(0, 1, n)))
    return out


IMPLS = [pytest.param(svo_amd.SCALE_K2V, id="K2V"), pytest.param(svo_amd.SCALE_K2R, id="K2R")]


def _fits(impl, v):
    return impl != svo_amd.SCALE_K2V or len(v) <= svo_amd.SCALE_K2V_MAX_SLOTS


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("case", residual_vectors(), ids=lambda c: c[0])
def test_debug_robust_scale_matches_nth_element(case, impl):
    _, v = case
    if not _fits(impl, v):
        pytest.skip("vector larger than K2V's registers (K2R covers it)")
    n = int((v < DBL_MAX).sum())
    med, mad = svo_amd.debug_robust_scale(v, n, impl=impl)
    med_c, mad_c = oracle_med_mad(v, n)
    assert med == med_c and mad == mad_c, (med, med_c, mad, mad_c)


@pytest.mark.gpu
def test_debug_robust_scale_k2v_extremes():
    """K2V at the capacity of each register layout (LayA 50 176 slots, LayB 60 416, LayC 65 536: every register row
    and LDS row in use), vectors whose first round needs a chunked exchange (Ks > the mailbox: reversed order; LayB's
    4 352-slot mailbox chunks most of its first rounds), all-invisible tails, and n_valid far below the length; each
    through the diagnostics kernel and through the product kernel."""
    rng = np.random.default_rng(11)
    cases = []
    for cap in sorted({svo_amd.SCALE_K2V_LAYA_SLOTS, svo_amd.SCALE_K2V_LAYB_SLOTS, svo_amd.SCALE_K2V_MAX_SLOTS}):
        v = rng.normal(0, 8, cap)
        v[np.repeat(rng.random(cap // 25 + 1) < 0.2, 25)[:len(v)]] = DBL_MAX
        cases.append(v)
    desc = len(cases)
    cases.append(np.arange(50000, 0, -1, dtype=np.float64) * 0.01)  # descending: maximal swaps per round
    cases.append(np.arange(60000, 0, -1, dtype=np.float64) * 0.01)  # (LayB)
    cases.append(np.arange(65536, 0, -1, dtype=np.float64) * 0.01)  # (LayC: a 1344-swap mailbox)
    cases.append(np.concatenate([rng.normal(0, 3, 30000), np.full(20000, DBL_MAX)]))
    w = rng.normal(0, 3, 40000)
    w[rng.random(40000) < 0.9] = DBL_MAX
    cases.append(w)
    chunked = []
    for v in cases:
        n = int((v < DBL_MAX).sum())
        med, mad, dg = svo_amd.debug_robust_scale(v, n, impl=svo_amd.SCALE_K2V, diagnostics=True)
        med_c, mad_c = oracle_med_mad(v, n)
        assert med == med_c and mad == mad_c, (len(v), n, med, med_c, mad, mad_c, dg[:10])
        chunked.append(dg[4] + dg[9])  # block rounds whose exchange ran in mailbox chunks (both passes)
        # the product kernel on the same vector (its layouts' one-wave size and wave retirement)
        pm, pd = svo_amd.debug_robust_scale(v, n, impl=svo_amd.SCALE_K2V)
        assert pm == med_c and pd == mad_c, ("product", len(v), n, pm, med_c, pd, mad_c)
    assert all(chunked[desc + i] >= 1 for i in range(3)), chunked  # the descending vectors exercise the chunked exchange


@pytest.mark.gpu
def test_debug_robust_scale_k2v_rejects_large_vectors():
    with pytest.raises(svo_amd.SvoError):
        svo_amd.debug_robust_scale(np.zeros(svo_amd.SCALE_K2V_MAX_SLOTS + 1), 10, impl=svo_amd.SCALE_K2V)


@pytest.mark.gpu
def test_debug_robust_scale_heap_select_path(tmp_path):
    """Inputs that exhaust introselect's depth limit: written by the C++ model's adversary."""
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "imodel"
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "introselect_model.cpp")])
    for n in (200, 5000, 50000):
        out = tmp_path / f"k{n}.bin"
        subprocess.check_call([str(exe), "killer", str(n), str(n // 2), str(out)])
        raw = np.fromfile(out, np.float64)
        v = raw / n * 500.0 - 250.0  # order-preserving map into the residual range
        med_c, mad_c = oracle_med_mad(v, len(v))
        for impl in (svo_amd.SCALE_K2V, svo_amd.SCALE_K2R):
            med, mad = svo_amd.debug_robust_scale(v, len(v), impl=impl)
            assert med == med_c and mad == mad_c, (n, impl, med, med_c, mad, mad_c)


def _check_ref_traces(tr_gpu, tr_cpu, min_level, max_level):
    for l in range(max_level, min_level - 1, -1):
        g, c = tr_gpu[l], tr_cpu[l]
        assert (g.n_ref_vis, g.n_vis, g.status) == (c.n_ref_vis, c.n_vis, c.status), (l, g.n_vis, c.n_vis)
        if l == max_level:  # later levels start from poses that differ by ~1e-13 (summation order)
            assert (g.median, g.mad, g.sigma) == (c.median, c.mad, c.sigma), (l, g.median, c.median, g.mad, c.mad)
        else:
            assert abs(g.sigma - c.sigma) <= 1e-9 * abs(c.sigma), l


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [dict(patch=5, min_level=0, max_level=4, nf=2000),   # config 2
                                 dict(patch=4, min_level=0, max_level=2, nf=200),    # config 1 (5x5 footprint)
                                 dict(patch=7, min_level=1, max_level=3, nf=600)])
def test_align_reference_mode_matches_oracle(cfg):
    pairs = make_pairs(4, n_features=cfg["nf"], patch_size=cfg["patch"])
    b, _ = gpu_batch(pairs, cfg["patch"], cfg["min_level"], cfg["max_level"], median_mode=svo_amd.MEDIAN_REFERENCE)
    b.run()
    poses, err, st = b.results()
    for i, s in enumerate(pairs):
        pose_c, err_c, st_c, tr_c = oracle_align(s, cfg["patch"], cfg["min_level"], cfg["max_level"], mode=0)
        _check_ref_traces(b.traces(i), tr_c, cfg["min_level"], cfg["max_level"])
        assert np.abs(canon(poses[i]) - canon(pose_c)).max() <= 1e-9
        assert abs(err[i] - err_c) <= 1e-9 * abs(err_c)
        assert st[i] == st_c


@pytest.mark.gpu
@pytest.mark.parametrize("n_slots", [98000, 300000])
def test_debug_robust_scale_large_vectors(n_slots):
    """Vectors past 64512 slots take K2R's large instantiation (step records in the pair's global scratch,
    17 register rows of block prefixes): patch 7 at 2000 features is 98000 slots."""
    rng = np.random.default_rng(n_slots)
    v = rng.normal(0, 8, n_slots)
    v[rng.random(n_slots) < 0.15] = DBL_MAX
    n = int((v < DBL_MAX).sum())
    med, mad = svo_amd.debug_robust_scale(v, n, impl=svo_amd.SCALE_K2R)
    med_c, mad_c = oracle_med_mad(v, n)
    assert med == med_c and mad == mad_c, (med, med_c, mad, mad_c)


@pytest.mark.gpu
def test_align_reference_mode_large_vector():
    """A whole alignment whose residual vector exceeds 64512 slots (patch 7, 2000 features: 98000)."""
    pairs = make_pairs(2, n_features=2000, patch_size=7)
    b, _ = gpu_batch(pairs, 7, 1, 3, median_mode=svo_amd.MEDIAN_REFERENCE)
    b.run()
    poses, err, st = b.results()
    for i, s in enumerate(pairs):
        pose_c, err_c, st_c, tr_c = oracle_align(s, 7, 1, 3, mode=0)
        _check_ref_traces(b.traces(i), tr_c, 1, 3)
        assert np.abs(canon(poses[i]) - canon(pose_c)).max() <= 1e-9
        assert st[i] == st_c
