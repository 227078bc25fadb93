"""K2V reproduces libstdc++'s introselect round for round (median_mode SVO_MEDIAN_REFERENCE).

The robust scale of the reference (src/algorithm.cpp:834-865) reads vec[n/2 - 1] from std::nth_element's
post-state, so every partition round has to happen exactly as libstdc++ does it.  tests/introselect_rounds.py
restates the rounds in numpy (the round form of tests/cpp/introselect_model.cpp, which is checked there against the
real std::nth_element); the CPU tests pin that restatement to the oracle's std::nth_element path.  The GPU tests
turn on the debug kernel's round trace (svo_debug_robust_scale with out_len > 206: per round the segment, pivot, Ks,
#GE, #LE, cut and the whole vector after the round) and require, for every block round, every one-wave round and
every one-row round of both passes:
    segment, pivot, Ks, #GE, #LE, cut ......... equal to the model's
    the kept segment's values .................. bit-equal to the model's array
"""
import numpy as np
import pytest

import introselect_rounds as IR
import oracle as O

DBL_MAX = np.finfo(np.float64).max
HEAD = 8


def residual_like(ns, seed, vis=0.8, ints=False):
    rng = np.random.default_rng(seed)
    v = np.round(rng.normal(0, 6, ns)) if ints else rng.normal(0, 8, ns)
    hide = np.repeat(rng.random(ns // 25 + 1) > vis, 25)[:ns]
    v[hide] = DBL_MAX
    if not (v < DBL_MAX).any():
        v[0] = 0.0
    return v, int((v < DBL_MAX).sum())


FAMILIES = [("normal", 50000, 1, 0.8, False), ("normal", 60000, 1, 0.8, False), ("normal", 65000, 8, 0.8, False), ("normal", 65536, 9, 0.9, False), ("normal", 50176, 3, 1.0, False),
            ("integers", 50000, 4, 0.9, True), ("normal", 12000, 5, 0.7, False), ("integers", 3000, 6, 1.0, True),
            ("normal", 700, 7, 0.8, False)]


@pytest.mark.parametrize("fam", FAMILIES, ids=[f"{f[0]}-{f[1]}" for f in FAMILIES])
def test_round_model_matches_oracle(fam):
    """CPU: the numpy rounds give the oracle's std::nth_element median and MAD."""
    _, ns, seed, vis, ints = fam
    v, n = residual_like(ns, seed, vis, ints)
    med, mad = IR.robust_scale(v, n)
    med_o = O.median(v, n, 0)
    d = np.abs(v - med_o)
    d[v >= DBL_MAX] = DBL_MAX
    assert med == med_o and mad == O.median(d, n, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("fam", FAMILIES, ids=[f"{f[0]}-{f[1]}" for f in FAMILIES])
def test_k2v_every_round_matches_model(fam):
    import svo_amd
    from svo_amd import _capi
    _, ns, seed, vis, ints = fam
    v, n = residual_like(ns, seed, vis, ints)
    nrec = 96
    out = np.zeros(206 + nrec * (HEAD + ns))
    ctx = svo_amd.default_context()
    _capi.check(_capi.lib().svo_debug_robust_scale(ctx.handle, _capi.ptr(v), ns, n, svo_amd.SCALE_K2V, _capi.ptr(out),
                                                   len(out)))
    recs = out[206:].reshape(nrec, HEAD + ns)
    nth = n // 2
    ri = 0
    med = None
    for P in range(2):
        x = v if P == 0 else np.where(v >= DBL_MAX, DBL_MAX, np.abs(v - med))
        gen = IR.rounds(x, nth)
        lo = None
        try:
            while True:
                f0, l0, p, ks, ng, nl, cut, a = next(gen)
                h = recs[ri, :HEAD]
                got = (int(h[0]) % 10, int(h[1]), int(h[2]), h[3], int(h[4]), int(h[5]), int(h[6]), int(h[7]))
                assert got == (P, f0, l0, p, ks, ng, nl, cut), f"round {ri} (pass {P}, kind {int(h[0]) // 10})"
                first, last = (cut, l0) if cut <= nth else (f0, cut)
                vec = recs[ri, HEAD:]
                bad = np.nonzero(vec[first:last] != a[first:last])[0]
                assert len(bad) == 0, f"round {ri}: kept segment differs at {(bad[:8] + first).tolist()}"
                if cut == nth and lo is None and nth >= 1:
                    lo = float(a[nth - 1])
                ri += 1
        except StopIteration as e:
            first, last, a = e.value
        assert last - first <= 3
        a[first:last] = np.sort(a[first:last])
        hi = float(a[nth])
        lo = lo if lo is not None else float(a[nth - 1])
        r = (lo + hi) / 2.0 if ns % 2 == 0 and nth >= 1 else hi
        if P == 0:
            med = r
            assert out[0] == r
        else:
            assert out[1] == r
    assert ri >= 10 or ns < 1000
    # the product kernel (2048-position one-wave rounds in LayA / LayB, waves 1-7 retiring) on the same
    # vector: the same introselect, so the same median and MAD
    pm, pd = svo_amd.debug_robust_scale(v, n, impl=svo_amd.SCALE_K2V)
    assert (pm, pd) == (out[0], out[1]), ("product", pm, out[0], pd, out[1])
