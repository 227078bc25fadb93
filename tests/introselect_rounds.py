"""numpy restatement of libstdc++'s introselect as the parallel Hoare rounds K2V / K2R run (test infrastructure).

One round (tests/cpp/introselect_model.cpp round_pf, checked there against the real std::nth_element):
median of three of (first + 1, first + S/2, last - 1) moved to first, pivot p; GE = positions in (first, last) with
!(a < p) left to right (L_1 < L_2 < ...), LE = positions in [first, last) with !(p < a) right to left
(R_1 > R_2 > ...); L_k and R_k swap for k <= Ks = max over split points t of min(#GE before t, #LE from t on);
cut = min(L_{Ks+1}, R_{Ks}).  `rounds` yields every round's (first, last, pivot, Ks, #GE, #LE, cut) and the array
after it, so a device trace (svo_debug_robust_scale with its round trace) can be compared round for round.
"""
import math

import numpy as np

DBL_MAX = np.finfo(np.float64).max


def round_pf(a, first, last):
    S = last - first
    A, B, C = first + 1, first + S // 2, last - 1
    if a[A] < a[B]:
        ch = B if a[B] < a[C] else (C if a[A] < a[C] else A)
    else:
        ch = A if a[A] < a[C] else (C if a[B] < a[C] else B)
    a[first], a[ch] = a[ch], a[first]
    p = a[first]
    body = a[first + 1:last]
    isge = ~(body < p)
    isle = ~(p < body)
    ge = np.nonzero(isge)[0] + first + 1
    le = np.nonzero(~(p < a[first:last]))[0][::-1] + first
    G = np.concatenate([[0], np.cumsum(isge)])
    Lc = np.concatenate([np.cumsum(isle[::-1])[::-1], [0]])
    ks = int(np.max(np.minimum(G, Lc)))
    cut = int(ge[ks]) if len(ge) > ks else 1 << 40
    if ks > 0:
        cut = min(cut, int(le[ks - 1]))
    gi, li = ge[:ks].copy(), le[:ks].copy()
    t = a[gi].copy()
    a[gi] = a[li]
    a[li] = t
    return float(p), ks, len(ge), len(le), cut


def rounds(v, nth):
    """Every round of std::nth_element(v, v + nth) until the depth limit or <= 3 positions; yields
    (first, last, pivot, ks, n_ge, n_le, cut, array_after) and returns through StopIteration.value the final
    (first, last, array) (the heap-select path is not modelled: callers check that it was not needed)."""
    a = np.array(v, dtype=np.float64)
    first, last = 0, len(a)
    depth = 2 * int(math.floor(math.log2(len(a)))) if len(a) > 1 else 0
    while last - first > 3 and depth > 0:
        depth -= 1
        f0, l0 = first, last
        p, ks, ng, nl, cut = round_pf(a, first, last)
        if cut <= nth:
            first = cut
        else:
            last = cut
        yield f0, l0, p, ks, ng, nl, cut, a
    return first, last, a


def robust_scale(v, n_valid):
    """computeMedian / computeMAD of the reference (src/algorithm.cpp:834-865) through the round model:
    (median, mad, recorded vec[nth - 1] of each pass).  Only for inputs that end by the <= 3 rule."""
    out = []
    x = np.array(v, dtype=np.float64)
    for _ in range(2):
        nth = n_valid // 2
        gen = rounds(x, nth)
        lo = None
        try:
            while True:
                f0, l0, p, ks, ng, nl, cut, a = next(gen)
                if cut == nth and lo is None and nth >= 1:
                    lo = float(a[nth - 1])
        except StopIteration as e:
            first, last, a = e.value
        assert last - first <= 3, "depth limit reached: heap select not modelled"
        a[first:last] = np.sort(a[first:last])
        hi = float(a[nth])
        if lo is None:
            lo = float(a[nth - 1]) if nth >= 1 else 0.0
        r = (lo + hi) / 2.0 if len(x) % 2 == 0 and nth >= 1 else hi
        out.append(r)
        if len(out) == 1:
            med = r
            x = np.abs(np.array(v, dtype=np.float64) - med)
            x[np.array(v) >= DBL_MAX] = DBL_MAX
    return out[0], out[1]
