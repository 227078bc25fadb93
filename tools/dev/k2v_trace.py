"""K2V round trace against a numpy model of the parallel Hoare rounds (development; GPU).

Runs svo_debug_robust_scale (K2V) on the probe's vector with the round trace on (out_len > 206) and replays every
round on the host (tests/cpp/introselect_model.cpp's round_pf, vectorised); prints the first round whose header
(segment, pivot, Ks, counts, cut) or kept segment differs, with the differing positions' row / wave / lane.
usage: python3 tools/dev/k2v_trace.py [n_slots=50000] [seed=1]
"""
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import svo_amd  # noqa: E402
from svo_amd import _capi  # noqa: E402

DBL_MAX = np.finfo(np.float64).max
HEAD = 8


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
    le_all = np.nonzero(~(p < a[first:last]))[0][::-1] + first
    G = np.concatenate([[0], np.cumsum(isge)])
    Lc = np.concatenate([np.cumsum(isle[::-1])[::-1], [0]])
    ks = int(np.max(np.minimum(G, Lc)))
    cut = ge[ks] if len(ge) > ks else 1 << 40
    if ks > 0:
        cut = min(cut, le_all[ks - 1])
    gi, li = ge[:ks].copy(), le_all[:ks].copy()
    t = a[gi].copy()
    a[gi] = a[li]
    a[li] = t
    return p, ks, len(ge), len(le_all), int(cut)


def where(q):
    return f"q={q} row={q // 512} wave={(q // 64) % 8} lane={q % 64}"


def main():
    NS = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rng = np.random.default_rng(seed)
    v = rng.normal(0, 8, NS)
    v[np.repeat(rng.random(NS // 25) < 0.2, 25)] = DBL_MAX
    n = int((v < 1e300).sum())
    ctx = svo_amd.default_context()
    nrec = 80
    out = np.zeros(206 + nrec * (HEAD + NS))
    _capi.check(_capi.lib().svo_debug_robust_scale(ctx.handle, _capi.ptr(v), NS, n, svo_amd.SCALE_K2V, _capi.ptr(out),
                                                   len(out)))
    recs = out[206:].reshape(nrec, HEAD + NS)
    print(f"device med {out[0]!r} mad {out[1]!r}")
    nth = n // 2
    a = v.copy()
    med = None
    ri = 0
    for P in range(2):
        if P == 1:
            a = np.abs(v - med)
            a[v >= DBL_MAX] = DBL_MAX
        first, last = 0, NS
        depth = 2 * int(math.floor(math.log2(NS)))
        while last - first > 3 and depth > 0:
            depth -= 1
            f0, l0 = first, last
            p, ks, tg, tl, cut = round_pf(a, first, last)
            if cut <= nth:
                first = cut
            else:
                last = cut
            h = recs[ri, :HEAD]
            kind = int(h[0]) // 10
            got = dict(P=int(h[0]) % 10, f=int(h[1]), l=int(h[2]), p=h[3], ks=int(h[4]), tg=int(h[5]), tl=int(h[6]),
                       cut=int(h[7]))
            exp = dict(P=P, f=f0, l=l0, p=p, ks=ks, tg=tg - 0, tl=tl, cut=cut)
            vec = recs[ri, HEAD:]
            if kind == 1:  # one-wave record: only the 512 slots of the one-wave segment were written
                lo, hi = first, last
            else:
                lo, hi = first, last
            dif = np.nonzero(vec[lo:hi] != a[lo:hi])[0] + lo
            bad = [k for k in exp if (exp[k] != got[k])]
            tag = "block" if kind == 0 else "wave"
            print(f"round {ri} pass {P} {tag}: f {f0} l {l0} S {l0 - f0} ks {ks} cut {cut}"
                  f"{'  HEADER ' + str({k: (got[k], exp[k]) for k in bad}) if bad else ''}"
                  f"{'  kept-segment diffs ' + str(len(dif)) if len(dif) else ''}")
            if bad or len(dif):
                same_multiset = np.array_equal(np.sort(vec[lo:hi]), np.sort(a[lo:hi]))
                print(f"  kept segment [{lo}, {hi}) same multiset: {same_multiset}")
                for q in dif[:12]:
                    print(f"  {where(int(q))}: device {vec[q]!r} model {a[q]!r}")
                if len(dif):
                    rows = np.unique(dif // 512)
                    waves = np.unique((dif // 64) % 8)
                    print(f"  rows {rows[:40].tolist()} waves {waves.tolist()}")
                return 3
            ri += 1
        if last - first <= 3:
            a[first:last] = np.sort(a[first:last])
        hi_v = a[nth]
        lo_v = a[nth - 1]
        r = (lo_v + hi_v) / 2 if NS % 2 == 0 else hi_v
        if P == 0:
            med = r
            print(f"model med {med!r}")
        else:
            print(f"model mad {r!r}")
    print("all rounds match")
    return 0


if __name__ == "__main__":
    sys.exit(main())
