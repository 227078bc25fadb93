# quick GPU sanity run (not a test module): python tests/gpu_smoke.py
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
from common import make_pairs, gpu_batch, oracle_align, canon
pairs = make_pairs(2)
b, ps = gpu_batch(pairs, 5, 0, 4)
b.run(); p, e, st = b.results()
for i, s in enumerate(pairs):
    pc, ec, stc, trc = oracle_align(s, 5, 0, 4, mode=1)
    tg = b.traces(i)
    for l in range(4, -1, -1):
        print(l, tg[l].n_ref_vis, trc[l].n_ref_vis, tg[l].n_vis, trc[l].n_vis, tg[l].median, trc[l].median, tg[l].sigma, trc[l].sigma)
    print("pose diff", np.abs(canon(p[i]) - canon(pc)).max(), "err", e[i], ec, st[i], stc)
