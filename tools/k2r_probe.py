"""K2R latency probe: svo_debug_robust_scale on a config-2-shaped residual vector (50 000 slots, 80 %
visible, sigma 8), with the kernel's clock stamps (SVO_DEBUG_STAMPS=1): cycles of round 1 and of the
remaining rounds per pass, and the number of global / LDS rounds."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SVO_DEBUG_STAMPS"] = sys.argv[1] if len(sys.argv) > 1 else "1"  # "2": phases of round 1 only
import svo_amd  # noqa: E402
from svo_amd import _capi  # noqa: E402

rng = np.random.default_rng(1)
v = rng.normal(0, 8, 50000)
v[np.repeat(rng.random(2000) < 0.2, 25)] = np.finfo(np.float64).max
n = int((v < 1e300).sum())
ctx = svo_amd.default_context()
out = np.zeros(218)
for _ in range(3):
    _capi.check(_capi.lib().svo_debug_robust_scale(ctx.handle, _capi.ptr(v), len(v), n, _capi.ptr(out)))
t0 = time.perf_counter()
for _ in range(20):
    _capi.check(_capi.lib().svo_debug_robust_scale(ctx.handle, _capi.ptr(v), len(v), n, _capi.ptr(out)))
dt = (time.perf_counter() - t0) / 20
print(f"med {out[0]!r} mad {out[1]!r}  call {dt * 1e6:.1f} us")
for p in range(2):
    r1, rest, nb, nw = out[2 + 4 * p: 6 + 4 * p]
    print(f"pass {p}: round1 {r1:.0f} cycles, rest {rest:.0f} cycles, block rounds {nb:.0f}, wave rounds {nw:.0f}")
names = ("pivot", "sweep", "crossing", "partners", "swaps/copy")
for w, kind in enumerate(("round 1", "global rounds", "lds rounds")):
    ph = out[10 + 5 * w: 15 + 5 * w]
    print(f"{kind:14s} cycles per phase (both passes): " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, ph)))
ph = out[25:30]
print("wave rounds    cycles per phase (both passes): " + ", ".join(f"{n} {v:.0f}" for n, v in zip(("pivot", "sweep", "crossing", "partners", "swaps"), ph)))
print(f"exact classifications: pass 0 {out[30]:.0f}, pass 1 {out[31]:.0f}")
wl = out[32:98].reshape(-1, 3)
print("wave rounds (steps, sweep cycles, round cycles):", [tuple(int(x) for x in r) for r in wl if r[0] >= 0])
bl = out[98:218].reshape(-1, 3)
print("block rounds (S, where 0 src 1 glb 2 lds, cycles):", [tuple(int(x) for x in r) for r in bl if r[0] >= 0])
