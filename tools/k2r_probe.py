"""K2R / K2V latency probe (argument: 1 K2R, 2 K2V): svo_debug_robust_scale on a config-2-shaped residual vector (50 000 slots, 80 %
visible, sigma 8) with the kernel's diagnostics (SVO_DEBUG_STAMPS=1): cycles per pass, block / one-wave round
counts, and per block round the segment size, where it lived (0 K1's array, 1 global scratch, 2 LDS) and its
cycles.  The result is checked against the oracle's std::nth_element."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ["SVO_DEBUG_STAMPS"] = "1"  # (K2R's phase stamps; K2V always reports its counters)
import svo_amd  # noqa: E402
from svo_amd import _capi  # noqa: E402
import oracle as O  # noqa: E402

DBL_MAX = np.finfo(np.float64).max
rng = np.random.default_rng(1)
NS = int(os.environ.get("SVO_PROBE_SLOTS", "50000"))  # (60000: K2V's larger register layout)
v = rng.normal(0, 8, NS)
v[np.repeat(rng.random(NS // 25) < 0.2, 25)] = DBL_MAX
n = int((v < 1e300).sum())
ctx = svo_amd.default_context()
impl = int(sys.argv[1]) if len(sys.argv) > 1 else svo_amd.SCALE_K2R
# SVO_PROBE_PLAIN=1: out_len 2, so K2V runs the product kernel (plain_robust_scale_v_kernel: product layouts, one-wave
# size 2048, wave retirement) instead of the diagnostics kernel; only the result and the call time are reported, the
# kernel's own duration comes from a kernel trace of this run.
plain = bool(os.environ.get("SVO_PROBE_PLAIN"))
out = np.zeros(2 if plain else 206)
for _ in range(3):
    _capi.check(_capi.lib().svo_debug_robust_scale(ctx.handle, _capi.ptr(v), len(v), n, impl, _capi.ptr(out), len(out)))
t0 = time.perf_counter()
for _ in range(20):
    _capi.check(_capi.lib().svo_debug_robust_scale(ctx.handle, _capi.ptr(v), len(v), n, impl, _capi.ptr(out), len(out)))
dt = (time.perf_counter() - t0) / 20
med_c = O.median(v, n, 0)
d = np.abs(v - med_c)
d[v >= DBL_MAX] = DBL_MAX
mad_c = O.median(d, n, 0)
match = out[0] == med_c and out[1] == mad_c
print(f"med {out[0]!r} mad {out[1]!r}  oracle {med_c!r} {mad_c!r}  match {match}  call {dt * 1e6:.1f} us"
      + ("  (product kernel)" if plain else ""))
if plain:
    sys.exit(0 if match else 3)
if impl == svo_amd.SCALE_K2V:
    for p in range(2):
        cyc, nb, nl, hp, ch = out[2 + 5 * p: 7 + 5 * p]
        print(f"K2V pass {p}: {cyc:.0f} cycles, block rounds {nb:.0f}, one-wave rounds {nl:.0f}, heap select {hp:.0f}, "
              f"chunked exchanges {ch:.0f}")
    names = ("load", "classify", "barrier1", "publish+ranks", "sources", "barrier2", "targets", "exits", "scan",
             "crossing", "searches")
    print("K2V cycles per phase (thread 0, both passes): " + ", ".join(f"{a} {x:.0f}" for a, x in zip(names, out[12:23])))
    if os.environ.get("SVO_PROBE_WAVES"):  # (make stamps STAMPS_WAVES=1: every wave's cycles per phase)
        pw = out[24:24 + 96].reshape(8, 12)
        print("K2V cycles per phase and wave (both passes; rows: waves 0-7):")
        print("      " + " ".join(f"{a[:9]:>9}" for a in names))
        for w in range(8):
            print(f"  w{w}  " + " ".join(f"{x:9.0f}" for x in pw[w, :11]))
    else:
        log = out[24:152].reshape(-1, 2)
        print("K2V block rounds (S, cycles; stamps build):", [tuple(int(x) for x in r) for r in log if r[0] >= 0])
    sys.exit(0 if match else 3)
for p in range(2):
    cyc, nb, nl, hp = out[2 + 4 * p: 6 + 4 * p]
    print(f"pass {p}: {cyc:.0f} cycles, block rounds {nb:.0f}, one-wave rounds {nl:.0f}, heap select {hp:.0f}")
bl = out[10:190].reshape(-1, 3)
print("block rounds (S, where, cycles):", [tuple(int(x) for x in r) for r in bl if r[0] >= 0])
names = ("sweep", "barrier1", "scan+search", "mailbox", "barrier2", "targets", "barrier3", "pivot")
for w, kind in enumerate(("global", "LDS")):
    print(f"{kind:6s} rounds, cycles per phase (thread 0, both passes): " + ", ".join(f"{n} {x:.0f}" for n, x in zip(names, out[190 + 8 * w: 198 + 8 * w])))
sys.exit(0 if match else 3)
