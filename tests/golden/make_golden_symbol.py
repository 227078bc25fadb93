"""Generates tests/golden/symbol_jac.npz: the reference's own symbolic 2x6 image Jacobian
(python/symbol.py:50-60, `final = first * second`, derived with sympy) evaluated at seeded camera points.

Run here, where /root/reference exists (it does not travel to the GPU box):
    python3 tests/golden/make_golden_symbol.py
The reference script is executed as it stands (runpy; its pretty-printing goes to /dev/null) and its
`final` matrix is lambdified over (fx, fy, x, y, z, z2) with z2 = z * z.  The fixture holds only data:
the inputs and the 2x6 outputs."""
import contextlib
import io
import os
import runpy

import numpy as np
import sympy as sym

REF = "/root/reference/python/symbol.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "symbol_jac.npz")


def main():
    with contextlib.redirect_stdout(io.StringIO()):
        g = runpy.run_path(REF)
    final = g["final"]
    fx, fy, x, y, z, z2 = (g[k] for k in ("fx", "fy", "x", "y", "z", "z2"))
    f = sym.lambdify((fx, fy, x, y, z, z2), final, "numpy")
    rng = np.random.default_rng(20240)
    n = 64
    inp = np.stack([rng.uniform(300, 900, n), rng.uniform(300, 900, n), rng.uniform(-20, 20, n),
                    rng.uniform(-8, 8, n), rng.uniform(2, 80, n)], axis=1)
    inp[0] = [721.5377, 721.5377, 1.5, -0.75, 12.0]  # the KITTI focal length (resource/kitti.yaml)
    jac = np.stack([np.array(f(a, b, c, d, e, e * e), dtype=np.float64) for a, b, c, d, e in inp])
    np.savez(OUT, inputs=inp, jac=jac, source=np.array("python/symbol.py:50-60 final = first * second"))
    print(f"wrote {OUT}: {n} points")


if __name__ == "__main__":
    main()
