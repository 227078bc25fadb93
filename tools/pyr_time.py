"""Pyramid build timing (diagnostic): 1536 KITTI-shaped frames (bench.py's pyramid_build), median of 9 builds after a
warm-up, hipEvents on the context stream, and the bytes against the oracle for two frames.
    python3 tools/pyr_time.py            (SVO_PYR=0: the round-4 kernels)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402
import oracle as O  # noqa: E402

N, L = 1536, 5
ctx = svo_amd.default_context()
sc = [synth.make_pair(seed=synth.SEED_BASE + i) for i in range(4)]
imgs = np.stack([im for s in sc for im in (s.ref_img, s.kf_img, s.cur_img)])
W, H = imgs.shape[2], imgs.shape[1]
ps = svo_amd.PyramidSet(N, W, H, L, ctx)
for f in range(0, N, len(imgs)):
    ps.upload(f, imgs[:min(len(imgs), N - f)])
ps.build()
runs = []
for _ in range(9):
    ctx.record(2)
    ps.build()
    ctx.record(3)
    runs.append(ctx.elapsed_ms(2, 3))
ms = float(np.median(runs))
sizes, w, h = [], W, H
for _ in range(L):
    sizes.append(w * h)
    w, h = (w + 1) // 2, (h + 1) // 2
alg = 2 * W * H + 2 * sum(sizes[1:])
ok = True
for f in (0, N - 1):
    oi, og = O.build_pyramid(imgs[f % len(imgs)], L)
    li, lg = O.unpack_levels(oi, W, H, L), O.unpack_levels(og, W, H, L)
    for l in range(L):
        ok &= np.array_equal(ps.download(f, l, False), li[l]) and np.array_equal(ps.download(f, l, True), lg[l])
print(f"pyramid build SVO_PYR={os.environ.get('SVO_PYR', '1')}: {ms:.4f} ms for {N} frames (runs {min(runs):.4f}.."
      f"{max(runs):.4f}), {N * alg / (ms * 1e-3) / 1e9:.1f} GB/s algorithmic = {N * alg / (ms * 1e-3) / 8e12:.4f} of "
      f"8 TB/s, bytes equal to the oracle: {ok}")
sys.exit(0 if ok else 3)
