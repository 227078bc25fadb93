"""Where does a synchronous FeatureAlignment call (config 3, p 8) spend its time?  (development check; GPU)

Times svo_amd.FeatureAlignment.align_batch and the bare C-ABI call in a fresh context, then again after the
context ran a config-2 alignment batch (set_pairs + runs), as bench.py's `secondary` section does."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402


def timeit(fn, reps=50):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts)), 1e3 * float(np.min(ts))


def fa_calls(tag, ctx, scene, camera, cam):
    ps = svo_amd.PyramidSet(2, cam["width"], cam["height"], 1, ctx)
    ps.upload(0, np.stack([scene.ref_img, scene.cur_img]))
    ps.build()
    rng = np.random.default_rng(3)
    n = min(2000, len(scene.px))
    ref_px = np.ascontiguousarray(scene.px[:n])
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    fa = svo_amd.FeatureAlignment(8, ctx=ctx)

    def call():
        px = np.ascontiguousarray(init.copy())
        fa.align_batch(ps, 0, ps, 1, ref_px, px, camera)

    med, mn = timeit(call)
    print(f"{tag}: FeatureAlignment p8 n={n}: median {med:.4f} ms, min {mn:.4f} ms per call", flush=True)
    sync = timeit(ctx.synchronize)
    print(f"{tag}: ctx.synchronize alone: median {sync[0]:.4f} ms", flush=True)


def main():
    scene = synth.make_pair(seed=synth.SEED_BASE, n_features=2000, patch_size=5, nthreads=8, cell_order=30)
    cam = scene.camera
    camera = svo_amd.PinholeCamera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"])
    ctx = svo_amd.Context(0)
    fa_calls("fresh ctx", ctx, scene, camera, cam)
    if len(sys.argv) > 1 and sys.argv[1] == "fresh":
        return
    # the stages bench.py runs before `secondary`, one at a time
    import bench
    bench.svo_amd, bench.synth = svo_amd, synth
    P = 64
    ps = svo_amd.PyramidSet(3 * P, cam["width"], cam["height"], 5, ctx)
    ps.upload(0, np.stack([im for _ in range(P) for im in (scene.ref_img, scene.kf_img, scene.cur_img)]))
    ps.build()
    batch = svo_amd.AlignBatch(camera, 5, 0, 4, P, 2000, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    batch.set_pairs(0, ps, ps, ps, *bench.packed_pairs([scene], P, 1))
    batch.run()
    batch.results()
    ctx.synchronize()
    fa_calls("after set_pairs + run", ctx, scene, camera, cam)
    b2 = svo_amd.AlignBatch(camera, 5, 0, 4, P, 2000, ctx, median_mode=svo_amd.MEDIAN_EXACT)
    b2.set_pairs(0, ps, ps, ps, *bench.packed_pairs([scene], P, 1))
    b2.run()
    b2.results()
    b2.close()
    fa_calls("after exact batch + close", ctx, scene, camera, cam)
    L = 5
    for n in (64, 512):
        ps2 = svo_amd.PyramidSet(3 * n, cam["width"], cam["height"], L, ctx)
        ps2.upload(0, np.stack([im for _ in range(n) for im in (scene.ref_img, scene.kf_img, scene.cur_img)]))
        ps2.build()
        fa_calls(f"after PyramidSet({3 * n})", ctx, scene, camera, cam)
        b = svo_amd.AlignBatch(camera, 5, 0, L - 1, n, 2000, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
        fa_calls(f"after AlignBatch({n})", ctx, scene, camera, cam)
        b.set_pairs(0, ps2, ps2, ps2, *bench.packed_pairs([scene], n, 1))
        fa_calls(f"after set_pairs({n})", ctx, scene, camera, cam)
        b.run()
        b.results()
        fa_calls(f"after run({n})", ctx, scene, camera, cam)
    import gc
    b.close()
    fa_calls("after AlignBatch(512).close", ctx, scene, camera, cam)
    del b
    gc.collect()
    fa_calls("after del AlignBatch(512)", ctx, scene, camera, cam)
    del ps2
    gc.collect()
    fa_calls("after del PyramidSet(1536)", ctx, scene, camera, cam)

if __name__ == "__main__":
    main()
