"""BASELINE config 4 (512 synthetic frame pairs, independent, sharded over GPUs with no collective) and the
robust-scale kernel choice.

* the headline batch shape: one 512-pair reference-mode batch (four 128-pair K2V chains) over 16 distinct scenes,
  every pair against the oracle's std::nth_element path and bit for bit against a single-pair run of its scene;
* config 4 as SURVEY 8(d) defines it: 512 pairs on 512 distinct scenes (seeds 0x5EED0000 + pair), every pair against
  the oracle;
* the N > 1 rank path on the GPU: bench.py --gpus 2 (both ranks on device 0, SVO_BENCH_SHARED_GPU=1) dumps every
  pair's pose; a --gpus 1 run over the same 2 x P pairs (--scene-block P) must give the same bits (SURVEY §8(e):
  per-pair outputs independent of the number of ranks);
* the kernel follows each frame's own residual vector (src/image_alignment.cpp:30-38 sizes it per frame), not the
  grow-only capacity: 2000 -> 2400 -> 2000-feature frames through svo_amd.ImageAlignment, the trace field
  scale_kernel read at every level;
* K2R's 8-wave batch instantiations in whole alignments (vectors past K2V's capacity, chains of > 128 pairs).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import svo_amd
import svo_amd.synth as synth
from common import canon, oracle_align

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCH, L = 5, 5


def _bench_mod():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.synth = synth
    return m


def test_scene_seeds_independent_of_ranks():
    """CPU: with --scene-block B the job's pair -> scene map is the same for any number of ranks."""
    b = _bench_mod()
    P, D = 256, 8
    one = b.scene_seeds(0, 2 * P, P, D)
    two = b.scene_seeds(0, P, P, D) + b.scene_seeds(P, P, P, D)
    assert one == two
    assert len(set(one)) == 2 * D and one[:D] == [synth.SEED_BASE + i for i in range(D)]
    # the default block (--pairs) is the earlier per-rank mapping: rank r's scenes seeded SEED_BASE + first + i % D
    assert b.scene_seeds(512, 512, 512, 16)[:20] == [synth.SEED_BASE + 512 + i % 16 for i in range(20)]


def _camera(s):
    c = s.camera
    return svo_amd.PinholeCamera(c["width"], c["height"], c["fx"], c["fy"], c["cx"], c["cy"])


def _packed(sc, pairs):
    d = len(sc)
    frames = np.array([[3 * (i % d), 3 * (i % d) + 1, 3 * (i % d) + 2] for i in pairs], np.int32)
    poses = np.stack([np.concatenate([sc[i % d].ref_pose, sc[i % d].kf_pose, sc[i % d].cur_init_pose]) for i in pairs])
    n_feat = np.array([[sc[i % d].n_ref, sc[i % d].n_kf] for i in pairs], np.int32)
    cat = lambda f: np.concatenate([getattr(sc[i % d], f) for i in pairs])
    return frames, poses, n_feat, cat("px"), cat("bearing"), cat("point"), cat("has_point")


def _pyramids(sc, ctx):
    c = sc[0].camera
    ps = svo_amd.PyramidSet(3 * len(sc), c["width"], c["height"], L, ctx)
    ps.upload(0, np.stack([im for s in sc for im in (s.ref_img, s.kf_img, s.cur_img)]))
    ps.build()
    return ps


def _single(ps, d, s, cam, ctx, nf):
    b1 = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, 1, nf, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    b1.set_pair(0, (ps, 3 * d), (ps, 3 * d + 1), (ps, 3 * d + 2), s.ref_pose, s.kf_pose, s.cur_init_pose,
                s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
    b1.run()
    r = b1.results()
    tr = [b1.traces(0)[l].scale_kernel for l in range(L)]
    b1.close()
    return r, tr


@pytest.mark.gpu
def test_gpu_config4_batch_512_pairs():
    ctx = svo_amd.default_context()
    D, P, NF = 16, 512, 2000
    sc = [synth.make_pair(seed=synth.SEED_BASE + 700 + i, n_features=NF, patch_size=PATCH) for i in range(D)]
    ps = _pyramids(sc, ctx)
    cam = _camera(sc[0])
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    b.set_pairs(0, ps, ps, ps, *_packed(sc, range(P)))
    b.run()
    poses, err, st = b.results()
    for i in (0, 127, 128, 255, 256, 383, 384, 511):  # every 128-pair chain (capi.hip kSplitsRefv) ran K2V at every level
        assert [b.traces(i)[l].scale_kernel for l in range(L)] == [svo_amd.SCALE_K2V] * L, i
    ref = [oracle_align(s, PATCH, 0, L - 1, mode=0, trace=False) for s in sc]
    for i in range(P):
        pc, ec, stc = ref[i % D][:3]
        assert st[i] == stc, i
        assert np.abs(canon(poses[i]) - canon(pc)).max() <= 1e-9, i
        assert abs(err[i] - ec) <= 1e-9 * max(ec, 1e-300), i
    for d in range(D):
        (p1, e1, s1), _ = _single(ps, d, sc[d], cam, ctx, NF)
        for i in range(d, P, D):
            assert np.array_equal(p1[0], poses[i]) and e1[0] == err[i] and s1[0] == st[i], (d, i)
    b.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_config4_512_distinct_scenes():
    """SURVEY 8(d) config 4 as defined: 512 pairs, pair p on the scene seeded 0x5EED0000 + p (no repeated scene), in
    the bench's detector cell order; every pair against the oracle's std::nth_element path.  The
    scenes and the oracle run on a host thread pool (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    ctx = svo_amd.default_context()
    P, NF = 512, 2000
    workers = max(1, min(16, os.cpu_count() or 1))
    with ThreadPoolExecutor(workers) as ex:
        sc = list(ex.map(lambda p: synth.make_pair(seed=synth.SEED_BASE + p, n_features=NF, patch_size=PATCH, nthreads=1,
                                                   cell_order=30), range(P)))
    print(f"512 scenes generated on {workers} threads", flush=True)
    ps = _pyramids(sc, ctx)
    cam = _camera(sc[0])
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, NF, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    b.set_pairs(0, ps, ps, ps, *_packed(sc, range(P)))
    b.run()
    poses, err, st = b.results()
    for i in (0, 127, 128, 255, 256, 383, 384, 511):
        assert [b.traces(i)[l].scale_kernel for l in range(L)] == [svo_amd.SCALE_K2V] * L, i
    b.run()  # a second run of the same batch: the same bits
    p2, e2, s2 = b.results()
    assert np.array_equal(p2, poses) and np.array_equal(e2, err) and np.array_equal(s2, st)
    b.close()
    with ThreadPoolExecutor(workers) as ex:
        ref = list(ex.map(lambda s: oracle_align(s, PATCH, 0, L - 1, mode=0, trace=False)[:3], sc))
    for i in range(P):
        pc, ec, stc = ref[i]
        assert st[i] == stc, i
        assert np.abs(canon(poses[i]) - canon(pc)).max() <= 1e-9, i
        assert abs(err[i] - ec) <= 1e-9 * max(ec, 1e-300), i


def _run_bench(args, out, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--dump-poses", out],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return np.load(out)


@pytest.mark.gpu
def test_gpu_two_ranks_match_one_rank(tmp_path):
    P, D = 256, 8
    common = ["--steps", "2", "--warmup", "1", "--distinct", str(D), "--no-cpu", "--no-secondary", "--core-only"]
    two = _run_bench(["--gpus", "2", "--pairs", str(P), *common], str(tmp_path / "g2.npz"),
                     {"SVO_BENCH_SHARED_GPU": "1"})
    one = _run_bench(["--gpus", "1", "--pairs", str(2 * P), "--scene-block", str(P), *common], str(tmp_path / "g1.npz"),
                     {})
    assert int(two["world"]) == 2 and int(one["world"]) == 1
    assert np.array_equal(two["seeds"], one["seeds"]) and len(one["seeds"]) == 2 * P
    assert len(set(one["seeds"].tolist())) == 2 * D  # the two ranks' blocks hold different scenes
    assert np.array_equal(two["poses"], one["poses"])
    assert np.array_equal(two["err"], one["err"]) and np.array_equal(two["status"], one["status"])
    # and the poses are the oracle's (one pair of each scene)
    for k, g in enumerate(sorted(set(one["seeds"].tolist()))):
        i = int(np.flatnonzero(one["seeds"] == g)[0])
        s = synth.make_pair(seed=g, n_features=2000, patch_size=PATCH, cell_order=30)
        pc, ec, stc = oracle_align(s, PATCH, 0, L - 1, mode=0, trace=False)[:3]
        assert one["status"][i] == stc and np.abs(canon(one["poses"][i]) - canon(pc)).max() <= 1e-9, (k, g)


def _class_frames(s, ctx):
    cam = svo_amd.PinholeCamera.kitti()
    kf = svo_amd.Frame(cam, s.kf_img, L, ctx=ctx)
    kf.abs_pose[:] = s.kf_pose
    ref = svo_amd.Frame(cam, s.ref_img, L, last_keyframe=kf, ctx=ctx)
    ref.abs_pose[:] = s.ref_pose
    cur = svo_amd.Frame(cam, s.cur_img, L, last_keyframe=kf, ctx=ctx)
    cur.abs_pose[:] = s.cur_init_pose
    for i in range(len(s.px)):
        fr = ref if i < s.n_ref else kf
        fr.add_feature(svo_amd.Feature(fr, s.px[i], bearing=s.bearing[i], point=svo_amd.Point(s.point[i])))
    return ref, cur


@pytest.mark.gpu
def test_gpu_scale_kernel_follows_the_frame():
    ctx = svo_amd.default_context()
    cap = svo_amd.robust_scale_capacity(svo_amd.SCALE_K2V)
    assert cap == svo_amd.SCALE_K2V_MAX_SLOTS
    ia = svo_amd.ImageAlignment(PATCH, 0, L - 1, ctx=ctx)
    scenes = {nf: synth.make_pair(seed=synth.SEED_BASE + 900 + nf, n_features=nf, patch_size=PATCH)
              for nf in (2000, 2400, 2600, 2621)}
    # 2000 -> LayA, 2400 -> LayB, 2600 (65 000 slots) and 2621 (65 525) -> LayC: K2V at every level
    for nf in (2000, 2400, 2600, 2621, 2000):
        s = scenes[nf]
        ref, cur = _class_frames(s, ctx)
        err = ia.align(ref, cur)
        pc, ec, stc, _ = oracle_align(s, PATCH, 0, L - 1, mode=0)
        assert ia.last_status == stc, nf
        assert np.abs(canon(cur.abs_pose) - canon(pc)).max() <= 1e-9, nf
        assert abs(err - ec) <= 1e-9 * ec, nf
        want = svo_amd.SCALE_K2V if nf * PATCH * PATCH <= cap else svo_amd.SCALE_K2R
        assert [t.scale_kernel for t in ia.last_traces] == [want] * L, (nf, cap)
        for fr in (ref, ref.last_keyframe, cur):
            fr.image_pyramid.clear()


@pytest.mark.gpu
@pytest.mark.parametrize("nf", ["above_k2v", 2700])
def test_gpu_k2r_wide_batch_instantiations(nf):
    """Chains of 132 pairs (> 128: the 8-wave, two-per-CU K2R instantiations) whose vectors exceed K2V's
    registers: just above K2V's capacity, and 2700 features (67 500 slots: the 17-block segment variant)."""
    ctx = svo_amd.default_context()
    cap = svo_amd.robust_scale_capacity(svo_amd.SCALE_K2V)
    if nf == "above_k2v":
        nf = cap // (PATCH * PATCH) + 40
    D, P = 4, 264
    sc = [synth.make_pair(seed=synth.SEED_BASE + 1100 + i, n_features=nf, patch_size=PATCH) for i in range(D)]
    ps = _pyramids(sc, ctx)
    cam = _camera(sc[0])
    b = svo_amd.AlignBatch(cam, PATCH, 0, L - 1, P, nf, ctx, median_mode=svo_amd.MEDIAN_REFERENCE)
    b.set_pairs(0, ps, ps, ps, *_packed(sc, range(P)))
    b.run()
    poses, err, st = b.results()
    for i in (0, 131, 132, 263):
        assert [b.traces(i)[l].scale_kernel for l in range(L)] == [svo_amd.SCALE_K2R] * L, i
    ref = [oracle_align(s, PATCH, 0, L - 1, mode=0, trace=False) for s in sc]
    for i in range(P):
        pc, ec, stc = ref[i % D][:3]
        assert st[i] == stc, i
        assert np.abs(canon(poses[i]) - canon(pc)).max() <= 1e-9, i
        assert np.array_equal(poses[i], poses[i % D]) and err[i] == err[i % D], i
    b.close()
