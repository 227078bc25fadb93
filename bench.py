#!/usr/bin/env python3
"""bench.py — frame-pair alignments/sec of the MI355X ImageAlignment path (BASELINE.json metric).

Workload (BASELINE.json configs[1] = SURVEY.md §8(d) config 2): sparse image alignment of KITTI-shaped
frame pairs, 1241x376 grey, 2000 features (1000 on the ref frame + 1000 on its last keyframe), patch 5,
5-level pyramid (levels 4..0), one Tukey-weighted LM step per level.  A "step" is one pass of the hot
path over one batch: --pairs independent pairs per GPU (default 512), inputs (pyramids, features,
poses) resident in HBM before the timed region.  Data: synthetic street scenes (svo_amd.synth, seeds
0x5EED0000 + global pair index, SURVEY.md §8(d): every pair its own scene; --distinct D repeats D scenes instead),
each pair in its own HBM buffers.  The line also times the round 1-5 workload (16 scenes repeated) on the same batch
(`workload_16_distinct_scenes`).

Multi-GPU: one process per GPU; pairs are independent, so each rank aligns its own --pairs (weak
scaling) and there is no data-path collective: the gloo process group is used only for the barrier and
the max-over-ranks time.  Under torch.distributed.run the ranks come from RANK / LOCAL_RANK / WORLD_SIZE
(which must equal --gpus); `python bench.py --gpus N` without them starts the N ranks itself (child
processes on 127.0.0.1, before anything touches the GPU) and exits with their status.  --cpu-rehearsal
runs the same launcher / barrier / max-over-ranks path with the CPU oracle as the step (tests only).

Prints one JSON line (rank 0).  See DESIGN.md §Measurement for the roofline and baseline definitions.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

svo_amd = shard = synth = None  # imported in main() once this process is known to be a rank (see spawn_ranks)

METRIC = "frame-pair alignments/sec @2000 feats, 5-lvl pyramid; SE(3) err vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_VALU_PEAK_TFS = 78.6  # MI355X spec fp64 vector (half the 157.3 TF FP32 vector rate of MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=512, help="frame pairs per GPU per step")
    ap.add_argument("--features", type=int, default=2000)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--patch", type=int, default=5)
    ap.add_argument("--distinct", type=int, default=0,
                    help="distinct synthetic scenes per scene block (0: every pair its own scene, SURVEY 8(d))")
    ap.add_argument("--scene-block", type=int, default=0,
                    help="global pair g uses the scene seeded SEED_BASE + (g // B) * B + (g % B) %% distinct, B = this "
                         "value (default: --pairs, i.e. each rank's own block): the job's pairs are then the same "
                         "whatever the number of ranks, e.g. --gpus 2 --pairs P and --gpus 1 --pairs 2P --scene-block P")
    ap.add_argument("--dump-poses", default="",
                    help="rank 0 writes every rank's per-pair seeds, poses, errors and statuses (gathered in rank order) "
                         "to this .npz (G-invariance tests)")
    ap.add_argument("--feature-order", choices=("cell", "shuffled"), default="cell",
                    help="cell: features in the order the reference detector emits them (30-px grid cells row by "
                         "row, src/feature_selection.cpp:103-141); shuffled: random order")
    ap.add_argument("--median", choices=("reference", "exact"), default="reference",
                    help="robust-scale semantics: reference = the reference's libstdc++ nth_element post-state "
                         "(median_mode SVO_MEDIAN_REFERENCE: K2V, the vector in registers; K2R past its capacity); "
                         "exact = true order statistics (K2)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the config 3 / config 5 lines")
    ap.add_argument("--core-only", action="store_true",
                    help="only the timed chain steps (no end-to-end, other-mode or latency runs): PMC passes, whose "
                         "per-launch bytes assume every align dispatch belongs to the P-pair chain")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="no GPU: each rank's step is the CPU oracle on its pairs (exercises the multi-rank path)")
    ap.add_argument("--kernel-stats", default=os.path.join(ROOT, "profiles", "headline_kernel_stats.csv"),
                    help="tools/headline_kernel_stats.py output of a headline-only kernel trace (roofline.dominant_kernel)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="rocprofv3 PMC traffic summary of this workload (tools/pmc_traffic.py output)")
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def level_bytes(w, h, levels):
    tot = 0
    for _ in range(levels):
        tot += w * h
        w, h = (w + 1) // 2, (h + 1) // 2
    return tot


def packed_pairs(scenes, P, D, idx=None):
    """svo_align_batch_set_pairs inputs for pairs 0..P-1 (pair i = scene idx[i], default i % D; frames 3i .. 3i+2)."""
    idx = [i % D for i in range(P)] if idx is None else idx
    frames = np.arange(3 * P, dtype=np.int32).reshape(P, 3)
    poses = np.stack([np.concatenate([scenes[idx[i]].ref_pose, scenes[idx[i]].kf_pose, scenes[idx[i]].cur_init_pose])
                      for i in range(P)])
    n_feat = np.array([[scenes[idx[i]].n_ref, scenes[idx[i]].n_kf] for i in range(P)], np.int32)
    cat = lambda f: np.ascontiguousarray(np.concatenate([getattr(scenes[idx[i]], f) for i in range(P)]))
    return frames, poses, n_feat, cat("px"), cat("bearing"), cat("point"), cat("has_point").astype(np.uint8)


def scene_seeds(first, count, block, distinct):
    """Seed of each global pair g in [first, first + count): SEED_BASE + (g // block) * block + (g % block) % distinct."""
    return [synth.SEED_BASE + (g // block) * block + (g % block) % distinct for g in range(first, first + count)]


def image_chunks(scenes, idx, chunk):
    """Base images of pairs [c, c + chunk) as (first pair, (3 * count, H, W) array) per chunk; chunks with the same
    scenes share one array (the default mapping repeats every `distinct` pairs, so there is one)."""
    out, cache = [], {}
    for c in range(0, len(idx), chunk):
        key = tuple(idx[c:c + chunk])
        if key not in cache:
            cache[key] = np.stack([im for k in key for im in (scenes[k].ref_img, scenes[k].kf_img, scenes[k].cur_img)])
        out.append((c, cache[key]))
    return out


def canon(p):
    p = np.array(p, dtype=np.float64)
    if p[3] < 0:
        p[:4] = -p[:4]
    return p


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """Start n ranks of this script as child processes (one per GPU) and wait for all of them; the parent
    never touches the GPU.  Returns the worst exit status."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # the launcher parent never loads the HIP library
    global svo_amd, shard, synth
    import svo_amd  # noqa: E402  (loads libsvo_hip.so before torch can bring its own HIP runtime)
    import svo_amd.shard as shard  # noqa: E402
    import svo_amd.synth as synth  # noqa: E402
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: E402  (gloo: host-side barrier / max only)
        dist.init_process_group(backend="gloo")
    if args.cpu_rehearsal:
        return rehearsal(args, rank, world, dist)

    # SVO_BENCH_SHARED_GPU=1: every rank on device 0 (a rehearsal of the N > 1 path on a one-GPU box; the
    # line then says so and its value is not a scaling number)
    shared_gpu = os.environ.get("SVO_BENCH_SHARED_GPU") == "1"
    ctx = svo_amd.Context(0 if shared_gpu else local_rank)
    P, nf, L, patch = args.pairs, args.features, args.levels, args.patch
    D = P if args.distinct <= 0 else max(1, min(args.distinct, P))
    nthreads = max(1, min(16, os.cpu_count() or 1))
    first, _ = shard.pair_block(world * P, rank, world)  # this rank's block of the job's world * P pairs
    cell = 30 if args.feature_order == "cell" else 0  # config "cell_pixel_size": 30
    seeds = scene_seeds(first, P, args.scene_block or P, D)
    useeds = sorted(set(seeds))
    sidx = [useeds.index(s) for s in seeds]  # pair j -> its scene in `scenes`
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(nthreads) as ex:  # (ctypes releases the GIL: one scene per host thread)
        scenes = list(ex.map(lambda sd: synth.make_pair(seed=sd, n_features=nf, patch_size=patch, nthreads=1,
                                                         cell_order=cell), useeds))
    cam = scenes[0].camera
    camera = svo_amd.PinholeCamera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"])
    rep = [sidx.index(k) for k in range(len(scenes))]  # the first pair of each scene

    # device-resident inputs: 3 pyramids per pair, each pair in its own buffers
    ps = svo_amd.PyramidSet(3 * P, cam["width"], cam["height"], L, ctx)
    chunks = image_chunks(scenes, sidx, D)
    for c, arr in chunks:
        ps.upload(3 * c, arr)
    ctx.synchronize()
    ps.build()  # warm-up (the first launch loads the code objects)
    pyr_runs = []
    for _ in range(5):  # median of 5 builds of all 3P frames (the build is idempotent: level 0 stays)
        ctx.record(2)
        ps.build()
        ctx.record(3)
        pyr_runs.append(ctx.elapsed_ms(2, 3))
    pyr_ms = float(np.median(pyr_runs))
    pyr_bytes = 2 * cam["width"] * cam["height"] + 2 * (level_bytes(cam["width"], cam["height"], L)
                                                       - cam["width"] * cam["height"])

    mode = svo_amd.MEDIAN_REFERENCE if args.median == "reference" else svo_amd.MEDIAN_EXACT
    batch = svo_amd.AlignBatch(camera, patch, 0, L - 1, P, nf, ctx, median_mode=mode)
    packed = packed_pairs(scenes, P, D, sidx)  # the caller's feature arrays (built outside every timed region)
    batch.set_pairs(0, ps, ps, ps, *packed)

    for _ in range(args.warmup):
        batch.run()
    ctx.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ctx.record(0)
    for _ in range(args.steps):
        batch.run()
    ctx.record(1)
    ctx.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    kernel_ms = ctx.elapsed_ms(0, 1) / args.steps
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    poses, err, status = batch.results()
    # every pair repeats its scene's pose bit for bit (the pairs of one scene run in different sub-batch chains)
    poses_repeat = bool(all(np.array_equal(poses[i], poses[rep[sidx[i]]]) and err[i] == err[rep[sidx[i]]]
                            for i in range(P)))
    if args.dump_poses:  # every rank's per-pair results, gathered in rank order (host side, outside the timing)
        mine = (np.array(seeds, np.int64), poses, err, status)
        parts = [mine]
        if dist:
            parts = [None] * world
            dist.all_gather_object(parts, mine)
        if rank == 0:
            np.savez(args.dump_poses, seeds=np.concatenate([q[0] for q in parts]),
                     poses=np.concatenate([q[1] for q in parts]), err=np.concatenate([q[2] for q in parts]),
                     status=np.concatenate([q[3] for q in parts]), world=world)
    # per-step time: median of 20 single synchronized steps (host clock), after the timed region
    step_s = []
    for _ in range(20):
        ctx.synchronize()
        t = time.perf_counter()
        batch.run()
        ctx.synchronize()
        step_s.append(time.perf_counter() - t)
    step_med = float(np.median(step_s))
    stages = batch.profile()  # one extra, event-instrumented run (outside the timed region)
    # the round 1-5 headline workload on the same batch and pyramids: pair i on scene i % 16 (SEED_BASE + i % 16, the
    # first 16 scenes of this set when every pair has its own scene); timed like the headline; not `value`
    w16 = None
    if D == P and P >= 16 and args.scene_block in (0, P):
        idx16 = [i % 16 for i in range(P)]
        pk16 = list(packed_pairs(scenes, P, 16, [sidx[k] for k in idx16]))
        pk16[0] = np.array([[3 * k, 3 * k + 1, 3 * k + 2] for k in idx16], np.int32)  # frames of scene i % 16
        batch.set_pairs(0, ps, ps, ps, *pk16)
        for _ in range(2):
            batch.run()
        ctx.synchronize()
        t16 = time.perf_counter()
        for _ in range(args.steps):
            batch.run()
        ctx.synchronize()
        dt16 = (time.perf_counter() - t16) / args.steps
        p16, _, _ = batch.results()
        w16 = {"pairs_per_s": round(P / dt16, 1), "ms_per_step": round(dt16 * 1e3, 4), "distinct_scenes": 16,
               "poses_equal_their_scene": bool(all(np.array_equal(p16[i], poses[i % 16]) for i in range(P))),
               "note": "rounds 1-5 headline workload: pair i on scene SEED_BASE + i % 16 (each scene 32 times); "
                       "same batch, pyramids and timing as the headline"}
        batch.set_pairs(0, ps, ps, ps, *packed)  # (back on the headline's pairs)
    # end to end from host memory (outside the timed region; never `value`): upload the 3P base images,
    # build the pyramids, hand over every pair's features and poses, align, read the results back
    ctx.synchronize()
    e2e_t0 = time.perf_counter()
    for c, arr in chunks:
        ps.upload(3 * c, arr)
    ps.build()
    batch.set_pairs(0, ps, ps, ps, *packed)
    batch.run()
    batch.results()
    e2e_s = time.perf_counter() - e2e_t0
    # SURVEY 8(d)'s end-to-end definition: base images already on the device (a decoder's output), the
    # pyramids built there, the features / poses handed over from the host, the results read back
    ctx.synchronize()
    e2d_runs = []
    for _ in range(5):  # median of 5 (each a whole hand-over: pyramids, features, alignment, results)
        ctx.synchronize()
        e2d_t0 = time.perf_counter()
        ps.build()
        batch.set_pairs(0, ps, ps, ps, *packed)
        batch.run()
        batch.results()
        e2d_runs.append(time.perf_counter() - e2d_t0)
    e2d_s = float(np.median(e2d_runs))
    # the same hand-over for a stream of batches (a tracker's steady state): batch i + 1's pyramids build on the
    # context's prep stream (a second PyramidSet) while batch i's features are handed over and it aligns
    # (src/frame.cpp:26 builds each frame's pyramid before the frame is aligned); per batch: one build, one
    # set_pairs, one alignment, one read-back
    e2p_ms = e2q_ms = None
    if not args.core_only:
        ps2 = svo_amd.PyramidSet(3 * P, cam["width"], cam["height"], L, ctx)
        for c, arr in chunks:
            ps2.upload(3 * c, arr)
        sets = (ps, ps2)
        ps.build()
        ctx.synchronize()
        K = 8
        e2p_t0 = time.perf_counter()
        for i in range(K):
            cur_set, nxt = sets[i % 2], sets[(i + 1) % 2]
            nxt.build_async()
            batch.set_pairs(0, cur_set, cur_set, cur_set, *packed)
            batch.run()
            pk, _, _ = batch.results()
            if not np.array_equal(pk, poses):
                raise SystemExit("bench.py: pipelined end-to-end poses differ from the timed run")
        e2p_ms = (time.perf_counter() - e2p_t0) / K * 1e3
        ctx.synchronize()
        # two batches in flight: batch i + 1's features go up (copy stream) and its pyramids build (prep stream) while
        # batch i aligns; then batch i's results come back and batch i + 1 is queued
        batch2 = svo_amd.AlignBatch(camera, patch, 0, L - 1, P, nf, ctx, median_mode=mode)
        bats = (batch, batch2)
        ps.build()
        bats[0].set_pairs(0, ps, ps, ps, *packed)
        ctx.synchronize()
        e2q_t0 = time.perf_counter()
        bats[0].run()
        for i in range(K):
            cur_b, nxt_b = bats[i % 2], bats[(i + 1) % 2]
            nxt_s = sets[(i + 1) % 2]
            if i + 1 < K:
                nxt_s.build_async()
                nxt_b.set_pairs(0, nxt_s, nxt_s, nxt_s, *packed)
            pk, _, _ = cur_b.results()
            if not np.array_equal(pk, poses):
                raise SystemExit("bench.py: two-batch end-to-end poses differ from the timed run")
            if i + 1 < K:
                nxt_b.run()
        e2q_ms = (time.perf_counter() - e2q_t0) / K * 1e3
        batch2.close()
        batch.set_pairs(0, ps, ps, ps, *packed)  # (back on the first set)
        del ps2
    # the other median semantics on the same pairs: its rate and how far its poses are from the reference's
    other = svo_amd.MEDIAN_EXACT if mode == svo_amd.MEDIAN_REFERENCE else svo_amd.MEDIAN_REFERENCE
    other_line, lat, scaling_lines = None, None, None
    if not args.core_only:
        b2 = svo_amd.AlignBatch(camera, patch, 0, L - 1, P, nf, ctx, median_mode=other)
        b2.set_pairs(0, ps, ps, ps, *packed)
        b2.run()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            b2.run()
        ctx.synchronize()
        other_s = (time.perf_counter() - t0) / args.steps
        p2, _, _ = b2.results()
        b2.close()
        dpose = max(float(np.abs(canon(p2[i]) - canon(poses[i])).max()) for i in range(D))
        other_line = {"mode": "exact" if other == svo_amd.MEDIAN_EXACT else "reference",
                      "pairs_per_s": round(P / other_s, 1), "ms_per_step": round(other_s * 1e3, 4),
                      "max_abs_pose_param_diff_vs_headline": dpose,
                      "note": "same pairs; exact order statistics are not the reference's numbers (DESIGN.md)"}
        lat = latency_lines(ctx, scenes, camera, cam, patch, L, nf, mode)
        scaling_lines = batch_scaling(args, ctx, scenes, sidx, camera, cam, patch, L, nf, D, mode, poses)
    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    value = world * P * args.steps / elapsed
    b_pair = 3 * level_bytes(cam["width"], cam["height"], L) + nf * 64
    achieved = b_pair * P / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = None, None
    if args.pmc_json and os.path.exists(args.pmc_json):
        with open(args.pmc_json) as f:
            pm = json.load(f)
        # only a summary measured on this exact workload shape counts
        if pm.get("pairs") == P and pm.get("features") == nf and pm.get("levels") == L and pm.get("patch") == patch:
            traffic = pm.get("hbm_bytes_per_launch")
            traffic_src = os.path.relpath(args.pmc_json, ROOT)
    dominant = dominant_kernel(args.kernel_stats, P, n_chains(P, mode), b_pair, L) if mode == svo_amd.MEDIAN_REFERENCE else None
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"config 2: ImageAlignment::align, {nf} feats ({nf // 2} ref + {nf - nf // 2} lastKF), "
                               f"patch {patch}, {L}-level pyramid, {cam['width']}x{cam['height']}, {P} pairs/GPU",
                   "pairs_per_gpu": P, "features": nf, "levels": L, "patch": patch, "distinct_scenes": D,
                   "feature_order": args.feature_order,
                   "parallelism": f"pairs sharded over {world} GPU(s), no collective"
                                  + (" (rehearsal: every rank on device 0)" if shared_gpu else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "kernel": f"align chain: {L} levels x (K1 residual [+ pair init at the first level], K2 robust scale, "
                               f"K3 weights + LM step), {3 * L} launches per chain, {n_chains(P, mode)} concurrent "
                               f"sub-batch chains",
                     "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": b_pair * P,
                     "algorithmic_bytes_per_pair": b_pair, "traffic_source": traffic_src,
                     "stages_ms": {k: round(v, 4) for k, v in stages.items()},
                     "dominant_stage": max(stages, key=stages.get),
                     "dominant_kernel": dominant},
        # the co-limiting roof SURVEY 8(d) names: ~1900 algorithmic fp64 flop per feature and level
        # (bilinear blends, Jacobian, SE3 / projection, weights, 5 factored accumulators, 21 x 3 expansion)
        "roofline_fp64_valu": {"achieved": round(1900.0 * nf * L * P / (kernel_ms * 1e-3) / 1e12, 3),
                               "peak": FP64_VALU_PEAK_TFS, "unit": "TFLOP/s",
                               "frac": round(1900.0 * nf * L * P / (kernel_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFS, 5),
                               "flop_per_pair": 1900 * nf * L,
                               "note": "algorithmic flops (SURVEY 8(d) estimate); the issued VALU instructions are "
                                       "several times more (address, conversion, select): DESIGN 7 SQ counters"},
        "pyramid_build": {"frames": 3 * P, "ms": round(pyr_ms, 4), "statistic": "median of 5 after a warm-up build",
                          "frames_per_s": round(3 * P / (pyr_ms * 1e-3), 1),
                          # algorithmic bytes per frame: read the base image once, write the gradient
                          # base and levels 1.. of both stacks (SURVEY 8(d) pyramid row)
                          "algorithmic_bytes_per_frame": pyr_bytes,
                          "achieved_GBps": round(3 * P * pyr_bytes / (pyr_ms * 1e-3) / 1e9, 1),
                          "frac_hbm_peak": round(3 * P * pyr_bytes / (pyr_ms * 1e-3) / 8.0e12, 4)},
        "status_counts": {svo_amd.STATUS_NAMES[int(k)]: int(v) for k, v in zip(*np.unique(status, return_counts=True))},
        "median_semantics": ("reference: the reference's libstdc++ nth_element post-state (SVO_MEDIAN_REFERENCE)"
                             if mode == svo_amd.MEDIAN_REFERENCE else "exact order statistics (SVO_MEDIAN_EXACT)"),
        "poses_repeat_bitexact": poses_repeat,
        "step_ms_median_of_20": round(step_med * 1e3, 4),
        "other_median_mode": other_line,
        "end_to_end": {"pairs": P, "ms": round(e2e_s * 1e3, 3), "pairs_per_s": round(P / e2e_s, 1),
                       "note": "from host memory: H2D of 3P base images (pageable), pyramid build, all pairs' "
                               "features / poses in one svo_align_batch_set_pairs call, alignment, D2H of the results"},
        # (rounds 1-3 and 5 on: this key is the one-batch-at-a-time median; round 4 alone reported the pipelined
        # stream under it)
        "end_to_end_device_images": {"pairs": P, "ms": round(e2d_s * 1e3, 3), "pairs_per_s": round(P / e2d_s, 1),
                                     "runs": 5, "statistic": "median",
                                     "note": "SURVEY 8(d): base images already in HBM; one batch at a time: pyramid "
                                             "build, all pairs' features / poses from host memory in one "
                                             "svo_align_batch_set_pairs call, alignment, D2H of the results"},
        "end_to_end_device_images_pipelined": None if e2p_ms is None else {
            "pairs": P, "ms": round(e2p_ms, 3), "pairs_per_s": round(P / (e2p_ms * 1e-3), 1), "batches": 8,
            "statistic": "mean over a stream of 8 batches",
            "note": "the same hand-over for a stream of batches: batch i+1's pyramids build "
                    "(svo_pyramid_set_build_async, a second PyramidSet) while batch i aligns"},
        "end_to_end_device_images_two_batches": None if e2q_ms is None else {
            "pairs": P, "ms": round(e2q_ms, 3), "pairs_per_s": round(P / (e2q_ms * 1e-3), 1), "batches": 8,
            "statistic": "mean over a stream of 8 batches",
            "note": "two AlignBatch objects in flight: batch i+1's pyramids build and its features go up (copy stream) "
                    "while batch i aligns; then batch i's results come back and batch i+1 is queued"},
        "latency": lat,
        "batch_scaling": scaling_lines,
        "workload_16_distinct_scenes": w16,
        # key meanings across rounds: end_to_end_device_images is one batch at a time in rounds 1-3 and 5-6
        # (round 4 alone reported the pipelined stream under it, now end_to_end_device_images_pipelined); the headline
        # runs every pair on its own scene from round 6 (16 repeated scenes in rounds 1-5: workload_16_distinct_scenes)
        "schema": {"round": 6, "end_to_end_device_images": "one batch at a time (rounds 1-3, 5-6)",
                   "headline_scenes": "one scene per pair (round 6); 16 repeated scenes (rounds 1-5)"},
    }
    if not args.no_secondary:
        out["secondary"] = secondary(args, ctx, scenes[0], cam, camera)
    if not args.no_cpu and world == 1:
        out.update(cpu_baseline(args, scenes, poses[rep], L, patch, nthreads, mode))
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def dominant_kernel(path, P, chains, b_pair, L):
    """The dominant kernel's roofline from a committed headline-only kernel trace (profiles/headline_kernel_stats.csv,
    tools/headline_kernel_stats.py): K2V's median duration per launch of P / chains pairs, its algorithmic bytes per
    launch (one level of b_pair per pair: the level's share of the three stacks and the features), the HBM fraction.
    Tracked-file arithmetic only (the live figure is the chain's, above); None without a matching file."""
    if not path or not os.path.exists(path):
        return None
    import csv
    per = P // chains
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["kernel"].startswith("void align_scale_refv_kernel") and int(r["grid_x"]) == per * int(r["workgroup_x"]):
                us = float(r["median_us"])
                byt = per * b_pair / L
                return {"name": "align_scale_refv_kernel (K2V)", "pairs_per_launch": per, "launch_median_us": us,
                        "launches_in_trace": int(r["count"]), "algorithmic_bytes_per_launch": round(byt),
                        "achieved_GBps": round(byt / (us * 1e-6) / 1e9, 1),
                        "frac": round(byt / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
                        # a launch holds one CU per pair: 256 / per launches fill the chip side by side
                        "frac_chip": round(byt / (us * 1e-6) / 1e9 / HBM_PEAK_GBS * 256 / per, 5),
                        "note": "one launch = one level of a chain's pairs on one CU each; frac_chip counts the "
                                "256 / pairs_per_launch launches that run side by side; latency-bound (DESIGN 16, 19)",
                        "source": os.path.relpath(path, ROOT)}
    return None


def n_chains(P, mode):
    """Concurrent sub-batch chains run_batch uses (csrc/capi.hip: kSplitMin, kSplits, kSplitsRefv*; the bench's vectors
    always fit K2V)."""
    if P < 64:
        return 1
    return 4 if mode == svo_amd.MEDIAN_REFERENCE and P >= 512 else 2


def batch_scaling(args, ctx, scenes, sidx, camera, cam, patch, L, nf, D, mode, poses):
    """The same workload at 2x and 4x the pairs per GPU (each pair with its own three pyramids, uploaded and built
    like the headline's), steps timed like the headline; every pair's pose must equal the headline's pair of the same
    scene bit for bit.  Not `value`: the headline's batch stays the round-to-round workload."""
    P = len(sidx)
    out = {}
    for mult in (2, 4):
        Q = mult * P
        idx = sidx * mult
        ps = svo_amd.PyramidSet(3 * Q, cam["width"], cam["height"], L, ctx)
        for c, arr in image_chunks(scenes, idx, D):
            ps.upload(3 * c, arr)
        ps.build()
        b = svo_amd.AlignBatch(camera, patch, 0, L - 1, Q, nf, ctx, median_mode=mode)
        b.set_pairs(0, ps, ps, ps, *packed_pairs(scenes, Q, D, idx))
        for _ in range(2):
            b.run()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            b.run()
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        pq, _, _ = b.results()
        same = bool(all(np.array_equal(pq[j], poses[j % P]) for j in range(Q)))
        b.close()
        ps.close()
        out[f"pairs_per_gpu_{Q}"] = {"pairs_per_s": round(Q / dt, 1), "ms_per_step": round(dt * 1e3, 4),
                                     "chains": n_chains(Q, mode), "poses_equal_headline": same}
    out["note"] = ("the headline's workload with more pairs per GPU per step (more independent chains fill the CUs a "
                   "K2V launch frees); not the headline value")
    return out


def latency_lines(ctx, scenes, camera, cam, patch, L, nf, mode, reps=20):
    """SURVEY 8(d) latency rows: n_pairs = 1 through the class surface (ImageAlignment::align as
    src/system.cpp:313 calls it, per frame, reusing its batch), and batches of 64 and 512 pairs (run +
    results); median of `reps` calls after 3 warm-ups, host clock."""
    out = {}
    s = scenes[0]
    kf = svo_amd.Frame(camera, s.kf_img, L, ctx=ctx)
    kf.abs_pose[:] = s.kf_pose
    ref = svo_amd.Frame(camera, s.ref_img, L, last_keyframe=kf, ctx=ctx)
    ref.abs_pose[:] = s.ref_pose
    cur = svo_amd.Frame(camera, s.cur_img, L, last_keyframe=kf, ctx=ctx)
    for i in range(len(s.px)):
        fr = ref if i < s.n_ref else kf
        fr.add_feature(svo_amd.Feature(fr, s.px[i], bearing=s.bearing[i], point=svo_amd.Point(s.point[i])))
    ia = svo_amd.ImageAlignment(patch, 0, L - 1, ctx=ctx, median_mode=mode)
    ts = []
    for r in range(reps + 3):
        cur.abs_pose[:] = s.cur_init_pose
        t = time.perf_counter()
        ia.align(ref, cur)
        if r >= 3:
            ts.append(time.perf_counter() - t)
    out["n_pairs_1_class_surface_ms"] = round(float(np.median(ts)) * 1e3, 4)
    # the same per-frame call through the C++ mirror (host/svo.hpp ImageAlignment via build/svo_host_check
    # align ... REPS): what the reference's C++ System pays, without the Python mirror's gather of the
    # Feature objects; reported only when its pose equals the class surface's bit for bit
    py_pose = np.array(cur.abs_pose, dtype=np.float64)
    out["n_pairs_1_cpp_mirror_ms"] = None
    exe = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    if os.path.exists(exe):
        import subprocess
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            paths = synth.write_align_problem(s, td)
            r = subprocess.run([exe, "align", *paths, str(patch), "0", str(L - 1), str(int(mode)), str(reps)],
                               capture_output=True, text=True, timeout=120)
            lines = r.stdout.splitlines() if r.returncode == 0 else []
            if len(lines) == 3 and lines[2].startswith("ms "):
                cpp_pose = np.array([float(x) for x in lines[0].split()[2:9]])
                if np.array_equal(cpp_pose, py_pose):
                    out["n_pairs_1_cpp_mirror_ms"] = round(float(lines[2].split()[1]), 4)
    for n in (64, 512):
        D = len(scenes)
        ps = svo_amd.PyramidSet(3 * n, cam["width"], cam["height"], L, ctx)
        base = np.stack([im for sc in scenes for im in (sc.ref_img, sc.kf_img, sc.cur_img)])
        for first in range(0, n, D):
            ps.upload(3 * first, base[:3 * min(D, n - first)])
        ps.build()
        b = svo_amd.AlignBatch(camera, patch, 0, L - 1, n, nf, ctx, median_mode=mode)
        b.set_pairs(0, ps, ps, ps, *packed_pairs(scenes, n, D))
        ts = []
        for r in range(reps + 3):
            ctx.synchronize()
            t = time.perf_counter()
            b.run()
            b.results()
            if r >= 3:
                ts.append(time.perf_counter() - t)
        out[f"n_pairs_{n}_ms"] = round(float(np.median(ts)) * 1e3, 4)
        b.close()
        del ps
    out["statistic"] = f"median of {reps} after 3 warm-ups (run + results, host clock)"
    return out


def rehearsal(args, rank, world, dist):
    """The multi-rank path without a GPU: each rank's step aligns its --pairs with the CPU oracle (tests)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402  (rehearsal only)
    P, nf, L, patch = args.pairs, args.features, args.levels, args.patch
    first, _ = shard.pair_block(world * P, rank, world)
    scenes = [synth.make_pair(seed=synth.SEED_BASE + first + i, n_features=nf, patch_size=patch, nthreads=1)
              for i in range(P)]
    pairs = []
    for s in scenes:
        pyr = [O.build_pyramid(im, L)[0] for im in (s.ref_img, s.kf_img, s.cur_img)]
        pairs.append(O.make_pair(pyr[0], pyr[1], pyr[2], s.ref_pose, s.kf_pose, s.n_ref, s.n_kf, s.px, s.bearing,
                                 s.point, s.has_point))

    def step():
        return [O.image_align(s.camera, patch, 0, L - 1, pr, s.cur_init_pose, 0)[0] for s, pr in zip(scenes, pairs)]

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        poses = step()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        gathered = shard.gather_blocks([list(map(float, p)) for p in poses], dist)
    else:
        gathered = [list(map(float, p)) for p in poses]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(world * P * args.steps / elapsed, 3), "unit": "pairs/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "cpu rehearsal (no GPU)",
                          "config": {"workload": "rehearsal", "pairs_per_gpu": P, "features": nf, "levels": L},
                          "poses": gathered}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def secondary(args, ctx, scene, cam, camera, reps=20):
    """BASELINE configs 3 and 5 on this GPU, through the synchronous C-ABI calls (each call includes its
    H2D / D2H copies and device allocations: end-to-end per call, not kernel time), with the oracle's
    single-thread time on the same input beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402  (CPU baseline only)
    res = {}
    # config 3: FeatureAlignment, 2000 candidates, level-0 gradients of the ref and cur frames
    ps = svo_amd.PyramidSet(2, cam["width"], cam["height"], 1, ctx)
    ps.upload(0, np.stack([scene.ref_img, scene.cur_img]))
    ps.build()
    rng = np.random.default_rng(3)
    n = min(2000, len(scene.px))
    ref_px = np.ascontiguousarray(scene.px[:n])
    init = ref_px + rng.uniform(-1.5, 1.5, ref_px.shape)
    rg, cg = O.build_pyramid(scene.ref_img, 1)[1], O.build_pyramid(scene.cur_img, 1)[1]
    for p in (8, 7):
        fa = svo_amd.FeatureAlignment(p, ctx=ctx)
        px = np.ascontiguousarray(init.copy())
        fa.align_batch(ps, 0, ps, 1, ref_px, px, camera)
        t0 = time.perf_counter()
        for _ in range(reps):
            px = np.ascontiguousarray(init.copy())
            fa.align_batch(ps, 0, ps, 1, ref_px, px, camera)
        g = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        pxc, _, _ = O.feature_align(scene.camera, p, rg.reshape(cam["height"], cam["width"]),
                                    cg.reshape(cam["height"], cam["width"]), ref_px, init)
        c = time.perf_counter() - t0
        res[f"config3_feature_align_p{p}"] = {
            "candidates": n, "gpu_ms_per_call": round(g * 1e3, 4), "candidates_per_s": round(n / g, 1),
            "cpu_ms_1_thread": round(c * 1e3, 3), "bitexact_vs_oracle": bool(np.array_equal(px, pxc))}
    # config 5: depth-filter update, 2000 seeds on the keyframe against the cur frame
    dp = synth.make_depth_problem(n_seeds=2000)
    ds = svo_amd.PyramidSet(2, cam["width"], cam["height"], 1, ctx)
    ds.upload(0, np.stack([dp.kf_img, dp.cur_img]))
    ds.build()
    seeds = svo_amd.depth_seeds(dp.px, dp.bearing, dp.depth_mean, dp.depth_min)
    out = svo_amd.depth_update(camera, [(ds, 0, dp.kf_pose)], (ds, 1), dp.cur_pose, seeds, ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        svo_amd.depth_update(camera, [(ds, 0, dp.kf_pose)], (ds, 1), dp.cur_pose, seeds, ctx)
    g = (time.perf_counter() - t0) / reps
    oseeds = O.make_seeds(dp.px, dp.bearing, dp.depth_mean, dp.depth_min)
    t0 = time.perf_counter()
    oc = O.depth_update(dp.camera, [dp.kf_img], dp.kf_pose[None], dp.cur_img, dp.cur_pose, oseeds)
    c = time.perf_counter() - t0
    res["config5_depth_filter"] = {
        "seeds": len(seeds), "gpu_ms_per_call": round(g * 1e3, 4), "seeds_per_s": round(len(seeds) / g, 1),
        "cpu_ms_1_thread": round(c * 1e3, 3), "outcomes": np.bincount(out[1], minlength=5).tolist(),
        "outcomes_match_oracle": bool(np.array_equal(out[1], oc[1]))}
    # Map::reprojectMap + addCandidateToFrame on a config-2 map (ref frame + last
    # keyframe, 2000 features, 150 depth-filter candidates): host plan + one batched FeatureAlignment
    # launch per call, against the oracle's one-alignment-at-a-time restatement.  Fresh object graphs
    # per repetition (the calls mutate the map), built outside the timed region.
    mp = synth.make_map_problem()
    graphs = [synth.map_objects(mp, ctx=ctx) for _ in range(reps + 1)]
    news = []
    t0 = None
    native = 0.0
    for i, (m, ref, _, cur, _, _) in enumerate(graphs):
        if i == 1:
            t0 = time.perf_counter()
        m.reproject_map(ref, cur, [])
        m.add_candidate_to_frame(cur)
        if i == 0:  # (the output checked below; the timed repetitions only run the calls)
            news.append(np.array([f.pixel_position for f in cur.features]))
        if i >= 1:
            native += m.native_seconds
    g = (time.perf_counter() - t0) / reps
    native /= reps
    gr = {k: O.unpack_levels(O.build_pyramid(img, 1)[1], cam["width"], cam["height"], 1)[0]
          for k, img in (("ref", mp.ref_img), ("kf", mp.kf_img), ("cur", mp.cur_img))}
    m0 = graphs[0][0]
    ptype, psucc = mp.point_type.copy(), mp.point_succ.copy()
    plast = np.full(len(mp.point_pos), np.uint64(2 ** 64 - 1), np.uint64)
    visited = np.zeros(len(m0.cell_orders), np.uint8)
    t0 = time.perf_counter()
    rep = O.reproject_map(mp.camera, mp.cell_size, m0.cell_orders, mp.cur_pose, graphs[0][3].id, gr["cur"],
                          [gr["ref"], gr["kf"]], np.array([0, mp.n_ref, mp.n_ref + mp.n_kf], np.int32), mp.feat_px,
                          mp.feat_point, mp.point_pos, ptype, psucc, plast, visited)
    cm, cpx = O.add_candidates(mp.camera, mp.cell_size, visited, mp.cur_pose, gr["cur"], [gr["kf"]] * len(mp.cand_feat),
                               mp.feat_px[mp.cand_feat], mp.cand_pos)
    c = time.perf_counter() - t0
    expect = np.concatenate([rep[1], cpx[cm]])
    for _, ref, kf, cur, _, _ in graphs:  # release the device pyramids now (Frame <-> Feature cycles)
        for fr in (ref, kf, cur):
            fr.image_pyramid.clear()
    del graphs
    # the same call through the C++ mirror (host/svo.hpp Map via build/svo_host_check map ... REPS): what a
    # C++ caller of the C ABI pays per frame; reported only when its output is the oracle's, bit for bit
    cpp_ms = None
    exe = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    if os.path.exists(exe):
        import subprocess
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            paths = synth.write_map_problem(mp, td, m0.cell_orders)
            r = subprocess.run([exe, "map", *paths, str(reps)], capture_output=True, text=True, timeout=120)
            lines = r.stdout.splitlines() if r.returncode == 0 else []
            cpx_cpp = np.array([[float(v) for v in ln.split()[1:]] for ln in lines if ln.startswith("px ")])
            if lines and lines[-1].startswith("ms ") and np.array_equal(cpx_cpp.reshape(-1, 2), expect):
                cpp_ms = float(lines[-1].split()[1])
    res["map_reproject"] = {
        "map_points": len(mp.point_pos), "candidates": len(mp.cand_feat), "matches": int(rep[4]),
        "new_features": int(len(expect)), "gpu_ms_per_call": round(g * 1e3, 4),
        "native_ms_per_call": round(native * 1e3, 4),
        "cpp_mirror_ms_per_call": None if cpp_ms is None else round(cpp_ms, 4), "cpu_ms_1_thread": round(c * 1e3, 3),
        "bitexact_vs_oracle": bool(np.array_equal(news[0], expect)),
        "note": "gpu: end to end per frame through the Python mirror (object bookkeeping included); native: the "
                "time inside the C ABI calls (host plan, projection, two batched FeatureAlignment launches); "
                "cpp_mirror: end to end through the C++ Map (null unless its output equals the oracle's)"}
    # FeatureSelection on a KITTI-shaped keyframe (threshold 50, 200 candidates,
    # bucketing in 30-px cells: src/system.cpp:253, config/config.json).  gpu = the whole call (device
    # detection + D2H of the keys + host std::sort / SSC); detect_call = svo_feature_detect alone (2 kernels +
    # the keys' D2H; the kernel times are in the rocprof summary).
    fr = svo_amd.Frame(camera, scene.ref_img, 1, ctx=ctx)
    fsel = svo_amd.FeatureSelection(cam["width"], cam["height"], 30, ctx=ctx)
    fsel.gradient_magnitude_with_ssc(fr, 50, 200, True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fr.features = []
        fsel.gradient_magnitude_with_ssc(fr, 50, 200, True)
    g = (time.perf_counter() - t0) / reps
    got = np.array([f.pixel_position for f in fr.features])
    t0 = time.perf_counter()
    for _ in range(reps):
        fsel.detect(fr, 50)
    det_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    opx, _, _, nk = O.feature_select_ssc(scene.ref_img, 50, 200, True, 30)
    c = time.perf_counter() - t0
    fr.features = []
    t0 = time.perf_counter()
    for _ in range(reps):
        fr.features = []
        fsel.gradient_magnitude_by_value(fr, 50)
    gv = (time.perf_counter() - t0) / reps
    gotv = np.array([f.pixel_position for f in fr.features])
    t0 = time.perf_counter()
    vpx, _, _ = O.feature_select_by_value(scene.ref_img, 50, 30)
    cv = time.perf_counter() - t0
    fr.image_pyramid.clear()
    # the same calls through the C++ mirror (host/svo.hpp FeatureSelection via build/svo_host_check with
    # SVO_CHECK_REPS): reported only when its features equal the oracle's
    cpp_fs = {"fs": None, "fv": None}
    exe = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    if os.path.exists(exe):
        import subprocess
        import tempfile
        with tempfile.NamedTemporaryFile(suffix=".raw") as tf:
            tf.write(np.ascontiguousarray(scene.ref_img, np.uint8).tobytes())
            tf.flush()
            W, H = str(cam["width"]), str(cam["height"])
            for mode, argv, want in (("fs", [W, H, "30", "50", "200", "1", tf.name], opx), ("fv", [W, H, "30", "50", tf.name], vpx)):
                r = subprocess.run([exe, mode, *argv], capture_output=True, text=True, timeout=120,
                                   env=dict(os.environ, SVO_CHECK_REPS=str(reps)))
                if r.returncode != 0:
                    continue
                got_cpp = np.array([[float(v) for v in ln.split()[:2]] for ln in r.stdout.splitlines()]).reshape(-1, 2)
                ms = [ln for ln in r.stderr.splitlines() if ln.startswith("ms ")]
                if ms and np.array_equal(got_cpp, want):
                    cpp_fs[mode] = round(float(ms[-1].split()[1]), 4)
    res["feature_selection"] = {
        "keypoints": int(nk), "features": int(len(opx)), "gpu_ms_per_call": round(g * 1e3, 4),
        "detect_call_ms": round(det_ms, 4), "cpu_ms_1_thread": round(c * 1e3, 3),
        "bitexact_vs_oracle": bool(np.array_equal(got, opx)),
        "by_value_gpu_ms_per_call": round(gv * 1e3, 4), "by_value_cpu_ms_1_thread": round(cv * 1e3, 3),
        "by_value_bitexact_vs_oracle": bool(np.array_equal(gotv, vpx)),
        "cpp_mirror_ms_per_call": cpp_fs["fs"], "by_value_cpp_mirror_ms_per_call": cpp_fs["fv"],
        "note": "gradientMagnitudeWithSSC end to end per keyframe (device detect + host sort/SSC, "
                "Python mirror); ByValue: one device launch per call"}
    # BundleAdjustment::optimizePose for 512 frames of 1000 features each (85 % with a
    # point, the flags a previous call left), one workgroup per frame, against the oracle on 32 of them.
    rng = np.random.default_rng(4)
    F, nfe = 512, 1000
    P = rng.normal(size=(F * nfe, 3)) * [4, 2, 3] + [0, 0, 12]
    bear = P / np.linalg.norm(P, axis=1, keepdims=True) + rng.normal(size=P.shape) * 2e-3
    has = (rng.random(F * nfe) > 0.15).astype(np.uint8)
    off = np.arange(F + 1, dtype=np.int32) * nfe
    poses0 = np.tile(np.array([0, 0, 0, 1, 0.02, -0.01, 0.03]), (F, 1))
    vis = has.copy()
    pz = poses0.copy()
    svo_amd.pose_optimize_batch(off, bear, P, has, vis, pz, ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        vis[:] = has
        pz[:] = poses0
        err_b, st_b = svo_amd.pose_optimize_batch(off, bear, P, has, vis, pz, ctx)
    g = (time.perf_counter() - t0) / reps
    ns = 32
    t0 = time.perf_counter()
    worst = 0.0
    for f in range(ns):
        sl = slice(f * nfe, (f + 1) * nfe)
        po, eo, so, _ = O.optimize_pose(bear[sl], P[sl], has[sl], has[sl], poses0[f])
        q = pz[f] if np.dot(pz[f][:4], po[:4]) >= 0 else np.concatenate([-pz[f][:4], pz[f][4:]])
        worst = max(worst, float(np.abs(q - po).max()))
    c = (time.perf_counter() - t0) / ns
    res["pose_ba"] = {
        "frames": F, "features_per_frame": nfe, "gpu_ms_per_call": round(g * 1e3, 4),
        "frames_per_s": round(F / g, 1), "cpu_ms_per_frame_1_thread": round(c * 1e3, 4),
        "cpu_frames_per_s_1_thread": round(1.0 / c, 1), "max_abs_pose_diff_vs_oracle": worst,
        "status_counts": np.bincount(st_b + 1, minlength=11).tolist(),
        "note": "BundleAdjustment::optimizePose batched (H2D of the features included); oracle: 32 frames"}
    return res


def physical_cores():
    """Physical cores of this host (sockets x "cpu cores" in /proc/cpuinfo), or None."""
    try:
        socks, cores = set(), None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    socks.add(line.split(":", 1)[1].strip())
                elif line.startswith("cpu cores") and cores is None:
                    cores = int(line.split(":", 1)[1])
        return len(socks or {"0"}) * cores if cores else None
    except (OSError, ValueError):
        return None


def cpu_baseline(args, scenes, gpu_poses, L, patch, nthreads, mode=None):
    """The oracle (faithful C++ restatement) timed on this host on a bounded sample of the same workload
    (SURVEY 8(d)(ii)), in two builds: the CPU-baseline build made here at bench time with BASELINE.md's Release
    flags (-O3 -DNDEBUG -march=native, FMA contraction allowed: oracle/Makefile `native`) and the portable parity
    build (-march=x86-64-v3 -ffp-contract=off, the checker).  One thread, and one pinned thread per available CPU
    (the process affinity mask, capped by the box's CPU share OMP_NUM_THREADS); each the median of 20 runs after
    3 warm-ups.  Also the SE(3) error of the GPU poses against the parity oracle on every distinct scene (the bench
    checks that all pairs repeat their scene's pose bit for bit, so this covers both half-batch chains)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402  (CPU baseline / checker only)
    omode = 1 if mode == svo_amd.MEDIAN_EXACT else 0  # oracle median_mode 0 = the reference's nth_element
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(nthreads)  # (the checker's pyramids and poses; ctypes releases the GIL)
    pyrs = list(pool.map(lambda s: [O.build_pyramid(im, L)[0] for im in (s.ref_img, s.kf_img, s.cur_img)], scenes))
    pairs = [O.make_pair(p[0], p[1], p[2], s.ref_pose, s.kf_pose, s.n_ref, s.n_kf, s.px, s.bearing, s.point, s.has_point)
             for p, s in zip(pyrs, scenes)]
    ref_poses = list(pool.map(lambda i: O.image_align(scenes[i].camera, patch, 0, L - 1, pairs[i],
                                                      scenes[i].cur_init_pose, omode)[0], range(len(scenes))))
    se3_err = max(float(np.abs(canon(ref_poses[i]) - canon(gpu_poses[i])).max()) for i in range(len(scenes)))
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", avail) or avail)
    threads = max(1, min(avail, share))
    n_mt = 2 * threads
    idx = [i % len(scenes) for i in range(n_mt)]
    sel = [pairs[i] for i in idx]
    init = np.stack([scenes[i].cur_init_pose for i in idx])

    def timed(Lib):
        ts = []  # one thread: 3 warm-ups, 20 timed alignments
        for r in range(23):
            i = r % len(scenes)
            t = time.perf_counter()
            O.image_align(scenes[i].camera, patch, 0, L - 1, pairs[i], scenes[i].cur_init_pose, omode, L=Lib)
            if r >= 3:
                ts.append(time.perf_counter() - t)
        rates = []  # all available CPUs, one pinned worker each: runs of 2 alignments per thread
        for r in range(23):
            t = time.perf_counter()
            O.image_align_batch(scenes[0].camera, patch, 0, L - 1, sel, init, omode, threads, L=Lib)
            if r >= 3:
                rates.append(n_mt / (time.perf_counter() - t))
        return 1.0 / float(np.median(ts)), float(np.median(rates))

    port_single, port_multi = timed(None)
    nat = O.native_lib()
    nat_single = nat_multi = None
    nat_diff = None
    if nat is not None:
        nat_single, nat_multi = timed(nat)
        nat_poses = list(pool.map(lambda i: O.image_align(scenes[i].camera, patch, 0, L - 1, pairs[i],
                                                          scenes[i].cur_init_pose, omode, L=nat)[0], range(len(scenes))))
        nat_diff = max(float(np.abs(canon(nat_poses[i]) - canon(ref_poses[i])).max()) for i in range(len(scenes)))
    pool.shutdown()
    single, multi = (nat_single, nat_multi) if nat is not None else (port_single, port_multi)
    build = ("oracle/svo_oracle.cpp, -O3 -DNDEBUG -march=native (built on this host at bench time, FMA contraction "
             "allowed)" if nat is not None else
             "oracle/svo_oracle.cpp, -O3 -DNDEBUG -march=x86-64-v3 -ffp-contract=off (the native build failed)")
    phys = physical_cores()
    return {
        "cpu_baseline": {"value": round(single, 3), "unit": "pairs/s", "cores": 1, "kind": "port",
                         "cpu_model": cpu_model(), "build": build,
                         "sample": "median of 20 single ImageAlignment::align calls (config 2 shape, "
                                   f"{len(scenes)} scenes) after 3 warm-ups, 1 host thread"},
        "cpu_baseline_multicore": {"value": round(multi, 3), "unit": "pairs/s", "cores": threads, "kind": "port",
                                   "available_cpus": avail, "cpu_share": share, "build": build,
                                   "sample": f"median of 20 runs of {n_mt} alignments ({threads} threads pinned one per "
                                             "available CPU, one alignment per thread at a time) after 3 warm-ups",
                                   "physical_cores_of_host": phys,
                                   "extrapolated_full_host_pairs_per_s": (round(single * phys, 1) if phys else None),
                                   "extrapolation_note": "1-thread rate x the host's physical cores (linear, no memory "
                                                         "or clock effects): the rate the whole host would give if every "
                                                         "core ran one alignment; this box grants the process only "
                                                         "cpu_share CPUs"},
        "cpu_baseline_portable_build": {"value": round(port_single, 3), "multicore_value": round(port_multi, 3),
                                        "unit": "pairs/s",
                                        "build": "oracle/svo_oracle.cpp, -O3 -DNDEBUG -march=x86-64-v3 -ffp-contract=off "
                                                 "(the parity checker)",
                                        "max_abs_pose_diff_native_vs_portable": nat_diff},
        "se3_err_vs_ref": {"max_abs_param_diff": se3_err, "pairs": len(scenes),
                           "reference_semantics": ("libstdc++ nth_element median (oracle median_mode 0)" if omode == 0
                                                   else "exact order statistics (oracle median_mode 1)")},
    }


if __name__ == "__main__":
    main()
