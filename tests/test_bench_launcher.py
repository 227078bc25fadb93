"""bench.py's multi-rank path on CPU: `bench.py --gpus 2` starts two ranks itself (child processes,
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, gloo barrier and max-over-ranks time), rank 0 prints one
JSON line.  --cpu-rehearsal replaces the GPU step by the CPU oracle, so the launcher, the sharding
(svo_amd.shard.pair_block, weak scaling) and the rank-order gather run here exactly as on a GPU node."""
import json
import os
import subprocess
import sys

import numpy as np

import svo_amd.synth as synth
from common import oracle_align

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--pairs", "2", "--features", "120", "--levels", "3", "--steps", "1", "--warmup", "0", "--cpu-rehearsal"]


def _run(extra, env=None):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS, *extra], capture_output=True,
                          text=True, timeout=600, env=e, cwd=ROOT)


def test_bench_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["value"] > 0
    poses = np.array(out["poses"])
    assert poses.shape == (4, 7)  # 2 pairs per rank, rank order
    for i in range(4):
        s = synth.make_pair(seed=synth.SEED_BASE + i, n_features=120, nthreads=1)
        pose, _, _, _ = oracle_align(s, 5, 0, 2, mode=0, trace=False)
        assert np.array_equal(poses[i], np.asarray(pose)), i


def test_bench_rejects_world_size_mismatch():
    r = _run(["--gpus", "2"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in (r.stderr + r.stdout)


def test_bench_chain_count_follows_the_library():
    """bench.py's n_chains (the `roofline.kernel` text and the batch-scaling lines) restates run_batch's split rule;
    the constants it restates are read from csrc/capi.hip so the two cannot drift apart."""
    import re
    sys.path.insert(0, ROOT)
    import bench
    import svo_amd
    src = open(os.path.join(ROOT, "semi-direct-visual-odometry_amd", "csrc", "capi.hip")).read()
    const = {k: int(re.search(rf"constexpr int(?:32_t)? {k} = (\d+);", src).group(1))
             for k in ("kSplitMin", "kSplits", "kSplitsRefv", "kSplitsRefvMin")}
    ref, exact = svo_amd.MEDIAN_REFERENCE, svo_amd.MEDIAN_EXACT
    bench.svo_amd = svo_amd
    assert bench.n_chains(const["kSplitMin"] - 1, ref) == 1
    assert bench.n_chains(const["kSplitMin"], ref) == const["kSplits"]
    assert bench.n_chains(const["kSplitsRefvMin"] - 1, ref) == const["kSplits"]
    assert bench.n_chains(const["kSplitsRefvMin"], ref) == const["kSplitsRefv"]
    assert bench.n_chains(const["kSplitsRefvMin"], exact) == const["kSplits"]
