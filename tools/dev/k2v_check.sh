#!/bin/bash
# K2V change check on the GPU box: the K2V parity tests, the probe's cycles, then an A/B of the bench against a
# baseline library (build/<base>): tools/dev/k2v_check.sh <base>
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    tests/test_k2v_rounds.py tests/test_reference_median.py tests/test_config4.py tests/test_batch_chains.py > gpurun_out/k2v_tests.log 2>&1
tail -2 gpurun_out/k2v_tests.log
timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/k2v_probe.txt 2>&1
SVO_LIB_DIR=semi-direct-visual-odometry_amd/build/$1 timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/k2v_probe_base.txt 2>&1
head -3 gpurun_out/k2v_probe.txt gpurun_out/k2v_probe_base.txt
tools/ab_libs.sh . "$1"
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
