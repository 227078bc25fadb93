#!/bin/bash
# GPU-box runner: each GPU step under its own time limit; stops at the first crash/timeout
# (exit >= 124), continues past ordinary test failures so the later measurements still run.
# usage: tools/gpu_round.sh <step>...   steps: smoke quick tests bench prof hprof d512 timeline pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
    local name=$1 limit=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ "$rc" -ge 124 ]; then echo "== stopping after $name (rc=$rc)"; exit "$rc"; fi
}
for step in "$@"; do
    case "$step" in
        smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
        quick) run quick 300 python3 tests/gpu_smoke.py ;;
        tests) run tests 900 python3 -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        bench) run bench 600 python3 bench.py ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu
              # the longest dispatches of the same trace, committed beside every kernel-stats summary
              python3 tools/top_dispatches.py gpurun_out/prof/run_kernel_trace.csv 10 > gpurun_out/top_dispatches.txt && cat gpurun_out/top_dispatches.txt ;;
        # the headline alone (no secondary / batch-scaling / latency lines), its kernel trace split by launch shape
        hprof) run hprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary --core-only
               python3 tools/headline_kernel_stats.py gpurun_out/hprof/run_kernel_trace.csv > gpurun_out/headline_kernel_stats.csv && cat gpurun_out/headline_kernel_stats.csv ;;
        # config 4's 512 distinct scenes (seeds 0x5EED0000 + pair), the timed loop only
        d512) run d512 600 python3 bench.py --distinct 512 --no-cpu --no-secondary --core-only ;;
        # per-workgroup K1 / K2V / K3 records of the headline (diagnostic build: make -C semi-direct-visual-odometry_amd timeline)
        timeline) run timeline 300 python3 tools/timeline.py --steps 3 --json gpurun_out/timeline.json ;;
        pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary --core-only
             run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary --core-only
             python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_traffic.json && cat gpurun_out/pmc_traffic.json ;;
        *) echo "unknown step $step" ;;
    esac
done
