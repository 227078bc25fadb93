#!/bin/bash
# Pyramid build measurements on the GPU box (each GPU step under its own limit, stops at the first crash / timeout):
#   1. tools/pyr_time.py under each SVO_PYR mode given (default: 1 0), two alternating rounds;
#   2. a kernel-trace summary of the default build (per-level launch durations);
#   3. FETCH_SIZE and WRITE_SIZE passes over the default build (each its own rocprofv3 run).
# usage: tools/pyr_measure.sh [modes...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pyr
mkdir -p "$out"
modes=${*:-1 0}
step() {
    local name=$1 limit=$2; shift 2
    timeout -k 10 "$limit" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    tail -n 3 "$out/$name.log"
    if [ "$rc" -ne 0 ]; then echo "== $name rc=$rc: stopping"; exit "$rc"; fi
}
for i in 1 2; do
    for m in $modes; do
        echo "== round $i SVO_PYR=$m"
        SVO_PYR=$m step "time_${m}_$i" 120 python3 tools/pyr_time.py
    done
done
echo "== kernel trace"
step trace 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 tools/pyr_time.py
echo "== FETCH_SIZE"
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 tools/pyr_time.py
echo "== WRITE_SIZE"
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 tools/pyr_time.py
echo "== done"
