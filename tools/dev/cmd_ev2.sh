# round evidence part 2 on the product library (build/): rocprof stats + top dispatches, PMC traffic, chain sweep,
# K2V probe (stamps build) and SQ counters
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_round.sh prof pmc
rc=$?
echo "round rc=$rc"
if [ "$rc" -ge 124 ]; then exit $rc; fi
SVO_LIB_DIR=semi-direct-visual-odometry_amd/build/stamps timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/ev_stamps.log 2>&1
echo "stamps rc=$?"; cat gpurun_out/ev_stamps.log
for c in 1 3 4; do
  SVO_CHAINS=$c timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary --core-only > gpurun_out/ev_chains$c.log 2>&1
  r=$?; echo "chains $c rc=$r"; grep -o '"value": [0-9.]*' gpurun_out/ev_chains$c.log
  if [ "$r" -ge 124 ]; then exit $r; fi
done
bash tools/dev/cmd_sq.sh > gpurun_out/ev_sq.log 2>&1; echo "sq rc=$?"
