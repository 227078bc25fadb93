# a dev library (argument: build dir under semi-direct-visual-odometry_amd/) : probe + stamps probe (config-2 shape),
# 60k probe, round traces vs the model, random sweep
set -u
export TMPDIR=/tmp
D=semi-direct-visual-odometry_amd/$1
mkdir -p gpurun_out
for n in 50000 60000; do
  SVO_LIB_DIR=$D timeout -k 10 150 python3 tools/dev/k2v_trace.py $n > gpurun_out/d_trace$n.log 2>&1; rc=$?
  echo "trace $n rc=$rc"; grep -v "^round" gpurun_out/d_trace$n.log; grep -A8 "HEADER\|diffs" gpurun_out/d_trace$n.log | head -20
  [ $rc -ne 0 ] && exit $rc
done
SVO_LIB_DIR=$D timeout -k 10 150 python3 tools/k2r_probe.py 2 > gpurun_out/d_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/d_probe.log
[ $rc -ne 0 ] && exit $rc
SVO_LIB_DIR=$D/stamps timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/d_stamps.log 2>&1; rc=$?
echo "stamps rc=$rc"; cat gpurun_out/d_stamps.log
[ $rc -ne 0 ] && exit $rc
SVO_PROBE_SLOTS=60000 SVO_LIB_DIR=$D timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/d_probe60k.log 2>&1; rc=$?
echo "probe60k rc=$rc"; cat gpurun_out/d_probe60k.log
[ $rc -ne 0 ] && exit $rc
SVO_LIB_DIR=$D timeout -k 10 300 python3 tools/dev/k2v_sweep.py 3 > gpurun_out/d_sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; tail -5 gpurun_out/d_sweep.log
exit $rc
