# K2V gate on the product library (build/): bit-exact probes (config-2 shape, LayB's 60k) and a random sweep; only
# when all agree with the oracle: smoke, the GPU tests, the full bench (then stop; profiles in the next call)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 50000 60000; do
  timeout -k 10 150 python3 tools/dev/k2v_trace.py $n > gpurun_out/g_trace$n.log 2>&1; rc=$?
  echo "trace $n rc=$rc"; grep -v "^round" gpurun_out/g_trace$n.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 150 python3 tools/k2r_probe.py 2 > gpurun_out/g_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/g_probe.log
[ $rc -ne 0 ] && exit $rc
SVO_PROBE_SLOTS=60000 timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/g_probe60k.log 2>&1; rc=$?
echo "probe60k rc=$rc"; cat gpurun_out/g_probe60k.log
[ $rc -ne 0 ] && exit $rc
SVO_LIB_DIR=semi-direct-visual-odometry_amd/build/stamps timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/g_stamps.log 2>&1; rc=$?
echo "stamps rc=$rc"; cat gpurun_out/g_stamps.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/dev/k2v_sweep.py 4 > gpurun_out/g_sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; tail -5 gpurun_out/g_sweep.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_round.sh smoke tests bench
