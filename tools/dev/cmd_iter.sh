# iteration loop on the GPU box: K2V probe (timing + bit-exactness), the reference-median tests, a short bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/probe.log 2>&1 && \
timeout -k 10 300 python3 -u -m pytest tests/test_batch_chains.py tests/test_gpu_parity.py tests/test_reference_median.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary > gpurun_out/it_bench.log 2>&1
rc=$?
echo rc=$rc
cat gpurun_out/probe.log; tail -3 gpurun_out/it_tests.log
python3 - <<'PY'
import json
for line in open('gpurun_out/it_bench.log'):
    if line.startswith('{'):
        d = json.loads(line)
        print('value', d['value'], 'ms', d['ms_per_step'], 'stages', d['roofline']['stages_ms'], 'lat', d['latency'], 'repeat', d['poses_repeat_bitexact'])
PY
if [ "${SQ:-0}" = 1 ] && [ $rc = 0 ]; then
  bash tools/pmc_probe.sh gpurun_out/sq_k2v "python3 tools/k2r_probe.py 2" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
    "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM" > gpurun_out/sq.log 2>&1
  tail -4 gpurun_out/sq.log
fi
