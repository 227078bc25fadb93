# SQ counters of the K2V debug kernel (tools/k2r_probe.py 2) for the product library and a dev library ($1)
set -u
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
bash tools/pmc_probe.sh gpurun_out/sq_prod "python3 tools/k2r_probe.py 2" "$P1" "$P2" || exit $?
python3 tools/pmc_summary.py gpurun_out/sq_prod/p1 gpurun_out/sq_prod/p2 > gpurun_out/sq_prod.txt; cat gpurun_out/sq_prod.txt
if [ $# -ge 1 ]; then
  export SVO_LIB_DIR=semi-direct-visual-odometry_amd/$1
  bash tools/pmc_probe.sh gpurun_out/sq_dev "python3 tools/k2r_probe.py 2" "$P1" "$P2" || exit $?
  python3 tools/pmc_summary.py gpurun_out/sq_dev/p1 gpurun_out/sq_dev/p2 > gpurun_out/sq_dev.txt; cat gpurun_out/sq_dev.txt
fi
