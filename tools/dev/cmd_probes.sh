# K2V probe (bit-exact + cycles) on each dev library given as arguments (dirs under semi-direct-visual-odometry_amd/)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in "$@"; do
  SVO_LIB_DIR=semi-direct-visual-odometry_amd/$d timeout -k 10 120 python3 tools/k2r_probe.py 2 > gpurun_out/p_$d.log 2>&1; rc=$?
  echo "== $d rc=$rc"; head -3 gpurun_out/p_$d.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
