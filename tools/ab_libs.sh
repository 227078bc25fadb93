# A/B of library builds on one box: tools/ab_libs.sh <dir>...  (each dir under semi-direct-visual-odometry_amd/build;
# "." = the in-tree build), two alternating rounds of the default bench without the CPU / secondary lines
set -e
for i in 1 2; do
  for d in "$@"; do
    SVO_LIB_DIR=semi-direct-visual-odometry_amd/build/$d timeout -k 5 200 python3 bench.py --no-cpu --no-secondary --steps 30 > gpurun_out/ab_${d//\//_}_$i.log 2>&1
  done
done
