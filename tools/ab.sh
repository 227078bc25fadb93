# A/B of two bench argument sets on one box, alternating: tools/ab.sh "<args A>" "<args B>"
set -e
for i in 1 2; do
timeout -k 5 200 python3 bench.py --no-cpu --no-secondary --steps 30 $1 > gpurun_out/new$i.log 2>&1
timeout -k 5 200 python3 bench.py --no-cpu --no-secondary --steps 30 $2 > gpurun_out/base$i.log 2>&1
done
