# A/B of environment settings on one box: tools/ab_env.sh "<env A>" "<env B>" ... (two alternating rounds)
set -e
for i in 1 2; do
  j=0
  for e in "$@"; do
    j=$((j+1))
    env $e timeout -k 5 200 python3 bench.py --no-cpu --no-secondary --steps 30 > gpurun_out/env${j}_$i.log 2>&1
  done
done
