set -e
for i in 1 2; do
for cfg in "2 512" "4 512" "2 1024" "4 1024" "4 2048"; do
  set -- $cfg
  SVO_CHAINS=$1 timeout -k 5 200 python3 bench.py --no-cpu --no-secondary --steps 20 --pairs $2 > gpurun_out/abp_c$1_p$2_$i.log 2>&1
done
done
