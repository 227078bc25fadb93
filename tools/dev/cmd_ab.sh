# A/B of measurement knobs on one box: bench value per variant (core-only, no CPU / secondary legs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary --core-only > gpurun_out/ab_$tag.log 2>&1 || return 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/ab_$tag.log') if l.startswith('{')][0]; print('$tag', d['value'], d['ms_per_step'], 'pyr', d['pyramid_build']['ms'], d['pyramid_build']['frac_hbm_peak'], 'e2e', d['end_to_end_device_images']['ms'])"
}
for v in "$@"; do
  tag=${v%%:*}; envs=${v#*:}
  run $tag $envs || exit 1
done
