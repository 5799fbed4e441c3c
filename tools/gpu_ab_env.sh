#!/bin/bash
# A/B of environment settings in the config-C step (and an optional kbench filter):
#   bash tools/gpu_ab_env.sh "kbench-regex" "ENV=a" "ENV=b" ...   ("-" = no extra setting)
export TMPDIR=/tmp; mkdir -p gpurun_out
KB=$1; shift
if [ -n "$KB" ]; then
for i in 1 2; do
  for v in "$@"; do
    e=$v; [ "$e" = "-" ] && e="BLINDNO_AB_NONE=1"
    env $e timeout -k 10 120 python -u tools/kbench.py "$KB" 2>&1 | sed "s|^|$v |" || exit 1
  done
done
fi
for i in 1 2 3; do
  for v in "$@"; do
    e=$v; [ "$e" = "-" ] && e="BLINDNO_AB_NONE=1"
    env $e timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('$v bench', d['value'], d['ms_per_step'], 'spectral', d['roofline_spectral']['frac'])" || exit 1
  done
done
