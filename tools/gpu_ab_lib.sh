#!/bin/bash
# A/B of library variants in the config-C step (and an optional kbench filter): bash tools/gpu_ab_lib.sh "kbench-regex" var1 var2 ...
export TMPDIR=/tmp; mkdir -p gpurun_out
KB=$1; shift
if [ -n "$KB" ]; then
for i in 1 2; do
  for v in cur $@; do
    lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
    BLINDNO_LIB=$lib timeout -k 10 120 python -u tools/kbench.py "$KB" 2>&1 | sed "s/^/$v /"
  done
done
fi
for i in 1 2 3; do
  for v in cur $@; do
    lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
    BLINDNO_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('$v bench', d['value'], d['ms_per_step'], 'spectral', d['roofline_spectral']['frac'], d['roofline_spectral']['ms_per_layer'])"
  done
done
