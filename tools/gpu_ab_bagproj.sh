#!/bin/bash
# A/B of bagproj forward variants: kbench (U = 75 and 52) and the config-C bench, alternated
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "bag or dedup" 2>&1 | tail -2
for i in 1 2; do
  for v in cur $@; do
    lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
    BLINDNO_LIB=$lib timeout -k 10 120 python -u tools/kbench.py "project_bag_fwd" 2>&1 | sed "s/^/$v /"
  done
done
for i in 1 2; do
  for v in cur $@; do
    lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
    BLINDNO_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('$v bench', d['value'], d['ms_per_step'], 'bagproj_fwd', d['roofline']['avg_ms'])"
  done
done
