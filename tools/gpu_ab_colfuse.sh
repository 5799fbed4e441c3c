#!/bin/bash
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused_column" 2>&1 | tail -2
for i in 1 2; do
  timeout -k 10 120 python -u tools/kbench.py "colpass" 2>&1 | sed "s/^/fuse /"
  BLINDNO_COLFUSE=0 timeout -k 10 120 python -u tools/kbench.py "colpass" 2>&1 | sed "s/^/split /"
done
for i in 1 2; do
  for v in 1 0; do
    BLINDNO_COLFUSE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('colfuse=$v bench', d['value'], d['ms_per_step'], 'spectral', d['roofline_spectral']['frac'], d['roofline_spectral']['ms_per_layer'])"
  done
done
