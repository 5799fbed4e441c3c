#!/bin/bash
TAG=${1:-r04f}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graphs.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -20; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python -u tools/kbench.py "colpass|layer" 2>&1 | sed "s/^/fuse /"
  BLINDNO_COLFUSE=0 timeout -k 10 120 python -u tools/kbench.py "colpass|layer" 2>&1 | sed "s/^/split /"
done
for i in 1 2; do
  for v in 1 0; do
    BLINDNO_COLFUSE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('colfuse=$v bench', d['value'], d['ms_per_step'], 'spectral', d['roofline_spectral']['frac'], d['roofline_spectral']['ms_per_layer'])"
  done
done
