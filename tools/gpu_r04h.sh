#!/bin/bash
TAG=${1:-r04h}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_rowfuse.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graphs.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_kb_variants.sh "epi\[input|bwd_rd.*input|layer" nh2
bash tools/gpu_ab_lib.sh "" nh2
