#!/bin/bash
TAG=${1:-r04c}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_graphs.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_D.json 2> gpurun_out/bench_${TAG}_D.err || { tail -5 gpurun_out/bench_${TAG}_D.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_D.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
