#!/bin/bash
# round 4 first call: the new config-D graph tests, the nio trainer test, bench C and D lines
TAG=${1:-r04a}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_graphs.py tests/test_gpu_configs.py::test_config_d_graphed_niofp2d_nc_128 \
  tests/test_gpu_trainer.py::test_trainer_nio_2d > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "graphed D|PASS|FAIL|Error|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
timeout -k 10 500 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_D.json 2> gpurun_out/bench_${TAG}_D.err || { tail -5 gpurun_out/bench_${TAG}_D.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_D.json
