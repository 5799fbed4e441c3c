#!/bin/bash
# One GPU iteration: parity tests, a bench line, a rocprofv3 kernel-trace profile.
# usage (on the GPU box, from the repo root): bash tools/gpu_cycle.sh TAG [bench args...]
TAG=${1:-x}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-700 gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?"
