#!/bin/bash
# One GPU iteration: parity tests, a bench line, a rocprofv3 kernel-trace profile.
# usage (on the GPU box, from the repo root): bash tools/gpu_cycle.sh TAG
TAG=${1:-x}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?"
cut -c1-250 gpurun_out/bench_$TAG.json
