#!/bin/bash
# round-4 verification: GPU suite, smoke, bench lines C (parity + cpu baseline), D (parity), E
TAG=${1:-x}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests_$TAG.log; grep FAILED gpurun_out/gpu_tests_$TAG.log | tail -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/bench_$TAG.json
for c in D E; do
  timeout -k 10 500 python -u bench.py --config $c --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cut -c1-200 gpurun_out/bench_${TAG}_$c.json
done
