#!/bin/bash
TAG=${1:-x}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "bag or dedup" > gpurun_out/bag_$TAG.log 2>&1
rc=$?; echo "bag tests rc=$rc"; tail -2 gpurun_out/bag_$TAG.log; [ $rc -eq 0 ] || exit $rc
F="project_bag"
timeout -k 10 200 python -u tools/kbench.py "$F" 2>/dev/null | grep input || exit 1
for lib in variants/*/libblindno.so; do
  v=$(basename $(dirname $lib)); echo "== $v"
  BLINDNO_LIB=$lib timeout -k 10 200 python -u tools/kbench.py "$F" 2>/dev/null | grep input || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu --no-parity > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/bench_$TAG.json
BLINDNO_LIB=variants/oldv/libblindno.so timeout -k 10 300 python -u bench.py --no-cpu --no-parity > gpurun_out/bench_${TAG}_old.json 2> gpurun_out/bench_${TAG}_old.err || { tail -5 gpurun_out/bench_${TAG}_old.err; exit 1; }
cut -c1-200 gpurun_out/bench_${TAG}_old.json
