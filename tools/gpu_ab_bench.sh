#!/bin/bash
# A/B of variant libraries (variants/*/libblindno.so) against the in-tree one on the bench line,
# alternating twice; plus an optional pytest selection first.  usage: bash tools/gpu_ab_bench.sh TAG [pytest -k expr]
TAG=${1:-x}; K=${2:-}
export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-parity --no-kernel-timer > gpurun_out/ab_${TAG}_base_$rep.json 2>/dev/null || exit 1
  echo "base $rep $(python3 -c "import json;d=json.loads(open('gpurun_out/ab_${TAG}_base_$rep.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  for lib in variants/*/libblindno.so; do
    v=$(basename $(dirname $lib))
    BLINDNO_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-parity --no-kernel-timer > gpurun_out/ab_${TAG}_${v}_$rep.json 2>/dev/null || exit 1
    echo "$v $rep $(python3 -c "import json;d=json.loads(open('gpurun_out/ab_${TAG}_${v}_$rep.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  done
done
