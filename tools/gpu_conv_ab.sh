#!/bin/bash
# Config-D conv A/B: conv GPU tests, per-layer kbench (in-tree and each variant), then the
# config-D bench line (in-tree vs variants/*).  usage: bash tools/gpu_conv_ab.sh TAG [pytest -k expr]
TAG=${1:-x}; K=${2:-"conv2d or encoder or config_d"}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/conv_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/conv_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kbench_conv.py > gpurun_out/kbconv_${TAG}_base.log 2>&1 || exit 1
cat gpurun_out/kbconv_${TAG}_base.log
for lib in variants/*/libblindno.so; do
  v=$(basename $(dirname $lib))
  BLINDNO_LIB=$lib timeout -k 10 200 python -u tools/kbench_conv.py > gpurun_out/kbconv_${TAG}_$v.log 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/kbconv_${TAG}_$v.log
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config D --no-cpu --no-parity --steps 6 --warmup 2 > gpurun_out/abD_${TAG}_base_$rep.json 2>/dev/null || exit 1
  echo "base $rep $(python3 -c "import json;d=json.loads(open('gpurun_out/abD_${TAG}_base_$rep.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])")"
  for lib in variants/*/libblindno.so; do
    v=$(basename $(dirname $lib))
    BLINDNO_LIB=$lib timeout -k 10 300 python -u bench.py --config D --no-cpu --no-parity --steps 6 --warmup 2 > gpurun_out/abD_${TAG}_${v}_$rep.json 2>/dev/null || exit 1
    echo "$v $rep $(python3 -c "import json;d=json.loads(open('gpurun_out/abD_${TAG}_${v}_$rep.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])")"
  done
done
