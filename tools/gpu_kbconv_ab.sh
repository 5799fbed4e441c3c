#!/bin/bash
# per-layer conv kbench, in-tree library then each variants/*: usage bash tools/gpu_kbconv_ab.sh TAG [layer-regex] [mode-regex] [pytest -k]
TAG=${1:-x}; L=${2:-}; M=${3:-}; K=${4:-}
export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/kbab_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/kbab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  echo "== base $rep"; timeout -k 10 200 python -u tools/kbench_conv.py 300 "$L" "$M" 2>/dev/null | grep -v amdgpu.ids || exit 1
  for lib in variants/*/libblindno.so; do
    v=$(basename $(dirname $lib))
    echo "== $v $rep"; BLINDNO_LIB=$lib timeout -k 10 200 python -u tools/kbench_conv.py 300 "$L" "$M" 2>/dev/null | grep -v amdgpu.ids || exit 1
  done
done
