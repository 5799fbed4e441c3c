#!/bin/bash
# rowfuse: correctness tests, kbench of the in-tree lib (ROWFUSE on/off) and every variant,
# then quick bench lines (fused vs general kernel).  usage: bash tools/gpu_ab_rowfuse.sh TAG
TAG=${1:-x}; FILT=${2:-rowidft|layer}
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_rowfuse.py tests/test_gpu_parity.py -s -k "rowfuse or rowinv or crop or fused" > gpurun_out/rowfuse_$TAG.log 2>&1
rc=$?; echo "rowfuse tests rc=$rc"; grep -E "rowfuse|passed|failed|Error" gpurun_out/rowfuse_$TAG.log | tail -14
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  BLINDNO_ROWFUSE=$v timeout -k 10 200 python -u tools/kbench.py "$FILT" > gpurun_out/kb_${TAG}_$v.log 2>&1 || { echo "kbench $v failed"; tail -5 gpurun_out/kb_${TAG}_$v.log; exit 1; }
  echo "== ROWFUSE=$v"; grep -v amdgpu.ids gpurun_out/kb_${TAG}_$v.log
done
for lib in variants/*/libblindno.so; do
  vn=$(basename $(dirname $lib))
  BLINDNO_LIB=$lib timeout -k 10 200 python -u tools/kbench.py "$FILT" > gpurun_out/kb_${TAG}_$vn.log 2>&1 || { echo "kbench $vn failed"; exit 1; }
  echo "== $vn"; grep -v amdgpu.ids gpurun_out/kb_${TAG}_$vn.log
done
for v in 1 0; do
  BLINDNO_ROWFUSE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-parity > gpurun_out/bench_${TAG}_f$v.json 2> gpurun_out/bench_${TAG}_f$v.err || { tail -5 gpurun_out/bench_${TAG}_f$v.err; exit 1; }
  echo "== bench ROWFUSE=$v"; cut -c1-200 gpurun_out/bench_${TAG}_f$v.json
done
