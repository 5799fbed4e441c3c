#!/bin/bash
# For every variants/*/libblindno.so: the GPU tests selected by TESTK (parity of the variant),
# kbench over KFILTER and a short bench line; the in-tree library first as the baseline.
# usage (GPU box, repo root): bash tools/gpu_variants.sh TAG KFILTER "TESTK"
TAG=${1:-x}; KF=${2:-colpass}; TK=${3:-spectral}
mkdir -p gpurun_out
run() {  # name lib
  local v=$1 lib=$2
  BLINDNO_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "$TK" --timeout 120 --timeout-method thread > gpurun_out/vt_${TAG}_$v.log 2>&1 || { echo "tests failed for $v"; tail -30 gpurun_out/vt_${TAG}_$v.log; return 1; }
  echo "== $v tests: $(tail -1 gpurun_out/vt_${TAG}_$v.log)"
  BLINDNO_LIB=$lib timeout -k 10 120 python -u tools/kbench.py "$KF" 2>/dev/null | grep -v amdgpu.ids
  BLINDNO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu --no-parity --no-kernel-timer > gpurun_out/benchv_${TAG}_$v.json 2>/dev/null || { echo "bench failed for $v"; return 1; }
  echo "== $v bench: $(cut -c1-160 gpurun_out/benchv_${TAG}_$v.json | sed 's/.*"value": \([0-9.]*\).*"ms_per_step": \([0-9.]*\).*/\1 bags\/s \2 ms/')"
}
run base reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so || exit 1
for lib in variants/*/libblindno.so; do
  run $(basename $(dirname $lib)) $lib || exit 1
done
