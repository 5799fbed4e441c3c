#!/bin/bash
# tests + bench + rocprof, then kbench over the variant libraries for FILTER.
TAG=${1:-x}; FILT=${2:-project}
bash tools/gpu_cycle.sh $TAG || exit $?
bash tools/gpu_kbench_variants.sh $TAG "$FILT" > gpurun_out/kbv_$TAG.log 2>&1 || { echo "kbench variants failed"; tail -20 gpurun_out/kbv_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kbv_$TAG.log
for lib in variants/*/libblindno.so; do
  v=$(basename $(dirname $lib))
  BLINDNO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu --no-parity --no-kernel-timer > gpurun_out/benchv_${TAG}_$v.json 2>/dev/null || { echo "bench variant $v failed"; exit 1; }
  echo "== bench $v"; cut -c1-200 gpurun_out/benchv_${TAG}_$v.json
done
