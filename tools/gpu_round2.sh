#!/bin/bash
# tests + bench + rocprof, then kbench over the variant libraries for FILTER.
TAG=${1:-x}; FILT=${2:-project}
bash tools/gpu_cycle.sh $TAG || exit $?
bash tools/gpu_kbench_variants.sh $TAG "$FILT" > gpurun_out/kbv_$TAG.log 2>&1 || { echo "kbench variants failed"; tail -20 gpurun_out/kbv_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kbv_$TAG.log
