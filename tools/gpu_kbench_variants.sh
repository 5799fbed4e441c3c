#!/bin/bash
# kbench over the in-tree library and every variants/*/libblindno.so (tools/build_variant.py).
# usage (GPU box, repo root): bash tools/gpu_kbench_variants.sh TAG FILTER
TAG=${1:-x}; FILT=${2:-input}
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/kbench.py "$FILT" > gpurun_out/kb_${TAG}_base.log 2>&1 || exit 1
echo "== base"; cat gpurun_out/kb_${TAG}_base.log
for lib in variants/*/libblindno.so; do
  v=$(basename $(dirname $lib))
  BLINDNO_LIB=$lib timeout -k 10 120 python -u tools/kbench.py "$FILT" > gpurun_out/kb_${TAG}_$v.log 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/kb_${TAG}_$v.log
done
