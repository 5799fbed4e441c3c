#!/bin/bash
# A/B of conv variants on one box: tools/kbench_conv.py under the in-tree library and under
# variants/<v>/libblindno.so, alternated.   usage: bash tools/ab_conv.sh TAG VARIANT [MODE-REGEX]
TAG=$1; V=$2; MODE=${3:-}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in cur $V; do
    lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so
    [ $v = cur ] || lib=variants/$v/libblindno.so
    echo "== $v (rep $rep)"
    BLINDNO_LIB=$lib timeout -k 10 200 python3 tools/kbench_conv.py 300 "" "$MODE" 2>/dev/null || exit 1
  done
done 2>&1 | tee gpurun_out/ab_conv_$TAG.txt
