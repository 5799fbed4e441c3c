#!/bin/bash
# kbench only, library variants alternated: bash tools/gpu_kb_variants.sh "regex" var1 var2 ...
export TMPDIR=/tmp; mkdir -p gpurun_out
KB=$1; shift
for i in 1 2; do
  for v in cur $@; do
    lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
    BLINDNO_LIB=$lib timeout -k 10 120 python -u tools/kbench.py "$KB" 2>&1 | sed "s/^/$v /"
  done
done
