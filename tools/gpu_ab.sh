#!/bin/bash
# A/B bench: the in-tree library against each variants/* library, alternated three times.
# usage (GPU box, repo root): bash tools/gpu_ab.sh
for i in 1 2 3; do
for v in base $(ls variants 2>/dev/null); do
  lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = base ] || lib=variants/$v/libblindno.so
  BLINDNO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 --no-cpu --no-parity --no-kernel-timer > gpurun_out/ab_$v$i.json 2>/dev/null || exit 1
  echo "$v $i $(python -c "import json;d=json.load(open('gpurun_out/ab_$v$i.json'));print(d['value'],d['ms_per_step'])")"
done; done
