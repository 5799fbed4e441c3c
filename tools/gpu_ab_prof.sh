#!/bin/bash
# Per-step kernel breakdown (tools/step_breakdown.py) of bench.py for the in-tree library and
# each variants/* library.  usage (GPU box, repo root): bash tools/gpu_ab_prof.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base $(ls variants); do
  lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = base ] || lib=variants/$v/libblindno.so
  BLINDNO_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abp_$v -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu --no-parity --no-kernel-timer > gpurun_out/abp_$v.json 2>gpurun_out/abp_$v.err || exit 1
done
for v in base $(ls variants); do
  python3 tools/step_breakdown.py $(ls gpurun_out/abp_$v/run_kernel_trace.csv gpurun_out/abp_$v/*/run_kernel_trace.csv 2>/dev/null | head -1) 6 16 0 > gpurun_out/abp_$v.txt
  rm -rf gpurun_out/abp_$v
done
