#!/bin/bash
# rowfuse ping-pong kbench (+ variants), config-D kernel profile, PMC of the encoder kernels.
TAG=${1:-x}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rowfuse.py tests/test_gpu_parity.py -k "rowfuse or rowinv or crop or fused" > gpurun_out/rowfuse_$TAG.log 2>&1
rc=$?; echo "rowfuse tests rc=$rc"; tail -2 gpurun_out/rowfuse_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_kb_variants_input.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profD_$TAG -o run \
  -- python3 bench.py --config D --steps 3 --warmup 2 --no-cpu --no-kernel-timer > gpurun_out/profD_$TAG.log 2>&1 || { echo "rocprof D failed"; tail -5 gpurun_out/profD_$TAG.log; exit 1; }
head -25 gpurun_out/profD_$TAG/run_kernel_stats.csv | cut -c1-220
rm -f gpurun_out/profD_$TAG/run_kernel_trace.csv
