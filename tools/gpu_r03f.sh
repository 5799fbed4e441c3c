#!/bin/bash
# step breakdowns fused / general, copy calibration, config D graphed, GPU suite.
TAG=${1:-x}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kbench.py "copy|rowidft|layer|rowdft|colpass" > gpurun_out/kb_$TAG.log 2>&1 || { tail -5 gpurun_out/kb_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kb_$TAG.log
for v in 1 0; do
  BLINDNO_ROWFUSE=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${TAG}_f$v -o run \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-parity --no-kernel-timer > gpurun_out/prof_${TAG}_f$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 gpurun_out/prof_${TAG}_f$v.log; exit 1; }
  echo "== ROWFUSE=$v"; python3 tools/step_breakdown.py gpurun_out/prof_${TAG}_f$v/run_kernel_trace.csv 8 22
done
timeout -k 10 400 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_D.json 2> gpurun_out/bench_${TAG}_D.err || { tail -5 gpurun_out/bench_${TAG}_D.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_D.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests_$TAG.log
