#!/bin/bash
# rocprofv3 kernel trace + stats of a config-C bench run; timeline of one graphed step
TAG=${1:-x}; CFG=${2:-C}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --config $CFG --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; echo "rocprof failed"; exit 1; }
python3 tools/step_breakdown.py gpurun_out/prof_$TAG/run_kernel_trace.csv 6 60 4 > gpurun_out/step_breakdown_$TAG.txt
python3 tools/timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv 6 > gpurun_out/timeline_$TAG.txt
head -40 gpurun_out/step_breakdown_$TAG.txt
tail -3 gpurun_out/timeline_$TAG.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv
