#!/bin/bash
# round-4 final evidence: GPU suite, smoke, bench C (parity + cpu baseline) / D / E, rocprofv3
# stats + step breakdown + timeline (C), dominant-kernel check, PMC over the benched step
TAG=${1:-r04z}
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_verify4.sh $TAG || exit 1
bash tools/gpu_prof.sh $TAG C || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run2 \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof2_$TAG.log 2>&1 || { echo "rocprof 2 failed"; exit 1; }
python3 tools/trace_kernel_avg.py gpurun_out/prof_$TAG/run2_kernel_trace.csv bagproj_fwd 4 > gpurun_out/dominant_check_$TAG.txt 2>&1
cat gpurun_out/dominant_check_$TAG.txt; rm -f gpurun_out/prof_$TAG/run2_kernel_trace.csv
bash tools/pmc_bench.sh $TAG bagproj_fwd C || exit 1
python3 tools/pmc_bench.py gpurun_out/pmcb_$TAG bagproj_fwd 8 > gpurun_out/pmc_bench_bagproj_$TAG.json; grep valu_issue gpurun_out/pmc_bench_bagproj_$TAG.json
find gpurun_out/pmcb_$TAG -name "*.csv" -size +8M -delete
echo done
