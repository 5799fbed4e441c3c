#!/bin/bash
# round-4 profile evidence on the current tree: rocprofv3 kernel stats + step breakdown +
# timeline (config C), dominant-kernel check, config D kernel stats, PMC over the benched step
# (bagproj_fwd) and over kbench [input] (traffic per kernel)
TAG=${1:-r04j}
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_prof.sh $TAG C || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run2 \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof2_$TAG.log 2>&1 || { echo "rocprof 2 failed"; exit 1; }
python3 tools/trace_kernel_avg.py gpurun_out/prof_$TAG/run2_kernel_trace.csv bagproj_fwd 4 > gpurun_out/dominant_check_$TAG.txt 2>&1
cat gpurun_out/dominant_check_$TAG.txt; rm -f gpurun_out/prof_$TAG/run2_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profD_$TAG -o run \
  -- python3 bench.py --config D --steps 4 --warmup 2 --no-cpu --no-parity > gpurun_out/profD_$TAG.log 2>&1 || { echo "rocprof D failed"; exit 1; }
rm -f gpurun_out/profD_$TAG/run_kernel_trace.csv
head -14 gpurun_out/profD_$TAG/run_kernel_stats.csv | cut -c1-150
bash tools/pmc_bench.sh $TAG bagproj_fwd C || exit 1
python3 tools/pmc_bench.py gpurun_out/pmcb_$TAG bagproj_fwd 8 > gpurun_out/pmc_bench_bagproj_$TAG.json; cat gpurun_out/pmc_bench_bagproj_$TAG.json | head -30
bash tools/pmc_kbench.sh $TAG "\[input\]" || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmck_$TAG > gpurun_out/pmc_traffic_$TAG.json || exit 1
find gpurun_out/pmck_$TAG gpurun_out/pmcb_$TAG -name "*.csv" -size +8M -delete
echo done
