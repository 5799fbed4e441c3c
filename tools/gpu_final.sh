#!/bin/bash
# Round-end evidence on the current tree: GPU suite, smoke, bench lines (C with parity + CPU
# baseline, D, E), rocprofv3 kernel stats + step breakdown, PMC passes over kbench [input].
# usage (GPU box, repo root): bash tools/gpu_final.sh TAG
TAG=${1:-x}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -s > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
for c in D E; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cut -c1-200 gpurun_out/bench_${TAG}_$c.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
cp gpurun_out/prof_$TAG.log gpurun_out/prof_bench_line_$TAG.json
python3 tools/step_breakdown.py gpurun_out/prof_$TAG/run_kernel_trace.csv 8 45 4 > gpurun_out/step_breakdown_$TAG.txt
head -30 gpurun_out/step_breakdown_$TAG.txt
python3 tools/trace_kernel_avg.py gpurun_out/prof_$TAG/run_kernel_trace.csv bagproj_fwd 4 > gpurun_out/dominant_check_$TAG.txt 2>&1 || true
cat gpurun_out/dominant_check_$TAG.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profD_$TAG -o run \
  -- python3 bench.py --config D --steps 4 --warmup 2 --no-cpu --no-parity > gpurun_out/profD_$TAG.log 2>&1 || { echo "rocprof D failed"; exit 1; }
rm -f gpurun_out/profD_$TAG/run_kernel_trace.csv
head -12 gpurun_out/profD_$TAG/run_kernel_stats.csv | cut -c1-160
bash tools/pmc_kbench.sh $TAG "\[input\]" || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmck_$TAG > gpurun_out/pmc_traffic_$TAG.json || exit 1
find gpurun_out/pmck_$TAG -name "*.csv" -size +8M -delete
echo done
