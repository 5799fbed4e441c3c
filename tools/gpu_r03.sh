#!/bin/bash
# Round-3 GPU iteration: new-kernel tests first, kernel A/B, the suite, bench lines, rocprof.
# usage (GPU box, repo root): bash tools/gpu_r03.sh TAG [kbench-filter]
TAG=${1:-x}; FILT=${2:-input}
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_rowfuse.py -s > gpurun_out/rowfuse_$TAG.log 2>&1
rc=$?; echo "rowfuse tests rc=$rc"; grep -E "rowfuse|passed|failed|Error" gpurun_out/rowfuse_$TAG.log | tail -20
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  BLINDNO_ROWFUSE=$v timeout -k 10 200 python -u tools/kbench.py "$FILT" > gpurun_out/kb_${TAG}_$v.log 2>&1 || { echo "kbench $v failed"; tail -5 gpurun_out/kb_${TAG}_$v.log; exit 1; }
  echo "== kbench ROWFUSE=$v"; grep -v amdgpu.ids gpurun_out/kb_${TAG}_$v.log
done
timeout -k 10 500 $PYT tests -m gpu > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_$TAG.json
BLINDNO_ROWFUSE=0 timeout -k 10 300 python -u bench.py --no-cpu --no-parity > gpurun_out/bench_${TAG}_nofuse.json 2> gpurun_out/bench_${TAG}_nofuse.err || { tail -5 gpurun_out/bench_${TAG}_nofuse.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_nofuse.json
timeout -k 10 400 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_D.json 2> gpurun_out/bench_${TAG}_D.err || { tail -5 gpurun_out/bench_${TAG}_D.err; exit 1; }
cut -c1-400 gpurun_out/bench_${TAG}_D.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?"
