#!/bin/bash
TAG=${1:-r04c}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_graphs.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_D.json 2> gpurun_out/bench_${TAG}_D.err || { tail -5 gpurun_out/bench_${TAG}_D.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_D.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
BLINDNO_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu --no-parity > gpurun_out/bench_${TAG}_n2gloo.json 2> gpurun_out/bench_${TAG}_n2gloo.err || { tail -5 gpurun_out/bench_${TAG}_n2gloo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_n2gloo.json').read().strip().splitlines()[-1]);print({k:d['dist'][k] for k in ('params_identical_across_ranks','params_max_abs_diff_vs_rank0','bag_ids_per_rank')})"
