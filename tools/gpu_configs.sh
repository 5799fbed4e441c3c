#!/bin/bash
# Bench line of every secondary config (1 x MI355X): usage bash tools/gpu_configs.sh TAG
TAG=${1:-x}
export TMPDIR=/tmp; mkdir -p gpurun_out
for c in A B C_attn U U_NC U1; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-parity --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  echo "$c $(python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$c.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
