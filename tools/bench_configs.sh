#!/bin/bash
# Bench BASELINE.json configs once each (C = the headline line).
# usage: bash tools/bench_configs.sh TAG [configs...]   (default: A B C D E)
TAG=${1:-x}
shift
CONFIGS=${@:-A B C D E}
mkdir -p gpurun_out
for c in $CONFIGS; do
  timeout -k 10 500 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu \
    > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "config $c failed"; tail -20 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  echo "== $c"; cut -c1-400 gpurun_out/bench_${TAG}_$c.json
done
