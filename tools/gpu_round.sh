#!/bin/bash
# Full GPU iteration: tests, bench line, rocprof profile, kbench variants, PMC passes.
# usage (GPU box, repo root): bash tools/gpu_round.sh TAG
TAG=${1:-x}
bash tools/gpu_cycle.sh $TAG || exit $?
bash tools/gpu_kbench_variants.sh $TAG "input" > gpurun_out/kbv_$TAG.log 2>&1 || { echo "kbench variants failed"; tail -20 gpurun_out/kbv_$TAG.log; exit 1; }
echo "kbench variants ok"
bash tools/pmc_kbench.sh $TAG "input" || exit $?
echo "pmc ok"
