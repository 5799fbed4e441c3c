#!/bin/bash
# Round-final GPU evidence: tests, bench line + rocprof stats, PMC passes over kbench "[input]".
# usage (GPU box, repo root): bash tools/gpu_final.sh TAG
TAG=${1:-x}
bash tools/gpu_cycle.sh $TAG || exit $?
bash tools/pmc_kbench.sh $TAG "input" || exit $?
timeout -k 10 120 python -u tools/kbench.py "head" > gpurun_out/kb_${TAG}_head.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/kb_${TAG}_head.log
