#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, as gfx950 requires).
# usage (GPU box, repo root): bash tools/pmc_passes.sh TAG
TAG=${1:-x}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
rocprofv3 -L > gpurun_out/pmc_$TAG/counters_list.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run \
    -- python3 bench.py --steps 3 --warmup 2 --no-cpu --no-kernel-timer > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
