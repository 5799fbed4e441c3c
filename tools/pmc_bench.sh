#!/bin/bash
# PMC passes over the benched step (bench.py CFG, graph replays), one counter group per run,
# restricted to kernels matching REGEX.   usage: bash tools/pmc_bench.sh TAG REGEX [CFG]
TAG=${1:-x}; RX=${2:-bagproj_fwd}; CFG=${3:-C}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcb_$TAG
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVES" "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmcb_$TAG/p$i -o run \
    -- python3 bench.py --config $CFG --steps 6 --warmup 2 --no-cpu --no-parity --timer-steps 2 > gpurun_out/pmcb_$TAG/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
