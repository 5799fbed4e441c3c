set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcconv
timeout -k 10 200 python3 tools/kbench_conv.py 300 > gpurun_out/kbench_conv_r06c.txt 2>&1
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD" "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcconv/p$i -o run \
    -- python3 tools/kbench_conv.py 300 "cb2_2|cb3_2|cb4_2|cb3_1" > gpurun_out/pmcconv/p$i.log 2>&1
  echo "pass $i rc=$?"
done
