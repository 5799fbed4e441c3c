export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/pmc_kbench.sh r04n "head2" || exit 1
python3 tools/pmc_summary.py gpurun_out/pmck_r04n > gpurun_out/pmc_head2_r04n.txt 2>&1
find gpurun_out/pmck_r04n -name "*.csv" -size +8M -delete
cat gpurun_out/pmc_head2_r04n.txt | grep -v "vectorized_elem\|rocclr\|Fill" | head -40
