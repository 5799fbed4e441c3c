export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_ab_lib.sh "rowdft\[" rd_s2 rd_w2k rd_w2k_s1
