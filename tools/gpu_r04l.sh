export TMPDIR=/tmp; mkdir -p gpurun_out
true
bash tools/gpu_ab_env.sh "colpass\[head" "-" "BLINDNO_LIB=variants/cf16/libblindno.so BLINDNO_COLFUSE_WAVES=16"
