export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 250 --timeout-method thread -x > gpurun_out/t_cf8.log 2>&1; rc=$?; tail -2 gpurun_out/t_cf8.log; [ $rc -eq 0 ] || exit $rc
BLINDNO_COLFUSE_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 250 --timeout-method thread -x -k "colpass or column or fused" > gpurun_out/t_cf8b.log 2>&1; rc=$?; tail -2 gpurun_out/t_cf8b.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh "colpass\[head" "BLINDNO_COLFUSE_WAVES=4" "-"
