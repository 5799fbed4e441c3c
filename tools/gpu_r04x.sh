export TMPDIR=/tmp; mkdir -p gpurun_out
BLINDNO_LIB=variants/rega/libblindno.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 250 --timeout-method thread -x > gpurun_out/t_rega.log 2>&1; rc=$?; tail -2 gpurun_out/t_rega.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh "project_bwd\[head" dzm rega
