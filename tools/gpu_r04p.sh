export TMPDIR=/tmp; mkdir -p gpurun_out
BLINDNO_LIB=variants/pbw/libblindno.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 250 --timeout-method thread -x -k "project or head or grouped" > gpurun_out/t_pbw.log 2>&1; rc=$?; tail -2 gpurun_out/t_pbw.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_ab_lib.sh "project_bwd\[head" pbw pbwu2
