export TMPDIR=/tmp; mkdir -p gpurun_out
BLINDNO_LIB=variants/sc12/libblindno.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 250 --timeout-method thread -x -k "bag_stats or dedup" > gpurun_out/t_sc.log 2>&1; rc=$?; tail -1 gpurun_out/t_sc.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh "project_bag_fwd\[u52" sc4 sc12 sc16
