export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1; rc=$?; tail -1 gpurun_out/gpu_tests_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
