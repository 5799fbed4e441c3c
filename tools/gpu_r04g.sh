#!/bin/bash
TAG=${1:-r04g}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_rowfuse.py tests/test_gpu_parity.py tests/test_gpu_configs.py::test_config_c_niofp2d_fno_128 tests/test_gpu_graphs.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in rf_pk rf_pk_nopf; do
  BLINDNO_LIB=variants/$v/libblindno.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rowfuse.py tests/test_gpu_configs.py::test_config_c_niofp2d_fno_128 2>&1 | tail -1 | sed "s/^/$v tests: /"
done
bash tools/gpu_kb_variants.sh "epi.*input|bwd.*input|project_bag" rf_pk rf_pk_nopf rf_nopf rf_nogelu rf_nord
bash tools/gpu_ab_lib.sh "" rf_pk rf_pk_nopf
