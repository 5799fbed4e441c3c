#!/bin/bash
# the libblindno NIO path (linear / FFN trunk / DeepONet bag), its graphed step and the poison diag
TAG=${1:-r04b}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_encoder.py tests/test_gpu_graphs.py::test_graphed_nio_step_matches_eager \
  tests/test_gpu_configs.py::test_config_d_graphed_niofp2d_nc_128 tests/test_gpu_configs.py::test_config_d_niofp2d_nc_128 \
  tests/test_gpu_evaluators.py tests/test_gpu_trainer.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "graphed D|FAIL|Error|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/diag_graph_d.py 128 shared poison
