export TMPDIR=/tmp; mkdir -p gpurun_out
BLINDNO_LIB=variants/dzm/libblindno.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graphs.py -m gpu -q --timeout 250 --timeout-method thread -x > gpurun_out/t_dzm.log 2>&1; rc=$?; tail -2 gpurun_out/t_dzm.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh "project_bwd\[head" dzm
for i in 1 2; do
for v in cur dzm; do
  lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
  BLINDNO_LIB=$lib timeout -k 10 400 python -u bench.py --config E --no-cpu --no-parity --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('$v E', d['value'], d['ms_per_step'])" || exit 1
done
done
