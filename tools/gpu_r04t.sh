export TMPDIR=/tmp; mkdir -p gpurun_out
BLINDNO_LIB=variants/cf16/libblindno.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v --timeout 250 --timeout-method thread -s -k "fused_column or config_e or fp16 or mix16 or 256" > gpurun_out/t_cf16.log 2>&1; rc=$?; grep -E "passed|failed|fp16 mix|PASS|FAIL" gpurun_out/t_cf16.log | tail -20; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
for v in cur cf16; do
  lib=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so; [ $v = cur ] || lib=variants/$v/libblindno.so
  BLINDNO_LIB=$lib timeout -k 10 400 python -u bench.py --config E --no-cpu --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);p=d.get('parity',{});print('$v E', d['value'], d['ms_per_step'], 'pass', p.get('pass'), p.get('gpu_vs_fp64',{}).get('fwd'), p.get('gpu_vs_fp64',{}).get('grad_max'))" || exit 1
done
done
