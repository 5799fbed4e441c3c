export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -m gpu -q --timeout 250 --timeout-method thread -x -k batch_select > gpurun_out/t_bsel.log 2>&1; rc=$?; tail -2 gpurun_out/t_bsel.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04v -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof_r04v.log 2>&1 || exit 1
python3 tools/step_breakdown.py gpurun_out/prof_r04v/run_kernel_trace.csv 6 60 4 > gpurun_out/step_breakdown_r04v.txt; head -2 gpurun_out/step_breakdown_r04v.txt; grep -i "gather\|index\|copy" gpurun_out/step_breakdown_r04v.txt
rm -f gpurun_out/prof_r04v/run_kernel_trace.csv
