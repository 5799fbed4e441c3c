export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_encoder.py -m gpu -q --timeout 250 --timeout-method thread -x -k "config_d or ffn or trunk" > gpurun_out/t_tm.log 2>&1; rc=$?; tail -2 gpurun_out/t_tm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_r04y_D.json 2> gpurun_out/bench_r04y_D.err || { tail -5 gpurun_out/bench_r04y_D.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_r04y_D.json').read().strip().splitlines()[-1]);p=d['parity'];print(d['value'], p['pass'], json.dumps(p['gpu_vs_fp64']), json.dumps(p['trunk_branch_flips']), json.dumps(p['trunk_stage']))"
