export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_trunk_graph.py 13 > gpurun_out/diag_tg.log 2>&1; rc=$?; grep -v "amdgpu.ids\|Warning\|warn" gpurun_out/diag_tg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_configs.py -m gpu -x -q --timeout 250 --timeout-method thread -k "bn_act or config_d or linear or ffn or deeponet" > gpurun_out/t_bn.log 2>&1; rc=$?; tail -3 gpurun_out/t_bn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config D --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_dpar_D.json 2> gpurun_out/bench_dpar_D.err || { tail -5 gpurun_out/bench_dpar_D.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_dpar_D.json').read().strip().splitlines()[-1]);p=d['parity'];print(d['value'], json.dumps(p['gpu_vs_fp64']), json.dumps(p['trunk_stage']), json.dumps(p['grads_worst_full_chain']), p['pass'])"
