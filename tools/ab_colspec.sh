export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
for cs in 1 0; do
BLINDNO_COLSPEC=$cs timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);r=d.get('roofline_spectral',{});print('colspec=$cs bench', d['value'], d['ms_per_step'], 'spectral', r.get('frac'), r.get('ms_per_layer'))" || exit 1
done
done
