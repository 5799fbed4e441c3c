export TMPDIR=/tmp; mkdir -p gpurun_out
F="rowidft|layer"
timeout -k 10 200 python -u tools/kbench.py "$F" 2>/dev/null | grep input > gpurun_out/kbv_base.log || exit 1
echo "== base (b512 zpre)"; cat gpurun_out/kbv_base.log
for lib in variants/*/libblindno.so; do
  v=$(basename $(dirname $lib))
  BLINDNO_LIB=$lib timeout -k 10 200 python -u tools/kbench.py "$F" 2>/dev/null | grep input > gpurun_out/kbv_$v.log || exit 1
  echo "== $v"; cat gpurun_out/kbv_$v.log
done
