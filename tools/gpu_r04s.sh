export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profE_r04s -o run \
  -- python3 bench.py --config E --steps 6 --warmup 2 --no-cpu --no-parity > gpurun_out/profE_r04s.log 2>&1 || { tail -5 gpurun_out/profE_r04s.log; exit 1; }
python3 tools/step_breakdown.py gpurun_out/profE_r04s/run_kernel_trace.csv 4 60 4 > gpurun_out/step_breakdown_E_r04s.txt
head -45 gpurun_out/step_breakdown_E_r04s.txt
rm -f gpurun_out/profE_r04s/run_kernel_trace.csv
