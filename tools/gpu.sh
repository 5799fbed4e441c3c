#!/bin/bash
# The one launcher for GPU-box work (run under gpurun from the repo root):
#     bash tools/gpu.sh TAG STEP [STEP ...]
# every step writes gpurun_out/<step>_<TAG>[_<i>].* and runs under its own time limit; the script
# stops at the first failing step (no retries).  Steps:
#   tests[:EXPR]      pytest -m gpu (optionally -k EXPR; "tests:file=tests/x.py" for one file)
#   smoke             __graft_entry__.smoke()
#   bench[:CFG]       bench.py --config CFG (default C, with parity + cpu baseline)
#   benchq[:CFG]      bench.py --config CFG --no-cpu --steps 10 --warmup 3 (parity kept)
#   prof[:CFG]        rocprofv3 kernel trace + stats of a bench run, step breakdown, timeline
#   kbench:REGEX      tools/kbench.py REGEX (per-kernel timing at Bn = 300)
#   ab:VARS[:REGEX]   A/B of library variants (variants/<v>/libblindno.so, comma separated)
#                     against the in-tree library: 3 alternations of the config-C bench
#   abenv:VAR=a,b     the config-C bench under VAR=a, VAR=b, ... (3 alternations), e.g.
#                     abenv:BLINDNO_BENCH_BACKEND=nccl,gloo (any environment variable bench.py reads)
#   pmc:KERNEL        PMC counters over the benched step for KERNEL (tools/pmc_bench.sh)
#   pmck:REGEX        PMC HBM traffic of kbench kernels (tools/pmc_kbench.sh -> pmc_traffic)
# Index of the round-by-round evidence these produce: DESIGN.md section 8.
TAG=${1:?tag}; shift
export TMPDIR=/tmp; mkdir -p gpurun_out
LIB=reconstruction-of-pde-without-time-label_amd/blindno/libblindno.so
i=0
for step in "$@"; do
  i=$((i+1))
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "== $name $arg"
  case $name in
    tests)
      sel=(tests); kx=()
      if [[ $arg == file=* ]]; then sel=(${arg#file=}); elif [ -n "$arg" ]; then kx=(-k "$arg"); fi
      timeout -k 10 900 python -u -m pytest "${sel[@]}" -m gpu -v --timeout 300 --timeout-method thread -s "${kx[@]}" \
        > gpurun_out/tests_${TAG}_$i.log 2>&1
      rc=$?; tail -2 gpurun_out/tests_${TAG}_$i.log; grep -E "FAILED|Error" gpurun_out/tests_${TAG}_$i.log | tail -8
      [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
        || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
      tail -1 gpurun_out/smoke_$TAG.log ;;
    bench|benchq)
      cfg=${arg:-C}; extra=(); [ $name = benchq ] && extra=(--no-cpu --steps 10 --warmup 3)
      timeout -k 10 600 python -u bench.py --config $cfg "${extra[@]}" > gpurun_out/bench_${TAG}_$cfg.json \
        2> gpurun_out/bench_${TAG}_$cfg.err || { tail -5 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
      cut -c1-300 gpurun_out/bench_${TAG}_$cfg.json ;;
    prof)
      cfg=${arg:-C}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
        -- python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/prof_$TAG.log 2>&1 \
        || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
      python3 tools/step_breakdown.py gpurun_out/prof_$TAG/run_kernel_trace.csv 6 60 4 > gpurun_out/step_breakdown_$TAG.txt
      python3 tools/timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv 6 > gpurun_out/timeline_$TAG.txt
      python3 tools/trace_kernel_avg.py gpurun_out/prof_$TAG/run_kernel_trace.csv bagproj_fwd 4 \
        > gpurun_out/dominant_check_$TAG.txt 2>&1
      head -45 gpurun_out/step_breakdown_$TAG.txt
      rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv ;;
    kbench)
      timeout -k 10 300 python -u tools/kbench.py "$arg" > gpurun_out/kbench_$TAG.txt 2>&1 \
        || { tail -5 gpurun_out/kbench_$TAG.txt; exit 1; }
      cat gpurun_out/kbench_$TAG.txt ;;
    ab)
      vars=${arg%%:*}; kb=${arg#*:}; [ "$kb" = "$arg" ] && kb=""
      for rep in 1 2 3; do
        for v in cur ${vars//,/ }; do
          lib=$LIB; [ $v = cur ] || lib=variants/$v/libblindno.so
          if [ -n "$kb" ] && [ $rep -le 2 ]; then
            BLINDNO_LIB=$lib timeout -k 10 200 python -u tools/kbench.py "$kb" 2>&1 | sed "s/^/$v /"
          fi
          BLINDNO_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c \
            "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);r=d.get('roofline_spectral',{});print('$v bench', d['value'], d['ms_per_step'], 'spectral', r.get('frac'), r.get('ms_per_layer'))" \
            || exit 1
        done
      done 2>&1 | tee gpurun_out/ab_$TAG.txt ;;
    abenv)
      var=${arg%%=*}; vals=${arg#*=}
      for rep in 1 2 3; do
        for val in ${vals//,/ }; do
          env $var=$val timeout -k 10 300 python -u bench.py --no-cpu --no-parity 2>/dev/null | python3 -c \
            "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);r=d.get('roofline_spectral',{});print('$var=$val bench', d['value'], d['ms_per_step'], 'spectral', r.get('frac'), r.get('ms_per_layer'))" \
            || exit 1
        done
      done 2>&1 | tee gpurun_out/abenv_$TAG.txt ;;
    pmc)
      bash tools/pmc_bench.sh $TAG "$arg" C || exit 1
      python3 tools/pmc_bench.py gpurun_out/pmcb_$TAG "$arg" 8 > gpurun_out/pmc_bench_$TAG.json
      find gpurun_out/pmcb_$TAG -name "*.csv" -size +8M -delete
      cat gpurun_out/pmc_bench_$TAG.json ;;
    pmck)
      bash tools/pmc_kbench.sh $TAG "$arg" || exit 1 ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG done"
