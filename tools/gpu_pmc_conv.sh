#!/bin/bash
# SQ counters of one config-D conv layer / mode (tools/kbench_conv.py filters), in-tree library
# and each variants/*: usage bash tools/gpu_pmc_conv.sh TAG LAYER MODE
TAG=${1:-x}; L=${2:-cb2_2}; M=${3:-fwd}
export TMPDIR=/tmp; mkdir -p gpurun_out/pmcconv_$TAG
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"
run() {  # lib-tag
  local v=$1
  local i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmcconv_$TAG/${v}_p$i -o p --output-format csv -- python3 tools/kbench_conv.py 300 "$L" "$M" > gpurun_out/pmcconv_$TAG/${v}_p$i.log 2>&1 || { echo "pmc $v p$i failed"; tail -5 gpurun_out/pmcconv_$TAG/${v}_p$i.log; return 1; }
    i=$((i+1))
  done
}
run base || exit 1
for lib in variants/*/libblindno.so; do
  v=$(basename $(dirname $lib))
  BLINDNO_LIB=$lib run $v || exit 1
done
python3 - "$TAG" <<'PY'
import csv, glob, os, sys, collections
tag = sys.argv[1]
root = f"gpurun_out/pmcconv_{tag}"
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/**/*counter_collection.csv", recursive=True):
    v = os.path.relpath(f, root).split(os.sep)[0].rsplit("_p", 1)[0]
    for r in csv.DictReader(open(f)):
        if "conv_igemm" not in r["Kernel_Name"]:
            continue
        res[v][r["Counter_Name"]].append(float(r["Counter_Value"]))
for v, d in res.items():
    print(v, "  ".join(f"{k}={sum(x)/len(x):.4g}" for k, x in sorted(d.items())))
PY
