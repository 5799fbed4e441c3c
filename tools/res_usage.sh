#!/bin/bash
# Per-kernel register / occupancy summary of one HIP source (compiler remarks).
# usage: [RES_FLAGS="-DMACRO=1"] bash tools/res_usage.sh csrc/FILE.hip [kernel-name-regex]
cd "$(dirname "$0")/../reconstruction-of-pde-without-time-label_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I ../include -I csrc -fvisibility=hidden \
  -Wno-unused-function $RES_FLAGS -c "$1" -o /tmp/res_usage.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys, subprocess
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None: cur[k] = v
for r in rows:
    if re.search(pat, r["name"]):
        n = r["name"].replace("(anonymous namespace)::", "")
        n = n[:n.find("(")] if "(" in n else n
        g = r.get
        print("%-70s v%s a%s occ%s sspill%s vspill%s scr%s" % (n, g("VGPRs"), g("AGPRs"), g("Occupancy [waves/SIMD]"), g("SGPRs Spill"), g("VGPRs Spill"), g("ScratchSize [bytes/lane]")))
' "$2"
