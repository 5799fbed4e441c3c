#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 --pmc passes over a bench.py run (the benched, graph-
replayed step), as tools/pmc_bench.sh collects them: one directory per counter group.

    python tools/pmc_bench.py gpurun_out/pmcb_TAG REGEX [LAST]

For the dispatches of the kernels matching REGEX (the LAST of each pass: the timed steps and the
kernel-timer steps, not the capture warm-ups) it averages every counter per dispatch and reports
the VALU issue utilisation with pmc_traffic.py's formula

    valu_issue_util = (4 (VALU - MFMA - TRANS) + 8 TRANS) / (1024 SIMDs x clock x duration),

the clock from GRBM_GUI_ACTIVE / 8 XCDs / duration, and HBM bytes per dispatch
(2 FETCH_SIZE + WRITE_SIZE, KiB, MI355X_MICROARCH.md's gfx950 correction)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main():
    root, pat = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    per = defaultdict(list)       # counter -> values (last dispatches of each pass)
    durs = []
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if re.search(pat, r["Kernel_Name"])]
        by_disp = defaultdict(dict)
        meta = {}
        for r in rows:
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        ds = sorted(by_disp, key=lambda d: meta[d][0])[-last:]
        for d in ds:
            for c, v in by_disp[d].items():
                per[c].append(v)
            durs.append((meta[d][1] - meta[d][0]) * 1e-9)
    a = {c: sum(v) / len(v) for c, v in per.items()}
    t = sum(durs) / len(durs)
    out = {"kernel_regex": pat, "dispatches_per_pass": last, "us_per_dispatch_profiled": round(t * 1e6, 2),
           "counters": {c: round(v, 1) for c, v in sorted(a.items())}}
    if "FETCH_SIZE" in a:
        out["hbm_bytes_per_dispatch"] = int(2 * 1024 * a["FETCH_SIZE"] + 1024 * a.get("WRITE_SIZE", 0.0))
    if "SQ_INSTS_VALU" in a and "GRBM_GUI_ACTIVE" in a:
        valu, trans, mfma = a["SQ_INSTS_VALU"], a.get("SQ_INSTS_VALU_TRANS_F32", 0.0), a.get("SQ_INSTS_MFMA", 0.0)
        clk = a["GRBM_GUI_ACTIVE"] / 8 / t
        out["clock_GHz"] = round(clk / 1e9, 3)
        out["valu_issue_util"] = round((4 * (valu - mfma - trans) + 8 * trans) / (1024 * clk * t), 3)
    if "SQ_ACTIVE_INST_VALU" in a and "SQ_BUSY_CYCLES" in a:
        out["note"] = "SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES are summed over SEs (raw)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
