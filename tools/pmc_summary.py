#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (tools/pmc_passes.sh output).

    python tools/pmc_summary.py gpurun_out/pmc_TAG [kernel-regex] [--json out.json]

Groups dispatches by (short kernel name, grid size), averages every counter over the
dispatches of each group and prints one row per group.  FETCH_SIZE is reported as measured
(KiB) and doubled (the gfx950 correction for 16-B streaming reads, MI355X_MICROARCH.md HBM).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"::(\w+)(<[^(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:48]


def load(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("FETCH_SIZE",):
                dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return acc, dur


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    acc, dur = load(root)
    rows = []
    for key, cs in acc.items():
        if pat and not re.search(pat, key[0]):
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = sum(dur[key]) / len(dur[key]) if dur[key] else 0.0
        rows.append((key, d, avg))
    rows.sort(key=lambda r: -r[1] * len(acc[r[0]].get("FETCH_SIZE", [1])))
    out = []
    for (name, grid, wg), d, a in rows[:40]:
        fetch = a.get("FETCH_SIZE", 0.0)
        write = a.get("WRITE_SIZE", 0.0)
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        rec = {"kernel": name, "grid": grid, "wg": wg, "us": round(d, 2),
               "fetch_MB_x2": round(2 * fetch / 1024, 3), "write_MB": round(write / 1024, 3)}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_WAVES", "SQ_BUSY_CYCLES",
                  "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            if c in a:
                rec[c] = a[c]
        if wc:
            rec["wait_any_frac"] = round(a.get("SQ_WAIT_ANY", 0) / wc, 3)
            rec["wait_inst_frac"] = round(a.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
            rec["active_frac"] = round(a.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
            rec["valu_frac"] = round(a.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
            rec["lds_frac"] = round(a.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3)
        out.append(rec)
        gbs = (2 * fetch + write) * 1024 / (d * 1e-6) / 1e9 if d else 0
        print(f"{name[:40]:40s} g={grid:8d} {d:8.1f}us rd2x={2*fetch/1024:8.2f}MB wr={write/1024:8.2f}MB "
              f"{gbs:7.0f}GB/s valu={a.get('SQ_INSTS_VALU',0):10.0f} lds={a.get('SQ_INSTS_LDS',0):8.0f} "
              f"mfma={a.get('SQ_INSTS_MFMA',0):8.0f} bankc={a.get('SQ_LDS_BANK_CONFLICT',0):8.0f} "
              f"wait={rec.get('wait_any_frac',0):.2f} winst={rec.get('wait_inst_frac',0):.2f} "
              f"act={rec.get('active_frac',0):.2f}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
