#!/usr/bin/env python3
"""Write profiles/pmc_traffic.json from a tools/pmc_kbench.sh run over kbench's "[input]" cases
(config C's snapshot encoder at the mean bag size: Bn = 4 * 75 snapshots, P = 160, 128^2 crop).

    python tools/pmc_traffic.py gpurun_out/pmck_TAG [profiles/rNN/TAG_pmc_summary.json] [--n 256 --prefix E:]

--n / --prefix: the kbench run was at another encoder grid (KBENCH_N; config E: 256, its records
are stored as "E:<entry>"); records are merged into the existing file (other prefixes kept).

The optional second argument names the committed per-kernel summary of the same passes
(tools/pmc_summary.py --json), recorded as each entry's "source".

Per kernel: measured HBM bytes per dispatch (FETCH_SIZE doubled -- the gfx950 correction for
16-B streaming reads, MI355X_MICROARCH.md "HBM" -- plus WRITE_SIZE, both KiB per dispatch) and,
for the projection backward, bytes per crop point (bench.py scales it to the launch's points)
and its VALU issue utilisation:

    valu_issue_util = (4 (VALU - MFMA - TRANS) + 8 TRANS) / (1024 SIMDs x clock x duration)

with the issue costs of MI355X_MICROARCH.md's constants table (v_fma / v_add / v_pk_* 4 cycles,
v_exp / v_rcp 8 cycles per wave64 instruction; MFMA issue holds are left out), SQ_INSTS_VALU,
SQ_INSTS_MFMA and SQ_INSTS_VALU_TRANS_F32 summed over the dispatch, and the clock from
GRBM_GUI_ACTIVE / 8 XCDs / duration (the guide's DVFS note)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ABI entry -> kernel-name pattern of its [input] kbench case (grid-size filter below)
KERNELS = {
    "blindno_project_bag_fwd": r"bagproj_fwd_kernel",
    "blindno_project_bag_bwd": r"bagproj_bwd_kernel",
    "blindno_project_bwd": r"project_bwd_mfma_kernel<4,",
    "blindno_project_fwd": r"project_fwd_mfma_kernel<4,",
    "blindno_rowdft": r"rowdft_mfma_kernel<",
    "blindno_rowidft_epi": r"rowfuse_kernel<0, 1, 0, 0, 0, .*false, false",
    "colfuse (blindno_colpass, FNO_input)": r"colfuse_kernel<0,",
    "blindno_rowidft_epi_rd": r"rowfuse_kernel<0, 1, 0, 0, 2, .*false, false",
    "blindno_rowidft_bwd": r"rowfuse_kernel<1, 1, 1, 0, 0, .*false, false",
    "blindno_rowidft_bwd_rd_crop": r"rowfuse_kernel<1, 1, 1, 0, 1, .*false, false",
    # the column pass folded into the row kernels (csrc/colspec.h)
    "blindno_colmix": r"colmix_kernel<0, false>",
    "blindno_rowidft_epi_zc": r"rowfuse_kernel<0, 1, 0, 0, 2, .*true, true",
    "blindno_rowdft_cd": r"rowdft_cd_kernel<2, true, false>",
    "blindno_rowidft_bwd_zc_crop": r"rowfuse_kernel<1, 1, 1, 0, 1, .*true, true",
    "coldft_mix (blindno_colpass)": r"coldft_mix_kernel<0,",
    "colidft (blindno_colpass)": r"colidft_kernel",
}


def main():
    args = sys.argv[1:]
    n_grid, prefix = 128, ""
    if "--n" in args:
        i = args.index("--n")
        n_grid = int(args[i + 1])
        del args[i:i + 2]
    if "--prefix" in args:
        i = args.index("--prefix")
        prefix = args[i + 1]
        del args[i:i + 2]
    root = args[0]
    src = args[1] if len(args) > 1 else os.path.relpath(root, ROOT)
    npts = 300 * n_grid * n_grid
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            for abi, pat in KERNELS.items():
                if re.search(pat, name):
                    # the [input] case is the largest grid of that kernel in the kbench run
                    key = (abi, int(r["Grid_Size"]))
                    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {}
    for abi in KERNELS:
        keys = [k for k in acc if k[0] == abi and "FETCH_SIZE" in acc[k]]
        if not keys:
            continue
        key = max(keys, key=lambda k: sum(acc[k]["FETCH_SIZE"]) / len(acc[k]["FETCH_SIZE"]))
        a = {c: sum(v) / len(v) for c, v in acc[key].items()}
        t = sum(dur[key]) / len(dur[key])
        fetch = 2 * 1024 * a["FETCH_SIZE"]
        write = 1024 * a.get("WRITE_SIZE", 0.0)
        rec = {"fetch_bytes_x2": int(fetch), "write_bytes": int(write),
               "hbm_bytes_per_dispatch": int(fetch + write), "us_per_dispatch_profiled": round(t * 1e6, 2),
               "grid": key[1], "source": src, "N": n_grid}
        if abi.startswith("blindno_project"):
            rec["bytes_per_point"] = round((fetch + write) / npts, 3)
            rec["points"] = npts
        if "SQ_INSTS_VALU" in a and "GRBM_GUI_ACTIVE" in a:
            valu, trans = a["SQ_INSTS_VALU"], a.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
            mfma = a.get("SQ_INSTS_MFMA", 0.0)
            clk = a["GRBM_GUI_ACTIVE"] / 8 / t
            cyc = 4 * (valu - mfma - trans) + 8 * trans
            rec.update({"SQ_INSTS_VALU": int(valu), "SQ_INSTS_VALU_TRANS_F32": int(trans),
                        "SQ_INSTS_MFMA": int(mfma), "clock_GHz": round(clk / 1e9, 3),
                        "valu_issue_util": round(cyc / (1024 * clk * t), 3)})
        out[prefix + abi] = rec
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    # replace this prefix's records, keep the others
    merged = {k: v for k, v in old.items() if not (k.startswith(prefix) and (prefix or ":" not in k))}
    merged.update(out)
    json.dump(merged, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
