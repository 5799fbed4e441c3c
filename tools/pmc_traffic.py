#!/usr/bin/env python3
"""Write profiles/pmc_traffic.json: measured HBM bytes per crop point of the dominant kernel
from a tools/pmc_kbench.sh run (FETCH_SIZE doubled -- the gfx950 correction for 16-B streaming
reads, MI355X_MICROARCH.md "HBM" -- plus WRITE_SIZE, both in KiB per dispatch).

    python tools/pmc_traffic.py gpurun_out/pmck_TAG
The kbench shape is config C's snapshot encoder at the mean bag size: Bn = 4 * 75, 128 x 128.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"blindno_project_bwd": "project_bwd_mfma_kernel<4,"}
NPTS = 300 * 128 * 128


def main():
    root = sys.argv[1]
    out = {}
    for abi, pat in KERNELS.items():
        vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
        for f in glob.glob(os.path.join(root, "p*", "run_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if pat in r["Kernel_Name"].replace(" ", "") and r["Counter_Name"] in vals:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if not vals["FETCH_SIZE"] or not vals["WRITE_SIZE"]:
            continue
        fetch = 2 * 1024 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
        write = 1024 * sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
        out[abi] = {"bytes_per_point": round((fetch + write) / NPTS, 3),
                    "fetch_bytes_x2": int(fetch), "write_bytes": int(write), "points": NPTS,
                    "source": os.path.relpath(root, ROOT)}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
