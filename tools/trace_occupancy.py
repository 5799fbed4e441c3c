#!/usr/bin/env python3
"""Per-kernel launch shape against the chip's resident capacity, from a rocprofv3 kernel trace:

    python tools/trace_occupancy.py run_kernel_trace.csv [regex]

For every (kernel, grid) pair: workgroups, waves per workgroup, VGPRs (arch + accumulation),
LDS per workgroup, the workgroups one CU holds at once (VGPR file 512 per SIMD lane, 8 waves per
SIMD, 160 KB LDS), the resident capacity of 256 CUs, the rounds the grid needs (a fractional
last round is a tail where most of the chip idles) and the average duration.
"""
import collections
import csv
import math
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    d = collections.defaultdict(list)
    for x in rows:
        n = x["Kernel_Name"]
        m = re.search(r"::(\w+)(<[^(]*>)?\(", n)
        short = (m.group(1) + (m.group(2) or "")) if m else n[:40]
        if pat and not re.search(pat, short):
            continue
        wg = int(x["Workgroup_Size_X"]) * int(x.get("Workgroup_Size_Y", 1) or 1) * int(x.get("Workgroup_Size_Z", 1) or 1)
        blocks = (int(x["Grid_Size_X"]) * int(x.get("Grid_Size_Y", 1) or 1) * int(x.get("Grid_Size_Z", 1) or 1)) // max(wg, 1)
        # the trace's VGPR_Count is half the compiler's figure on gfx950 (checked against the
        # kernel-resource-usage remarks of rowinv_wide (128), colfuse (240), bagproj_fwd (160))
        vg = 2 * (int(x.get("VGPR_Count", x.get("Arch_VGPR_Count", 0)) or 0) + int(x.get("Accum_VGPR_Count", 0) or 0))
        lds = int(x.get("LDS_Block_Size", x.get("Group_Segment_Size", 0)) or 0)
        key = (short, blocks, wg, vg, lds)
        d[key].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
    print(f"{'kernel':52s} {'blocks':>7s} {'wg':>4s} {'vgpr':>4s} {'lds':>6s} {'wg/CU':>5s} {'cap':>6s} {'rounds':>6s} {'n':>4s} {'avg us':>8s}")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        short, blocks, wg, vg, lds = k
        wpw = max(1, math.ceil(wg / 64))
        per_simd = min(8, 512 // max(8, 8 * math.ceil(vg / 8))) if vg else 8
        by_waves = (4 * per_simd) // wpw
        by_lds = (160 * 1024) // lds if lds else 64
        wgcu = max(0, min(by_waves, by_lds))
        cap = 256 * wgcu
        rounds = blocks / cap if cap else float("inf")
        print(f"{short[:52]:52s} {blocks:7d} {wg:4d} {vg:4d} {lds:6d} {wgcu:5d} {cap:6d} {rounds:6.2f} {len(v):4d} "
              f"{sum(v) / len(v) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
