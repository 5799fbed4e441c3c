#!/usr/bin/env python3
"""Print the kernel timeline of one training step from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/prof_TAG/run_kernel_trace.csv [step-from-end]

A step starts after the adam kernel of the previous step; times are us from the step start,
with the HIP queue of each kernel (concurrent branches show as different queues)."""
import csv
import re
import sys


def short(n):
    m = re.search(r"::(\w+)(<[^(]*>)?\(", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 r.get("Queue_Id", ""), r.get("Grid_Size", ""), r.get("Workgroup_Size", ""),
                 r.get("VGPR_Count", r.get("Arch_VGPR_Count", ""))) for r in rows)
    adams = [i for i, e in enumerate(ev) if e[2].startswith("adam")]
    a0, a1 = adams[-1 - back], adams[-back]
    t0 = ev[a0 + 1][0]
    busy = 0
    for e in ev[a0 + 1:a1 + 1]:
        wg = int(e[4]) // max(1, int(e[5])) if e[4] and e[5] else ""
        print(f"{(e[0] - t0) / 1e3:8.1f} {(e[1] - e[0]) / 1e3:7.1f} q{e[3]} wg={wg:<6} v{e[6]:<4} {e[2][:64]}")
        busy += e[1] - e[0]
    print(f"step {(ev[a1][1] - t0) / 1e3:.1f} us, kernel-busy sum {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
