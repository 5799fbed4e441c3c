#!/usr/bin/env python3
"""Per-step kernel breakdown of the LAST k training steps in a rocprofv3 kernel trace.

    python tools/step_breakdown.py gpurun_out/prof_TAG/run_kernel_trace.csv [k] [top] [skip]

skip: trailing Adam windows to drop first (bench.py's eager kernel-timer steps after the timed
region, 4 by default there).

A step ends with the fused Adam launch (adam_kernel); the k windows between the last k+1 Adam
launches are the timed steps.  Prints each kernel's time per step, its share of the summed
kernel time and the step's wall span (first start to Adam end), so idle gaps show up as
wall - busy."""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    ad = [i for i, r in enumerate(rows) if re.search(r"adam", r["Kernel_Name"])]
    if skip:
        ad = ad[:-skip]
    ad = ad[-(k + 1):]
    per = defaultdict(float)
    cnt = defaultdict(int)
    wall = 0.0
    for a, b in zip(ad[:-1], ad[1:]):
        win = rows[a + 1:b + 1]
        wall += (win[-1]["e"] - rows[a]["e"]) / 1e3
        for r in win:
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            name = re.sub(r"\(.*", "", name)
            per[name] += (r["e"] - r["s"]) / 1e3
            cnt[name] += 1
    n = len(ad) - 1
    busy = sum(per.values()) / n
    print(f"{n} steps: wall {wall / n:.1f} us/step, kernel busy {busy:.1f} us/step, "
          f"launches {sum(cnt.values()) / n:.0f}/step")
    for name, t in sorted(per.items(), key=lambda x: -x[1])[:top]:
        print(f"{t / n:8.1f} us {100 * t / n / busy:5.1f}%  x{cnt[name] / n:4.1f}  {name[:100]}")


if __name__ == "__main__":
    main()
