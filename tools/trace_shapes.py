"""Per-(kernel, grid) average durations from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for x in rows:
    n = x["Kernel_Name"]
    m = re.search(r"::(\w+)(<[^(]*>)?\(", n)
    short = (m.group(1) + (m.group(2) or "")) if m else n[:40]
    if pat and not re.search(pat, short):
        continue
    wg = int(x["Workgroup_Size_X"])
    key = (short, int(x["Grid_Size_X"]) // max(wg, 1), wg)
    d[key].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:45s} blocks={k[1]:8d} wg={k[2]:5d} n={len(v):4d} avg={sum(v)/len(v)/1e3:9.2f}us")
