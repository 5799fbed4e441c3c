#!/usr/bin/env python3
"""Average duration of the LAST n launches of a kernel in a rocprofv3 kernel trace.

    python tools/trace_kernel_avg.py gpurun_out/prof_TAG/run_kernel_trace.csv REGEX N

bench.py captures one graph per bag key before its timed region (each capture runs one eager
warm-up body, over the whole key range), so the rocprofv3 --stats average mixes those warm-ups
with the timed steps.  The last N launches are the timed steps and the kernel-timer steps that
bench.py's roofline.avg_ms is measured on."""
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if re.search(sys.argv[2], r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[3])
sel = rows[-n:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
print(f"{len(rows)} launches; last {len(sel)}: avg {sum(d) / len(d):.1f} us "
      f"(min {min(d):.1f}, max {max(d):.1f})")
