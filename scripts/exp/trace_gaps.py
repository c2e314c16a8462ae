"""Per-kernel mean duration and the mean idle gap before each kernel, from a rocprofv3
--kernel-trace CSV (experiment): python scripts/exp/trace_gaps.py DIR [last_n]."""
import csv
import glob
import re
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
rows = rows[-last:]
dur, gap = defaultdict(list), defaultdict(list)
prev_end = None
prev = ""
for r in rows:
    m = re.search(r"(qsgd_\w+|topk_\w+|omf\w+)", r["Kernel_Name"])
    name = (m.group(1) if m else r["Kernel_Name"][:40])
    name, prev = f"{name} (after {prev})", name
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[name].append(e - s)
    if prev_end is not None:
        gap[name].append(s - prev_end)
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"{len(rows)} kernels over {span:.1f} us")
for k in dur:
    g = gap.get(k, [0])
    print(f"  {k:28s} n={len(dur[k]):4d} dur={sum(dur[k]) / len(dur[k]) / 1e3:7.2f} us  gap before={sum(g) / len(g) / 1e3:6.2f} us")
