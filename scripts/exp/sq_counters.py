"""Summarise SQ/GRBM PMC passes per kernel (mean over dispatches): usage DIR [DIR...]."""
import csv
import glob
import os
import sys
from collections import defaultdict

per = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in per.items():
    if not any(s in k for s in ("qsgd", "topk")):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
