"""Kernel and HIP API timeline of one rocprofv3 run (experiment): the last N kernels with the gap
before each, and the HIP API calls issued in those gaps."""
import csv
import glob
import re
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
kt = sorted(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])),
            key=lambda r: int(r["Start_Timestamp"]))[-n:]
api = []
for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    api += list(csv.DictReader(open(f)))
api.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(kt[0]["Start_Timestamp"])
prev = None
for r in kt:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    m = re.search(r"(topk_\w+|qsgd_\w+|__amd_rocclr_\w+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:30]
    if prev is not None and s - prev > 3000:
        calls = [(int(a["Start_Timestamp"]) - t0, a["Function"]) for a in api
                 if prev - 400000 <= int(a["Start_Timestamp"]) <= s]
        print(f"   gap {(s - prev) / 1e3:.1f} us; API calls in the 400 us before: "
              + ", ".join(f"{fn}@{(ts) / 1e3:.1f}" for ts, fn in calls[-8:]))
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} us  {name}")
    prev = e
