#!/usr/bin/env python3
"""Per-kernel SQ counter summary from rocprofv3 --pmc passes (one directory per pass).

Usage: python scripts/sq_summary.py OUT_JSON ELEMENTS DIR [DIR ...]
Every counter is averaged over a kernel's dispatches.  Derived, per kernel:
  valu_insts_per_element  SQ_INSTS_VALU x 64 lanes / ELEMENTS (the wave-level count times the
                          wave width: lane-instructions per element of the arena)
  wave_wait_frac          SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves waiting on a counter or barrier)
  wave_issue_frac         SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  wave_stall_frac         SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (an instruction ready, not issued)
  valu_issue_frac         SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_ANY
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void\s+", "", name.replace("(anonymous namespace)::", ""))
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*[<(]", name)
    return m.group(1) if m else name


def main():
    out, elements, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                vals[short(r.get("Kernel_Name", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in vals.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "counters": {c: round(x, 1) for c, x in a.items()}}
        wc = a.get("SQ_WAVE_CYCLES")
        if "SQ_INSTS_VALU" in a:
            d["valu_insts_per_element"] = round(a["SQ_INSTS_VALU"] * 64 / elements, 2)
        if wc:
            for key, c in (("wave_wait_frac", "SQ_WAIT_ANY"), ("wave_issue_frac", "SQ_ACTIVE_INST_ANY"),
                           ("wave_stall_frac", "SQ_WAIT_INST_ANY")):
                if c in a:
                    d[key] = round(a[c] / wc, 3)
        if a.get("SQ_ACTIVE_INST_ANY") and "SQ_ACTIVE_INST_VALU" in a:
            d["valu_issue_frac"] = round(a["SQ_ACTIVE_INST_VALU"] / a["SQ_ACTIVE_INST_ANY"], 3)
        res[k] = d
    with open(out, "w") as fh:
        json.dump({"elements": elements, "kernels": res}, fh, indent=1)
    for k, d in sorted(res.items()):
        print(k, {x: y for x, y in d.items() if x != "counters"})


if __name__ == "__main__":
    main()
