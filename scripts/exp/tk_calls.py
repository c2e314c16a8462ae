"""Per-call Top-K kernel durations (us) from a rocprofv3 results DB, grouped by encode call
(an encode starts at topk_setup); experiment helper."""
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
calls, cur = [], None
for name, s, e in rows:
    short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if "topk_setup" in short:
        cur = {"_start": s, "_k": []}
        calls.append(cur)
    if cur is None:
        continue
    if "topk" not in short and "rocprim" not in short and "rocclr" not in short:
        continue
    cur["_k"].append((short[-28:], (e - s) / 1e3))
    cur["_end"] = e
for i, c in enumerate(calls):
    tot = sum(d for _, d in c["_k"])
    print(f"call {i:2d}: span {(c['_end'] - c['_start']) / 1e3:7.1f} us, kernels {tot:7.1f}: " +
          " ".join(f"{n.split('<')[0][-14:]}={d:.0f}" for n, d in c["_k"]))

# gaps: GPU idle between consecutive kernels inside each call, and before each call's setup
prev_end = None
for i, c in enumerate(calls):
    print(f"call {i:2d}: idle before setup {((c['_start'] - prev_end) / 1e3) if prev_end else 0:7.1f} us")
    prev_end = c["_end"]
