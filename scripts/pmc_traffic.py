#!/usr/bin/env python3
"""Per-launch HBM traffic of the codec kernels from two rocprofv3 --pmc passes.

Usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [config bits]
The measurement goes under runs["<config>/s<bits>"] of OUT_JSON; the other runs already in it are
kept when they were measured on the same kernel sources (source digest), dropped otherwise.
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128 B request of a wide
coalesced stream, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            per[name].append(float(r["Counter_Value"]))
    return per


# one encode call's launches: the planned scatter (the default since round 5), or plan + scatter;
# since round 6 the exact tail (zero fill, fallback) ends every call
TOPK_ENCODE_SETS = (("topk_sample", "topk_fused", "topk_fine_hist", "topk_scatter_planned", "topk_bucket_sort",
                     "topk_exact_tail"),
                    ("topk_sample", "topk_fused", "topk_fine_hist", "topk_plan", "topk_bucket_scatter",
                     "topk_bucket_sort", "topk_exact_tail"))
TOPK_ENCODE = tuple(sorted(set(TOPK_ENCODE_SETS[0] + TOPK_ENCODE_SETS[1])))
TOPK_DECODE = ("topk_dec_place", "topk_dec_tiles", "topk_dec_overflow")


def short(name):
    if "qsgd_spec_bracket_wide(" in name:  # the wide-level bracket kernel (bit widths 5-8)
        return "qsgd_spec_bracket"
    for k in ("qsgd_encode_pc", "qsgd_encode_ordered", "qsgd_encode_win", "qsgd_encode_grid", "qsgd_decode_flat",
              "qsgd_decode_arena", "qsgd_quant_sub",
              "qsgd_spec_bracket", "qsgd_spec_quant_fb", "qsgd_spec_quant_wfb", "qsgd_spec_quant", "qsgd_spec_finish",
              "topk_prep_hist", "topk_collect", "topk_gather", "topk_scatter_arena") + TOPK_ENCODE + TOPK_DECODE:
        if k + "(" in name or k + "<" in name:
            return k
    return None


def main():
    fdir, wdir, out = sys.argv[1:4]
    cfg = sys.argv[4] if len(sys.argv) > 4 else "llama400m"
    bits = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {}
    for name, vals in fetch.items():
        k = short(name)
        if not k or name not in write:
            continue
        f = 2 * 1024 * sum(vals) / len(vals)
        w = 1024 * sum(write[name]) / len(write[name])
        res[k] = {"fetch_bytes_corrected": f, "write_bytes": w, "launches": len(vals)}
    # the bracketed encoder: one launch of each per encode — bracket + quant + finish, or (the fused
    # bracket, the default at widths <= 4) quant_fb + finish, the bracket being quant_fb's first blocks
    # (wide levels since round 5: quant_wfb + finish, the bracket being quant_wfb's first one-wave blocks)
    for spec in (("qsgd_spec_bracket", "qsgd_spec_quant", "qsgd_spec_finish"), ("qsgd_spec_quant_fb", "qsgd_spec_finish"),
                 ("qsgd_spec_quant_wfb", "qsgd_spec_finish")):
        if all(k in res for k in spec):
            res["qsgd_spec_all"] = {kk: sum(res[k][kk] for k in spec) for kk in ("fetch_bytes_corrected", "write_bytes")}
            res["qsgd_spec_all"]["launches"] = res[spec[-2]]["launches"]
            break
    # Top-K: every launch of one encode call (resp. one tiled decode call), summed
    enc = next((p for p in TOPK_ENCODE_SETS if all(k in res for k in p)), TOPK_ENCODE_SETS[0])
    for agg, parts in (("topk_encode_all", enc), ("topk_decode_all", TOPK_DECODE)):
        if all(k in res for k in parts):
            res[agg] = {kk: sum(res[k][kk] for k in parts) for kk in ("fetch_bytes_corrected", "write_bytes")}
            res[agg]["launches"] = res[parts[-1]]["launches"]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from omnifed_amd.build import source_digest
    import datetime
    import subprocess

    commit = os.environ.get("OMF_COMMIT", "")  # the GPU box's copy has no .git: pass it in
    if not commit:
        try:
            commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True).stdout.strip()
        except OSError:
            commit = ""
    sha = source_digest()
    runs = {}
    try:
        with open(out) as fh:
            old = json.load(fh)
        if old.get("source_sha") == sha:
            runs = old.get("runs", {})
    except (OSError, ValueError):
        pass
    run = {"config": cfg, "bits": bits,
           "bytes_per_launch": {k: round(v["fetch_bytes_corrected"] + v["write_bytes"]) for k, v in res.items()},
           "detail": res}
    runs[f"{cfg}/s{bits}"] = run
    j = {"source_sha": sha, "commit": commit or None,
         "date": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%d"), "note": "FETCH_SIZE x2 (gfx950 wide-load correction) + WRITE_SIZE, KiB->B, "
         "average per launch; Infinity-Cache hits are counted as fetches",
         "runs": runs}
    with open(out, "w") as fh:
        json.dump(j, fh, indent=1)
    print(json.dumps(run["bytes_per_launch"]))


if __name__ == "__main__":
    main()
