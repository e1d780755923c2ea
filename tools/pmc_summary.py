#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the projector's kernels.

    python tools/pmc_summary.py <prof_dir> [--json out.json --key <bench key>]

<prof_dir> holds the kernel-trace run (``kt/*_kernel_stats.csv``) and PMC passes
(``p*/*_counter_collection.csv``), each PMC pass a separate rocprofv3 run.  Prints, per
asp kernel: calls, average duration, and per-dispatch averages of every counter.

HBM traffic per dispatch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports HALF
the bytes of wide coalesced streaming reads on gfx950, so it is doubled;
WRITE_SIZE (KiB) is taken as is:  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
The doubling is exact only for 16-B-per-lane streaming loads (the records and particle
arrays here); other access widths are uncalibrated.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

STAGE_OF = {"k_count": "count", "k_colscan": "colscan", "k_tilescan": "tilescan",
            "k_scatter": "scatter", "k_deposit": "deposit", "k_wide": "wide",
            "k_ratio": "ratio", "k_bin": "scatter", "k_deposit3d": "deposit",
            "k_gather": "gather", "k_merge": "merge"}


def short(name):
    m = re.search(r"asp::(k[0-9]?_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--key")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*_counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            meta[k] = {x: r[x] for x in ("VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                                         "Scratch_Size", "Workgroup_Size")}
        for (k, _, c), val in per.items():
            ctr[k][c].append(val)
    out = {}
    names = sorted(set(durs) | set(ctr), key=lambda k: -sum(durs.get(k, [0])))
    for k in names:
        d = durs.get(k, [])
        row = {"calls": len(d), "avg_us": (sum(d) / len(d) / 1e3) if d else None}
        for c, vals in sorted(ctr[k].items()):
            row[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in row or "WRITE_SIZE" in row:
            row["hbm_bytes_per_launch"] = (2 * row.get("FETCH_SIZE", 0.0)
                                          + row.get("WRITE_SIZE", 0.0)) * 1024
        row.update(meta.get(k, {}))
        out[k] = row
        print(f"== {k}")
        for c, val in row.items():
            print(f"   {c:24s} {val:,.3f}" if isinstance(val, float) else f"   {c:24s} {val}")
    if a.json:
        db = {}
        if os.path.exists(a.json):
            db = json.load(open(a.json))
        stage = {}
        for k, row in out.items():
            s = STAGE_OF.get(k.split("<")[0])
            # the placement trials' probe instantiation (k_scatter<KID, NOUT, ACC, CULL, SRC,
            # PROBE, NX>, PROBE = 1) is not the steady state: never the stage's record
            targs = [x.strip() for x in k[k.find("<") + 1:].rstrip(">").split(",")]
            if k.startswith("k_scatter<") and len(targs) >= 6 and targs[5] == "1":
                continue
            # the first (largest total time) kernel of a stage
            if s and s not in stage and "hbm_bytes_per_launch" in row:
                stage[s] = {"hbm_bytes_per_launch": row["hbm_bytes_per_launch"],
                            "avg_us": row["avg_us"], "kernel": k}
                stage[s].update({c: v for c, v in row.items() if c.startswith("SQ_")})
        stage["source"] = a.source
        db[a.key] = stage
        json.dump(db, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
