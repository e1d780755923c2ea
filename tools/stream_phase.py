#!/usr/bin/env python3
"""Per-stream durations of the scatter and deposit launches in a rocprofv3 kernel trace of
bench.py (the sequential region on one stream, then the overlapped region alternating two):
shows whether the overlapped region's alternating scatter times come from the workspace
slots (placement) or from which kernel each launch overlaps.
    python tools/stream_phase.py TRACE.csv [TRACE2.csv ...]"""
import csv
import sys

KERNELS = ("k_scatter<1, 2, 0, false, 0, 0, 0, 0>", "k_deposit<1, 2, 0, 0>")
for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    print(path)
    for k in KERNELS:
        sel = [r for r in rows if k in r["Kernel_Name"]]
        per = {}
        for r in sel:
            per.setdefault(r["Stream_Id"], []).append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f"  {k}: " + "; ".join(
            f"stream {s}: n={len(v)} mean {sum(v) / len(v):.0f} us (min {min(v):.0f}, max {max(v):.0f})"
            for s, v in per.items()))
        print("    in launch order (us/stream): " + " ".join(
            f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f}/{r['Stream_Id']}" for r in sel))
