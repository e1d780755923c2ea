#!/usr/bin/env python3
"""One map's launches from a rocprofv3 kernel trace: start, gap after the previous launch,
duration -- the inter-kernel gaps of the pipeline (the N = 8 share).
    python tools/timeline.py TRACE.csv [--maps 3] [--first k_count]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--maps", type=int, default=3, help="maps (from the last ones) to print")
ap.add_argument("--first", default="k_count", help="the first kernel of a map")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("void ", "") for r in rows]
starts = [i for i, n in enumerate(names) if a.first in n]
lo = starts[-a.maps - 1]
hi = starts[-1]
t0 = int(rows[lo]["Start_Timestamp"])
end = None
gaps = busy = 0.0
for r, n in zip(rows[lo:hi], names[lo:hi]):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0.0 if end is None else max(0.0, (s - end) / 1e3)
    gaps += gap
    busy += max(0.0, (e - max(s, end or s)) / 1e3)
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:6.1f}  {(e - s) / 1e3:8.1f} us  {n[:64]}")
    end = max(e, end or e)
print(f"{a.maps} maps: busy {busy:.1f} us, gaps {gaps:.1f} us ({gaps / max(1e-9, busy + gaps):.1%} of the span)")
