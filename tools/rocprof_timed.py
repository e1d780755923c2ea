#!/usr/bin/env python3
"""The rocprofv3 kernel trace of a bench.py command, restricted to the TIMED steps.

bench.py's line reports the dominant kernel's average launch time over its timed steps
(HIP events).  rocprofv3 --stats averages every launch of the process: warmup, the
placement trials (a kernel of their own, PROBE = 1), the timed steps, and -- when maps
alternate between streams -- the single-map latency phase, whose launches run alone.
This picks the steady-state launches of one kernel in start order and averages the
window the timed steps occupy.
  python tools/rocprof_timed.py TRACE.csv 'k_scatter<1, 2, 0, false, 0, 0, 0>' --skip 1 --count 10
(--skip: the steady-state launches before the timed steps = warmup maps not scattered by
the placement trials.)"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("kernel", help="substring of the kernel name")
ap.add_argument("--skip", type=int, default=0)
ap.add_argument("--count", type=int, default=10)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
win = us[a.skip:a.skip + a.count]
print(f"{len(us)} launches of {a.kernel!r}: " + " ".join(f"{x:.0f}" for x in us))
print(f"launches {a.skip}..{a.skip + len(win) - 1}: average {sum(win) / max(1, len(win)):.1f} us")
