#!/usr/bin/env python3
"""Print ms/step and the per-stage ms of bench.py JSON lines (one file per argument)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    st = {k: round(v["ms_per_launch"], 4) for k, v in d.get("stages", {}).items()}
    print(f, d["ms_per_step"], st, "frac", d["roofline"].get("frac"))
