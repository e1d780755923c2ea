#!/usr/bin/env python3
"""Copy one measurement session (tools/gpu/measure.sh -> gpurun_out/meas, prof_meas) into
the tracked profiles/<round>/ directory, and cross-check the rocprofv3 kernel averages
against the HIP-event stage times bench.py measured in its own run.

    python3 tools/collect_profiles.py r01
"""
import csv
import re
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGE_OF = {"k_scatter": "scatter", "k_deposit": "deposit", "k_count": "count",
            "k_merge": "merge", "k_colscan": "colscan", "k_tilescan": "tilescan",
            "k_wide": "wide", "k_ratio": "ratio", "k_band": "band"}


def main(tag):
    meas = os.path.join(REPO, "gpurun_out", "meas")
    prof = os.path.join(REPO, "gpurun_out", "prof_meas")
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(meas, "bench.json"), os.path.join(dst, f"bench_{tag}_n1.json"))
    g = os.path.join(meas, "bench_2rank_gloo.json")
    if os.path.exists(g):
        shutil.copy(g, os.path.join(dst, f"bench_{tag}_2rank_gloo_rehearsal.json"))
    shutil.copy(os.path.join(meas, "pmc_latest.json"), os.path.join(dst, f"pmc_{tag}.json"))
    shutil.copy(os.path.join(meas, "pmc_latest.json"), os.path.join(REPO, "profiles", "pmc_latest.json"))
    shutil.copy(os.path.join(prof, "summary.txt"), os.path.join(dst, f"pmc_summary_{tag}.txt"))
    ks = os.path.join(meas, "rocprof_bench", "bench_kernel_stats.csv")
    shutil.copy(ks, os.path.join(dst, f"rocprof_bench_kernel_stats_{tag}.csv"))
    with open(os.path.join(meas, "bench.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    lines = ["# rocprofv3 --kernel-trace --stats of `python3 bench.py --cpu-baseline off --steps 10 --warmup 3`",
             "# (13 calls = 3 warmup + 10 timed) vs the HIP-event stage times bench.py measured in its own run",
             "", f"{'kernel':40s} {'calls':>6s} {'rocprof avg us':>15s} {'bench event avg us':>19s}"]
    with open(ks) as f:
        for row in csv.DictReader(f):
            name = re.sub(r"^void ", "", row["Name"]).split("(")[0]
            if not name.startswith("asp::"):
                continue  # torch kernels of the input generation
            name = name[5:]
            base = name.split("<")[0]
            st = bench["stages"].get(STAGE_OF.get(base, ""), {})
            ev = st.get("ms_per_launch", 0.0) * 1e3 if st.get("launches") else float("nan")
            lines.append(f"{name[:40]:40s} {int(row['Calls']):6d} {float(row['AverageNs']) / 1e3:15.1f} {ev:19.1f}")
    with open(os.path.join(dst, f"rocprof_vs_events_{tag}.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
