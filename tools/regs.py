#!/usr/bin/env python3
"""Register / LDS / occupancy table of the HIP kernels in one source file (gfx950).

Usage: python tools/regs.py astro-sph-tools_amd/csrc/asp_project2d.hip [name-filter ...]
"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
       "-ffp-contract=off", "-munsafe-fp-atomics", "--cuda-device-only", "-c", "-o", "/dev/null",
       src, "-Rpass-analysis=kernel-resource-usage"]
txt = subprocess.run(cmd, capture_output=True, text=True).stderr
for b in txt.split("Function Name: ")[1:]:
    name = b.split()[0]
    m = re.search(r"_ZN3asp\w*?\d+(k_\w+?)(?:ILi(\d+)ELi(\d+)ELi(\d+)E|E)", name)
    short = m.group(1) + ("<%s,%s,%s>" % m.group(2, 3, 4) if m and m.group(2) else "") if m else name
    if filt and not any(f in short for f in filt):
        continue
    get = lambda k: (re.search(k + r": (\d+)", b) or [None, "?"])[1]  # noqa: E731
    occ, lds = get(r"Occupancy \[waves/SIMD\]"), get(r"LDS Size \[bytes/block\]")
    print(f"{short:28s} vgpr {get('VGPRs'):>4} spill {get('VGPRs Spill'):>3} occ {occ:>2} lds {lds:>6}")
