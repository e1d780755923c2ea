#!/usr/bin/env python3
"""Same-process A/B of cube settings (the record buffer keeps its placement across calls,
so the scatter's placement mode cancels): 10^8 Plummer particles, physical h, 512^3
Wendland-C2 cube, env knobs switched between calls, the cubes compared with the first
setting's.  Usage: python tools/cube_ab.py 'ASP_CUBE_COMPACT=0' 'ASP_CUBE_COMPACT=1' ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))
import torch  # noqa: E402
from asp_amd import _lib  # noqa: E402
from asp_amd.device import project3d  # noqa: E402
from asp_amd.plummer import plummer_torch  # noqa: E402

C = int(os.environ.get("AB_CUBE", "512"))
n = int(float(os.environ.get("AB_N", "1e8")))
dev = torch.device("cuda:0")
d = plummer_torch(n, seed=0, h_law="physical", extent=4.0, grid=C, device=dev)
args = (d["x"], d["y"], d["z"], d["h"], d["m"])
ext = (-4.0, 4.0) * 3
out = torch.empty((C, C, C), dtype=torch.float32, device=dev)


def run(k=4):
    for _ in range(2):
        project3d(*args, cube_size=(C, C, C), extent=ext, kernel="wendland_c2", out=out)
    torch.cuda.synchronize()
    _lib.profile(0, True)
    for _ in range(k):
        project3d(*args, cube_size=(C, C, C), extent=ext, kernel="wendland_c2", out=out)
    torch.cuda.synchronize()
    pr = _lib.profile_read(0)
    _lib.profile(0, False)
    return {k2: round(a / b, 3) for k2, (a, b) in pr.items() if b}


settings = sys.argv[1:]
ref = None
for rep in range(2):
    for s in settings:
        for kv in s.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
        st = run()
        tot = round(sum(st.values()), 3)
        diff = None
        if ref is None:
            ref = out.clone()
        else:
            diff = float(((out - ref).abs().max() / ref.abs().max()).item())
        print(f"rep {rep} {s:40s} total {tot} {st} maxreldiff {diff}", flush=True)
