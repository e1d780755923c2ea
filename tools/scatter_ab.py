#!/usr/bin/env python3
"""Same-process A/B of binning settings (the record buffer keeps its placement across
calls, so the scatter's placement mode cancels): cfg3 map, env knobs switched between
calls.  Usage: python tools/scatter_ab.py 'ASP_SCATTER_GROUP=4' 'ASP_SCATTER_GROUP=8' ..."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))
import torch  # noqa: E402
from asp_amd import _lib  # noqa: E402
from asp_amd.device import project2d  # noqa: E402
from asp_amd.plummer import plummer_torch  # noqa: E402

G, n = 4096, 100_000_000
dev = torch.device("cuda:0")
d = plummer_torch(n, seed=0, h_law="pixel", extent=4.0, grid=G, device=dev)
u, v, h = d["x"], d["y"], d["h"]
a0, a1 = (d["m"] * d["T"]).contiguous(), d["m"]
o = torch.empty((2, G, G), dtype=torch.float32, device=dev)
ext = (-4.0, 4.0, -4.0, 4.0)


def run(k=5):
    for _ in range(2):
        project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext, kernel="wendland_c2",
                  ratio=True, out0=o[0], out1=o[1])
    torch.cuda.synchronize()
    _lib.profile(0, True)
    for _ in range(k):
        project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext, kernel="wendland_c2",
                  ratio=True, out0=o[0], out1=o[1])
    torch.cuda.synchronize()
    pr = _lib.profile_read(0)
    _lib.profile(0, False)
    return {k2: round(a / b, 3) for k2, (a, b) in pr.items() if b}


settings = sys.argv[1:] or ["ASP_SCATTER_GROUP=4"]
ref = None  # the first setting's maps: every other setting's maps must agree
for rep in range(3):
    for s in settings:
        env = dict(kv.split("=") for kv in s.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        r = run()
        for k, val in old.items():
            if val is None:
                os.environ.pop(k)
            else:
                os.environ[k] = val
        if ref is None:
            ref = o.clone()
            dev_ = 0.0
        else:
            dev_ = float(((o - ref).abs().max() / ref.abs().max()).item())
        print(rep, s, r, f"maxdev {dev_:.2e}", flush=True)
        if dev_ > 1e-5 and not os.environ.get("AB_NOCHECK"):
            sys.exit(f"{s}: maps differ from {settings[0]} by {dev_:.2e} x max")
