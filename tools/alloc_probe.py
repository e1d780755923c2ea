#!/usr/bin/env python3
"""Does the scatter's time depend on where its record buffer lands?  One process, the
headline map (10^8 -> 4096^2, two maps); between trials the library's workspace is freed
(asp_release) and re-allocated, optionally after a torch allocation that shifts placement.
Prints the per-launch stage times of each trial."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))
import torch  # noqa: E402
from asp_amd import _lib  # noqa: E402
from asp_amd.device import project2d  # noqa: E402
from asp_amd.plummer import plummer_torch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
G = 4096
dev = torch.device("cuda:0")
d = plummer_torch(n, seed=0, h_law="pixel", extent=4.0, grid=G, device=dev)
u, v, h = d["x"], d["y"], d["h"]
a0, a1 = (d["m"] * d["T"]).contiguous(), d["m"]
o = torch.empty((2, G, G), dtype=torch.float32, device=dev)
ext = (-4.0, 4.0, -4.0, 4.0)
keep = []
for trial in range(int(os.environ.get("TRIALS", "6"))):
    if trial:
        _lib.check(_lib.lib().asp_release(0))
        if trial % 2 == 0 and not os.environ.get("NOSHIFT"):
            keep.append(torch.empty(int(0.35e9) * trial, dtype=torch.uint8, device=dev))
        torch.cuda.synchronize()
    for _ in range(2):
        project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext, kernel="wendland_c2",
                  ratio=True, out0=o[0], out1=o[1])
    torch.cuda.synchronize()
    _lib.profile(0, True)
    t = time.perf_counter()
    for _ in range(5):
        project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext, kernel="wendland_c2",
                  ratio=True, out0=o[0], out1=o[1])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 5 * 1e3
    pr = _lib.profile_read(0)
    _lib.profile(0, False)
    print(f"trial {trial} step {ms:.3f} ms", {k: round(a / b, 3) for k, (a, b) in pr.items() if b},
          flush=True)
