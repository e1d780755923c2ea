#!/usr/bin/env python3
"""Profiling driver: run the bench workload a few times (no CPU baseline, no JSON).

Used under rocprofv3 (kernel trace / PMC passes):
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/prof_driver.py
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--h-law", default="pixel")
    ap.add_argument("--kernel", default="wendland_c2")
    ap.add_argument("--map", default="weighted")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--workload", default="map", choices=["map", "cube", "knn"],
                    help="cube: --n particles (physical h) -> 512^3 (bench --workload cube); "
                         "knn: k = 32 smoothing lengths of --n particles")
    a = ap.parse_args()
    import torch
    from asp_amd.device import project2d, stats
    from asp_amd.plummer import plummer_torch
    if a.workload == "cube":
        from asp_amd.device import project3d
        d = plummer_torch(a.n, seed=0, h_law="physical", extent=4.0, grid=512, device="cuda:0")
        out = torch.empty((512, 512, 512), device="cuda:0")
        for _ in range(a.iters):
            project3d(d["x"], d["y"], d["z"], d["h"], d["m"], cube_size=(512, 512, 512),
                      extent=(-4.0, 4.0) * 3, kernel=a.kernel, planes=(0, 512), out=out)
        torch.cuda.synchronize()
        return
    if a.workload == "knn":
        from asp_amd.knn import knn_smoothing_lengths
        d = plummer_torch(a.n, seed=0, h_law="pixel", extent=4.0, grid=64, device="cuda:0")
        pos = torch.stack([d["x"], d["y"], d["z"]], dim=1).double().contiguous()
        for _ in range(a.iters):
            knn_smoothing_lengths(pos, 32)
        torch.cuda.synchronize()
        return
    G = a.grid
    d = plummer_torch(a.n, seed=0, h_law=a.h_law, extent=4.0, grid=G, device="cuda:0")
    u, v, h = d["x"], d["y"], d["h"]
    if a.map == "weighted":
        a0, a1 = (d["m"] * d["T"]).contiguous(), d["m"]
    else:
        a0, a1 = d["m"], None
    out0 = torch.empty((G, G), device="cuda:0")
    out1 = torch.empty((G, G), device="cuda:0") if a1 is not None else None
    for _ in range(a.iters):
        project2d(u, v, h, a0, a1, image_size=(G, G), extent=(-4, 4, -4, 4), kernel=a.kernel,
                  ratio=a1 is not None, out0=out0, out1=out1, deterministic=a.deterministic)
    torch.cuda.synchronize()
    print("stats", stats(0), file=sys.stderr)


if __name__ == "__main__":
    main()
