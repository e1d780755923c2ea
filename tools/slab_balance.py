#!/usr/bin/env python3
"""Time each of the W Z-slab shards bench.py would give the W ranks, on ONE GPU.

    python tools/slab_balance.py [--n 1e8] [--grid 4096] [--world 8] [--out f.json]

For the pixel-h (cfg3: weighted Wendland) and physical-h (surface density, cubic) Plummer
sets: the slab edges from equal counts (zslab_bounds) and from equal modelled work
(slab_cost weights), each slab projected onto the full grid alone (warm-up + median of 3),
so the spread is the straggler cost of the 8-GPU run.
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--laws", default="pixel,physical")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from asp_amd.device import project2d
    from asp_amd.distributed import slab_cost, zslab_bounds
    from asp_amd.plummer import plummer_torch
    dev = torch.device("cuda:0")
    G, ext = a.grid, (-4.0, 4.0, -4.0, 4.0)
    res = {"n": int(a.n), "grid": G, "world": a.world, "laws": {}}
    for law in a.laws.split(","):
        d = plummer_torch(int(a.n), seed=0, h_law=law, extent=4.0, grid=G, device=dev)
        weighted = law == "pixel"
        kern = "wendland_c2" if weighted else "cubic"
        w = slab_cost(d["x"], d["y"], d["h"], ext, 8.0 / G)
        out = {}
        for mode, wts in (("count", None), ("cost", w)):
            e = zslab_bounds(d["z"], a.world, weights=wts)
            rows = []
            for r in range(a.world):
                keep = (d["z"] >= e[r]) & (d["z"] < e[r + 1])
                u, v, h = d["x"][keep], d["y"][keep], d["h"][keep]
                m = d["m"][keep]
                a0, a1 = ((m * d["T"][keep]).contiguous(), m) if weighted else (m, None)
                o0 = torch.empty((G, G), dtype=torch.float32, device=dev)
                o1 = torch.empty_like(o0) if weighted else None

                def run():
                    project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext, kernel=kern,
                              ratio=False, out0=o0, out1=o1)
                run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.reps):
                    t = time.perf_counter()
                    run()
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t) * 1e3)
                rows.append({"slab": r, "particles": int(keep.sum()), "cost": float(w[keep].sum()),
                             "ms": round(statistics.median(ts), 3)})
                print(law, mode, rows[-1], flush=True)
                del u, v, h, m, a0, a1, o0, o1
            ms = [x["ms"] for x in rows]
            out[mode] = {"edges": e, "slabs": rows, "max_ms": max(ms), "mean_ms": sum(ms) / len(ms),
                         "spread": max(ms) / (sum(ms) / len(ms)) - 1.0}
            print(law, mode, "max %.3f mean %.3f spread %.1f%%" % (
                max(ms), out[mode]["mean_ms"], 100 * out[mode]["spread"]), flush=True)
        res["laws"][law] = out
        del d, w
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
