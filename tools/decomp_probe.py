#!/usr/bin/env python3
"""The two multi-GPU decompositions of the 2-D map, each rank's share timed on ONE GPU.

    python tools/decomp_probe.py [--n 1e8] [--grid 4096] [--world 8] [--out f.json]

SURVEY.md §8(e) / H2 ("measure both"), DESIGN.md §8:
* zslab -- the product path: rank r holds the particles of Z-slab r (equal counts) and
  projects them onto the FULL grid; a 2 x 64 MiB RCCL reduce then sums the grids.
* rows  -- image-plane ownership: rank r owns image rows [R[r], R[r+1]) (tile rows,
  balanced on the particle count), receives every particle whose 2h footprint reaches
  them (distributed.route_rows: halo duplication) and projects only its rows
  (asp_project2d_rows) with the ratio formed locally -- no grid collective.
Every share is projected alone (warm-up + median of --reps) on the weighted Wendland-C2
map of the bench (pixel-scale h).  The routing / partition itself is not timed (for
zslab it needs none; for rows it is one all-to-all of the particles per snapshot).

--interference: the zslab share of the middle rank timed alone and while a second stream
streams the reduce's HBM traffic beside it (out += in over 2 x 64 MiB fp32, k times per
map: read 2 x 128 MiB + write 128 MiB each, on CUs as RCCL's reduce kernels are), the
stand-in for the collective of map i overlapping the compute of map i + 1 (bench.py N > 1).
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))


def timed(run, reps):
    import torch
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--interference", action="store_true")
    ap.add_argument("--skip-decomp", action="store_true")
    ap.add_argument("--stages", action="store_true", help="per-stage device times of each row share")
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from asp_amd.device import project2d
    from asp_amd.distributed import route_rows, row_slabs, zslab_bounds
    from asp_amd.plummer import plummer_torch
    dev = torch.device("cuda:0")
    G, ext, W = a.grid, (-4.0, 4.0, -4.0, 4.0), a.world
    d = plummer_torch(int(a.n), seed=0, h_law="pixel", extent=4.0, grid=G, device=dev)
    a0_all = (d["m"] * d["T"]).contiguous()
    res = {"n": int(a.n), "grid": G, "world": W, "workload": "weighted Wendland-C2, pixel h"}
    full = torch.empty((2, G, G), dtype=torch.float32, device=dev)
    res["full_ms"] = round(timed(lambda: project2d(d["x"], d["y"], d["h"], a0_all, d["m"],
                                                   image_size=(G, G), extent=ext,
                                                   kernel="wendland_c2", ratio=True,
                                                   out0=full[0], out1=full[1]), a.reps), 4)
    print("full map", res["full_ms"], "ms", flush=True)
    e = zslab_bounds(d["z"], W)
    shares = {}
    if not a.skip_decomp:
        rows = []
        for r in range(W):
            keep = (d["z"] >= e[r]) & (d["z"] < e[r + 1])
            u, v, h, m = (d[k][keep].contiguous() for k in ("x", "y", "h", "m"))
            a0 = (m * d["T"][keep]).contiguous()
            ms = timed(lambda: project2d(u, v, h, a0, m, image_size=(G, G), extent=ext,
                                         kernel="wendland_c2", out0=full[0], out1=full[1]),
                       a.reps)
            rows.append({"rank": r, "particles": int(keep.sum()), "ms": round(ms, 4)})
            print("zslab", rows[-1], flush=True)
            del u, v, h, m, a0
        shares["zslab"] = rows
        R = row_slabs(G, W, d["x"], ext[:2])
        r0, r1 = route_rows(d["x"], d["h"], ext[:2], G, R)
        rows = []
        for r in range(W):
            keep = (r0 <= r) & (r1 >= r)
            u, v, h, m = (d[k][keep].contiguous() for k in ("x", "y", "h", "m"))
            a0 = (m * d["T"][keep]).contiguous()
            o0 = torch.empty((R[r + 1] - R[r], G), dtype=torch.float32, device=dev)
            o1 = torch.empty_like(o0)
            one = lambda: project2d(u, v, h, a0, m, image_size=(G, G), extent=ext,  # noqa: E731
                                    kernel="wendland_c2", ratio=True, out0=o0, out1=o1,
                                    rows=(R[r], R[r + 1]))
            ms = timed(one, a.reps)
            stages = None
            if a.stages:  # device time per stage and call (HIP events, asp_profile)
                from asp_amd import _lib
                _lib.profile(0, True)
                for _ in range(a.reps):
                    one()
                torch.cuda.synchronize()
                stages = {k: round(t / a.reps, 4) for k, (t, n) in _lib.profile_read(0).items() if n}
                _lib.profile(0, False)
            # the bench's N > 1 form: consecutive maps alternate two streams (and buffers)
            ss = [torch.cuda.Stream(device=dev) for _ in range(2)]
            ob = [(o0, o1), (torch.empty_like(o0), torch.empty_like(o1))]

            def two(k=8):
                for q in range(k):
                    with torch.cuda.stream(ss[q % 2]):
                        project2d(u, v, h, a0, m, image_size=(G, G), extent=ext,
                                  kernel="wendland_c2", ratio=True, out0=ob[q % 2][0],
                                  out1=ob[q % 2][1], rows=(R[r], R[r + 1]))
            ms2 = timed(two, a.reps) / 8
            rows.append({"rank": r, "rows": [R[r], R[r + 1]], "particles": int(keep.sum()),
                         "ms": round(ms, 4), "ms_two_streams": round(ms2, 4),
                         **({"stages_ms": stages} if stages else {})})
            print("rows", rows[-1], flush=True)
            del u, v, h, m, a0, o0, o1
        shares["rows"] = rows
        res["rows_bounds"] = R
        res["rows_duplication"] = round(sum(x["particles"] for x in rows) / int(a.n), 5)
        ms2 = [x["ms_two_streams"] for x in shares["rows"]]
        res["rows_two_streams_max_ms"] = max(ms2)
        print("rows, two streams: max %.4f mean %.4f" % (max(ms2), sum(ms2) / len(ms2)), flush=True)
        for k, rr in shares.items():
            ms = [x["ms"] for x in rr]
            res[k] = {"shares": rr, "max_ms": max(ms), "mean_ms": round(sum(ms) / len(ms), 4),
                      "ideal_speedup_vs_full": round(res["full_ms"] / max(ms), 3)}
            print(k, "max %.4f mean %.4f -> %.2fx of the full map before any collective" % (
                max(ms), res[k]["mean_ms"], res[k]["ideal_speedup_vs_full"]), flush=True)
    if a.interference:
        r = W // 2
        keep = (d["z"] >= e[r]) & (d["z"] < e[r + 1])
        u, v, h, m = (d[k][keep].contiguous() for k in ("x", "y", "h", "m"))
        a0 = (m * d["T"][keep]).contiguous()
        o = torch.empty((2, G, G), dtype=torch.float32, device=dev)
        src = torch.rand((2, G, G), dtype=torch.float32, device=dev)
        dst = torch.zeros_like(src)
        side = torch.cuda.Stream(device=dev)
        main_s = torch.cuda.current_stream(dev)
        rep = max(a.reps, 10)

        def run_map():
            project2d(u, v, h, a0, m, image_size=(G, G), extent=ext, kernel="wendland_c2",
                      out0=o[0], out1=o[1])

        def run_add(k):
            with torch.cuda.stream(side):
                for _ in range(k):
                    dst.add_(src)

        inter = {"rank": r, "particles": int(keep.sum()),
                 "map_alone_ms": round(timed(run_map, rep), 4),
                 "add_alone_ms": round(timed(lambda: (run_add(1), side.synchronize()), rep), 4)}
        for k in (1, 2, 3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            mt, at, wt = [], [], []
            for it in range(rep + 1):
                side.wait_stream(main_s)
                torch.cuda.synchronize()
                t = time.perf_counter()
                ev[0].record(main_s)
                ev[2].record(side)
                run_add(k)
                ev[3].record(side)
                run_map()
                ev[1].record(main_s)
                torch.cuda.synchronize()
                if it:
                    mt.append(ev[0].elapsed_time(ev[1]))
                    at.append(ev[2].elapsed_time(ev[3]))
                    wt.append((time.perf_counter() - t) * 1e3)
            inter[f"k{k}"] = {"map_ms": round(statistics.median(mt), 4),
                              "adds_ms": round(statistics.median(at), 4),
                              "wall_ms": round(statistics.median(wt), 4)}
            print("interference", k, inter[f"k{k}"], flush=True)
        inter["note"] = ("k adds of 2 x 64 MiB (read 256 MiB + write 128 MiB each) on a second "
                         "stream launched with the shard map; map_ms from events on the map's "
                         "stream")
        res["interference"] = inter
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
