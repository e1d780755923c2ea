#!/usr/bin/env python3
"""bench.py -- headline benchmark: 10^8-particle -> 4096^2 projection on 1..8 MI355X.

Workload (BASELINE.json configs[2], the metric's "10^8-particle 4096^2 projection"):
10^8 Plummer particles -> 4096^2 mass-weighted-temperature map (sum m T W / sum m W),
Wendland-C2, fp32, pixel-scale smoothing lengths (h = 0.75 px, the HBM-bound case of
SURVEY.md §8(d)).  Inputs are generated on the device and resident in HBM before the
timed region.  With N ranks (configs[3]) the particles are Z-slab sharded (equal modelled
work) and one RCCL reduce sums the two component maps on rank 0 (strong scaling: total
work fixed); ``--decomp rows`` is the image-row alternative of SURVEY H2 ("cfg4-rows").

One "step" = one full map: binning + deposit + (N > 1) RCCL reduce + ratio.  With N > 1
the component maps are double-buffered so the reduce of map i runs on RCCL's stream while
map i + 1 is binned and deposited (``--no-pipeline``: one map at a time).

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))

METRIC = "Mpixels/s + particles/s, 10^8-particle 4096² projection at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table: peak FP32 (vector), spec
# FP64 vector: half the FP32 vector rate on gfx950 (78.6 TFLOPS, AMD's MI355X spec; the
# guide's chip table lists only FP32 -- DESIGN.md §10 measures fp64 VALU at half rate)
VALU_F64_PEAK_TFLOPS = 78.6
# flops of one squared distance (dx, dy, dz: 3; dx dx: 1; two FMAs: 4)
DIST_FLOPS = 8
# Algorithmic fp32 flops per included (pixel, particle) pair, an FMA counted as 2
# (DESIGN.md §4 "compute roofline"): dx, dy (2), r^2 = dx dx + dy dy (3), sqrt (1),
# q = r / h (1), the shape, and a * W added into each map (2 per map).
SHAPE_FLOPS = {"wendland_c2": 7, "cubic": 10, "indicator": 0}
COMPUTE_BOUND = ("gather", "wide", "cube_deposit")  # kernels priced against the VALU peak


def pair_flops(kernel, nout):
    return 8 + SHAPE_FLOPS[kernel] + 2 * nout


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    # (--particles: the same; under torch.distributed.run "--n" is ambiguous with its own
    # options and is rejected before bench.py sees it)
    ap.add_argument("--n", "--particles", dest="n", type=int, default=100_000_000)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--h-law", default="pixel", choices=["pixel", "physical"])
    ap.add_argument("--order", default="random", choices=["random", "cell"],
                    help="particle order: random (the default workload) or sorted by "
                         "64x64-pixel tile in Morton order, as a cell-ordered snapshot "
                         "(SWIFT / EAGLE files store particles by cell): an input-order "
                         "sensitivity check, not the benchmark")
    ap.add_argument("--kernel", default="wendland_c2", choices=["wendland_c2", "cubic"])
    ap.add_argument("--map", default="weighted", choices=["weighted", "surface"])
    ap.add_argument("--op", default="reduce",
                    choices=["reduce", "allreduce", "reduce_scatter", "reduce_scatter_gather"])
    ap.add_argument("--decomp", default="zslab", choices=["zslab", "rows"],
                    help="N > 1: zslab (default; north_star, BASELINE configs[3]) = each "
                         "rank's Z-slab of the particles onto the FULL grid + one RCCL "
                         "collective on the grid (--op) -- any reader split needs no "
                         "exchange; rows = each rank owns image rows, the particles are "
                         "routed to the row owners by one all-to-all from the reader's split "
                         "(timed once, reported as partition_ms), each rank projects only "
                         "its rows with the ratio formed locally, and the ratio map's slabs "
                         "are gathered (--rows-gather); DESIGN.md §8")
    ap.add_argument("--rows-gather", default="all", choices=["all", "dst"],
                    help="--decomp rows: all-gather of the ratio map's (padded) row slabs on "
                         "every rank (default), or point-to-point sends of the exact slabs to "
                         "rank 0 (over gloo with CUDA tensors this path costs ~1.2-1.4 s per "
                         "map whatever the size: a gloo artifact, DESIGN.md §8)")
    ap.add_argument("--slab-weight", default="cost", choices=["cost", "count"],
                    help="N > 1 Z-slab edges: equal modelled work (distributed.slab_cost) or "
                         "equal particle counts")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget for the bounded CPU-baseline sample")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_latest.json"),
                    help="PMC summary (tools/pmc_summary.py) for roofline.traffic")
    ap.add_argument("--deterministic", action="store_true",
                    help="int64 fixed-point accumulation (bitwise reproducible maps); "
                         "surface-density maps only (--map surface): the library refuses "
                         "fixed-point ratio maps (DESIGN.md §4)")
    ap.add_argument("--workload", default="map", choices=["map", "cube", "stage", "knn", "ion"],
                    help="map: the headline 2-D projection; cube: BASELINE configs[4], "
                         "10^8 particles -> 512^3 density cube; stage: snapshot fp64 -> "
                         "device fp32 SoA staging (SURVEY 8(f)); the last two are not the "
                         "driver's line")
    ap.add_argument("--cube", type=int, default=512, help="cube edge (voxels), --workload cube")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams the TIMED region's consecutive maps (cubes) alternate "
                         "between (each its own workspace slot in the library).  0 (auto): 1 "
                         "on one GPU -- strictly in sequence, so every kernel's event-timed "
                         "duration (the roofline) is its own, not shared with another map's "
                         "kernels; 2 for maps on N > 1 GPUs (a rank's share is small, the "
                         "scatter gated behind the previous deposit for shares <= 2e7)")
    ap.add_argument("--overlap-streams", type=int, default=2,
                    help="N = 1: after the timed region, a second timed region of --steps maps "
                         "alternating between this many streams (0/1: none), reported as "
                         "'overlapped': map i + 1's binning and scatter run beside map i's "
                         "deposit (store-bound and LDS-bound kernels sharing the CUs), the "
                         "scatter gated behind the previous map's deposit (ASP_SCATTER_GATE) "
                         "for a rank's share of <= 2e7 particles unless the environment sets "
                         "it.  Same box, round 5: 10^8 3.25 -> 3.11 ms, 5e7 1.69 -> 1.59, "
                         "2.5e7 0.94 -> 0.86, 1.25e7 (gated) 0.58 -> 0.57 (DESIGN.md §7, §18)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="N > 1: wait for each map's collective before the next map")
    ap.add_argument("--no-stage-events", dest="stage_events", action="store_false",
                    help="diagnostic: no per-stage HIP events in the timed region (no roofline)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def chunk_cull_counts(pos, h, grid, cs, extent):
    """Particles the reference's chunk cull admits into each cs x cs chunk (_projector.py:
    38-48: u in [x_lo - 2h, x_hi + 2h) on both axes), per chunk (cx * ncy + cy): the
    regressor of the CPU-baseline cost model (the reference's per-chunk work is the O(N)
    cull plus one r^2 per (pixel, admitted particle)).  A 2-D difference array: O(N)."""
    import numpy as np
    nc = grid // cs
    w = 2.0 * extent / nc
    r = 2.0 * np.abs(h)
    lo = lambda a: np.clip(np.ceil((a - r + extent) / w) - 1, 0, nc)  # noqa: E731
    hi = lambda a: np.clip(np.floor((a + r + extent) / w), -1, nc - 1)  # noqa: E731
    x0, x1, y0, y1 = lo(pos[:, 0]), hi(pos[:, 0]), lo(pos[:, 1]), hi(pos[:, 1])
    ok = (x0 <= x1) & (y0 <= y1)
    x0, x1, y0, y1 = (a[ok].astype(np.int64) for a in (x0, x1, y0, y1))
    m = nc + 1
    cnt = lambda i, j: np.bincount(i * m + j, minlength=m * m)  # noqa: E731
    d = cnt(x0, y0) - cnt(x1 + 1, y0) - cnt(x0, y1 + 1) + cnt(x1 + 1, y1 + 1)
    d = d.reshape(m, m)
    return np.cumsum(np.cumsum(d, 0), 1)[:nc, :nc].reshape(-1).astype(np.float64)


def cpu_baseline(args, extent):
    """The oracle's gather restatement of the reference path on the host cores, over a
    bounded sample of the map's 64x64 chunks (all particles culled per chunk, as the
    reference does), extrapolated to the full map with a cost model.

    Chunk costs span orders of magnitude (the Plummer core's chunks admit ~10^5 particles,
    the outskirts' a few), so a plain random sample of a few dozen chunks extrapolates
    poorly (round 3: relative standard error 0.29).  Here: every chunk's admitted-particle
    count x_c is computed (chunk_cull_counts, O(N)); the chunks are stratified by x_c and
    sampled in batches of `cores` chunks of one stratum (one chunk per thread, similar
    costs, so a batch's wall time is its chunks' cost); the batch times fit
    t = alpha + beta * x (least squares: the O(N) cull and the per-(pixel, particle) test)
    and the map's time is sum_c (alpha + beta x_c) / cores, its standard error from the
    fit's covariance."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    from asp_amd.plummer import plummer
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    t0 = time.time()
    p = plummer(args.n, seed=0, h_law=args.h_law, grid=args.grid, extent=extent)
    pos = p["pos"].astype(np.float32).astype(np.float64)
    h = p["h"].astype(np.float32).astype(np.float64)
    m = p["m"].astype(np.float32).astype(np.float64)
    T = p["T"].astype(np.float32).astype(np.float64)
    del p
    maps = [m * T, m] if args.map == "weighted" else [m]
    cs = 64
    nch = (args.grid // cs) ** 2
    x = chunk_cull_counts(pos, h, args.grid, cs, extent)
    u, v = np.ascontiguousarray(pos[:, 0]), np.ascontiguousarray(pos[:, 1])
    del pos
    img = np.zeros((args.grid, args.grid))  # shared: calls write disjoint chunks
    ext4 = [-extent, extent] * 2
    log(f"[cpu] host data + chunk counts {time.time() - t0:.1f}s; sampling with {cores} threads")

    def one_chunk(c):  # the chunk's reference-style create_image call(s), one thread
        t = time.perf_counter()
        for A in maps:
            pyoracle.create_image_cols(u, v, h, A, (args.grid, args.grid), cs, *ext4,
                                       kernel=args.kernel, nthreads=1, chunk_ids=[c], out=img)
        return time.perf_counter() - t

    rng = np.random.default_rng(0)
    S = 8  # strata: equal chunk counts, by admitted particles
    order = np.argsort(x, kind="stable")
    strata = [rng.permutation(order[k * nch // S:(k + 1) * nch // S]) for k in range(S)]
    # chunks drawn round-robin from the strata (densest stratum first, so its costly chunk
    # starts at once), fed to `cores` threads continuously: a finished chunk's thread takes
    # the next, so cheap chunks keep flowing beside an expensive one and every thread runs
    # under the contention of the full run; no new chunk starts after the budget
    # (the densest 1 % of chunks -- tens of seconds each on one thread -- are left to the
    # cost model, so the sample's wall time stays near the budget)
    cap = np.quantile(x, 0.99)
    strata = [c[x[c] <= cap] for c in strata]
    seq = [int(strata[(S - 1 - j) % S][j // S]) for j in range(nch)
           if j // S < strata[(S - 1 - j) % S].size]
    from concurrent.futures import FIRST_COMPLETED, ThreadPoolExecutor, wait  # ctypes frees the GIL
    ids, secs = [], []
    t_start = time.perf_counter()
    with ThreadPoolExecutor(cores) as pool:
        nxt = 0
        pend = {}
        while nxt < len(seq) and len(pend) < cores:
            pend[pool.submit(one_chunk, seq[nxt])] = seq[nxt]
            nxt += 1
        while pend:
            done_f, _ = wait(list(pend), return_when=FIRST_COMPLETED)
            for f in done_f:
                ids.append(pend.pop(f))
                secs.append(f.result())
            while (nxt < len(seq) and len(pend) < cores
                   and time.perf_counter() - t_start < args.cpu_seconds):
                pend[pool.submit(one_chunk, seq[nxt])] = seq[nxt]
                nxt += 1
    spent = time.perf_counter() - t_start
    ids = np.array(ids)
    secs = np.array(secs)
    done = ids.size
    X = np.stack([np.ones(done), x[ids]], axis=1)
    theta, *_ = np.linalg.lstsq(X, secs, rcond=None)
    if theta[0] < 0 or theta[1] < 0:  # a cost is never negative: one-term fits instead
        b = float(secs @ x[ids] / max(x[ids] @ x[ids], 1e-300))
        a = float(secs.mean())
        theta = np.array([0.0, b]) if theta[1] > 0 else np.array([a, 0.0])
    resid = secs - X @ theta
    cov = (resid @ resid / max(1, done - 2)) * np.linalg.pinv(X.T @ X)
    g = np.array([nch, x.sum()]) / cores  # all chunks, spread over the cores
    full_s = float(g @ theta)
    rse = float(np.sqrt(max(g @ cov @ g, 0.0)) / full_s) if full_s > 0 else None
    # a cross-check without the model: per-stratum mean chunk time x stratum size
    strat = 0.0
    for k_, c in enumerate(strata):
        got = [t for i_, t in zip(ids, secs) if i_ in set(c.tolist())] if c.size else []
        strat += (np.mean(got) if got else 0.0) * (nch // S)
    model = {"alpha_s": float(theta[0]), "beta_s_per_particle": float(theta[1]),
             "chunks_timed": int(done), "fit": "least squares, t = alpha + beta * admitted",
             "stratified_mean_mpix": round(args.grid ** 2 / (strat / cores) / 1e6, 6)
             if strat > 0 else None,
             "note": "stratified_mean excludes the densest 1 % of chunks (the model covers "
                     "them), so it is an upper bound on the rate"}
    mpix = args.grid * args.grid / full_s / 1e6
    return {"value": mpix, "unit": "Mpixels/s", "cores": cores, "kind": "port",
            "rel_stderr": None if rse is None else round(rse, 4),
            "particles_per_s": args.n / full_s, "model": model,
            "sample": f"{done} of {nch} 64x64 chunks of the {args.n:.0e}-particle "
                      f"{args.grid}^2 map, each timed on one of {cores} concurrent threads "
                      f"({len(maps)} reference-style create_image call(s) per chunk; chunks "
                      f"drawn round-robin from {S} strata by admitted particles), oracle "
                      f"gather restatement (fp64, per-chunk O(N) cull), {spent:.1f}s "
                      f"of wall time; map time = sum over all {nch} chunks of the fitted "
                      f"alpha + beta * admitted, / cores"}


def run_cube(args, world, rank, local, dev):
    """BASELINE configs[4]: N Plummer particles (physical h) -> C^3 density cube (A = m).
    With N ranks each owns C/N voxel planes; particles are routed to the slabs their
    footprints reach (halo duplication) before the timed region, the cube stays sharded."""
    import torch
    import torch.distributed as dist
    from asp_amd import _lib
    from asp_amd.device import project3d, stats
    from asp_amd.distributed import plane_slabs, route_particles
    from asp_amd.plummer import plummer_torch
    C, extent = args.cube, 4.0
    ext = (-extent, extent) * 3
    kernel = "cubic" if args.kernel == "cubic" else args.kernel
    t0 = time.time()
    d = plummer_torch(args.n, seed=0, h_law="physical", extent=extent, grid=C, device=dev)
    K = plane_slabs(C, world)
    if world > 1:
        r0, r1 = route_particles(d["z"], d["h"], ext[4:6], C, world)
        keep = (r0 <= rank) & (r1 >= rank)
        d = {k: v[keep].contiguous() for k, v in d.items()}
    x, y, z, h, m = d["x"], d["y"], d["z"], d["h"], d["m"]
    n_local = x.shape[0]
    # consecutive cubes may alternate between --streams HIP streams, each with its own
    # output and library workspace slot (one cube's scatter beside the previous cube's
    # deposit).  Default 1: the deposit's LDS brick leaves no room for a scatter workgroup
    # beside it, and on the round-5 build two streams measure no faster (14.38-14.45 vs
    # 14.35 ms)
    ns = args.streams if args.streams > 0 else 1
    streams = ([torch.cuda.current_stream(dev)] if ns == 1 else
               [torch.cuda.Stream(device=dev) for _ in range(ns)])
    outs = [torch.empty((C, C, K[rank + 1] - K[rank]), dtype=torch.float32, device=dev)
            for _ in range(ns)]
    torch.cuda.synchronize()
    if not args.quiet:
        log(f"[rank {rank}] cube data ready: {n_local} particles in {time.time() - t0:.1f}s")
    it = [0]

    def step():
        k = it[0]
        it[0] += 1
        with torch.cuda.stream(streams[k % ns]):
            project3d(x, y, z, h, m, cube_size=(C, C, C), extent=ext, kernel=kernel,
                      planes=(K[rank], K[rank + 1]), out=outs[k % ns])
        return outs[k % ns]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _lib.profile(local, True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t
    prof = _lib.profile_read(local)
    _lib.profile(local, False)
    st = stats(local)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ok = bool(torch.isfinite(out).all().item()) and float(out.abs().sum().item()) > 0
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    prof = {k: v for k, v in prof.items() if v[1]}
    dom = max(prof, key=lambda k: prof[k][0])
    dom_ms = prof[dom][0] / max(1, prof[dom][1])
    bytes_alg = args.n * 20 + C ** 3 * 4  # x, y, z, h, m + the cube (SURVEY §8(d) cfg 5)
    pairs = None
    if dom in COMPUTE_BOUND:  # untimed: the exact voxel pairs (indicator cube, summed)
        cnt = project3d(x, y, z, h, torch.ones_like(h), cube_size=(C, C, C), extent=ext,
                        kernel="indicator", planes=(K[rank], K[rank + 1]))
        pairs = float(cnt.double().sum().item())
        del cnt
    res = {
        "metric": "Mvoxels/s + particles/s, 10^8-particle 512^3 density cube",
        "value": round(C ** 3 * args.steps / elapsed / 1e6, 3), "unit": "Mvoxels/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic Plummer sphere (a=1, M=1, seed 0, physical h) generated in HBM",
        "config": {"workload": f"cfg5: {args.n:.0e} particles -> {C}^3 density cube, {kernel}, "
                               f"physical h, fp32" + (f", voxel Z-slabs x{world}" if world > 1 else ""),
                   "particles": args.n, "cube": C, "kernel": kernel, "streams": ns,
                   "parallelism": f"planes{world}" if world > 1 else "single"},
        "particles_per_s": args.n * args.steps / elapsed,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(bytes_alg / (dom_ms * 1e-3) / 1e9, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(bytes_alg / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": None, "bytes_alg_per_launch": bytes_alg},
        "stages": {k: {"ms_per_launch": ms / n, "launches": n} for k, (ms, n) in prof.items()},
        "records_per_particle": round(st["records"] / max(1, n_local), 4),
        "work_items": st["items"], "output_ok": ok,
    }
    if pairs is not None:  # compute-bound: the VALU roofline, the HBM one beside it
        F = 11 + SHAPE_FLOPS[kernel] + 2  # dx, dy, dz (3), r^2 (5), sqrt, q, shape, a W
        tf = pairs * F / (dom_ms * 1e-3) / 1e12
        res["roofline_hbm"] = res["roofline"]
        res["roofline"] = {"bound": "valu", "kernel": dom, "achieved": round(tf, 3),
                           "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(tf / VALU_PEAK_TFLOPS, 4), "included_pairs": int(pairs),
                           "flops_per_pair": F, "pairs_per_s": pairs / (dom_ms * 1e-3)}
    for key in ("roofline", "roofline_hbm"):
        fr = res.get(key, {}).get("frac")
        if fr is not None and fr > 1.0:
            log(f"bench: {key}.frac = {fr} > 1 -- not a valid measurement; no line printed")
            sys.exit(4)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_stage(args, dev):
    """the reader's fp64 arrays (positions (N, 3), h, m, T) -> the
    projector's fp32 SoA (u, v, h, m*T, m) in HBM with asp_stage_particles.  Device-resident
    inputs are the timed rate (HBM-bound: 48 B read + 20 B written per particle); the host
    path (PCIe-inclusive, chunked copies overlapped with conversion) and NumPy's host-side
    conversion (what create_image did before, the CPU baseline) are timed on a bounded
    sample of 2^24 particles."""
    import numpy as np
    import torch
    from asp_amd.stage import stage_particles
    n = args.n
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    pos = torch.rand((n, 3), generator=g, device=dev, dtype=torch.float64) * 8.0 - 4.0
    h = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 1e-3 + 1e-3
    a0 = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    a1 = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    torch.cuda.synchronize()

    def step():
        return stage_particles(pos, h, a0, a1, projection_axis=2)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / args.steps * 1e3
    bytes_alg = n * (24 + 3 * 8 + 5 * 4)
    m = min(n, 1 << 24)
    hp = [x[:m].cpu().numpy() for x in (pos, h, a0, a1)]
    stage_particles(*hp, projection_axis=2)
    torch.cuda.synchronize()
    t = time.perf_counter()
    stage_particles(*hp, projection_axis=2)
    torch.cuda.synchronize()
    host_s = time.perf_counter() - t
    t = time.perf_counter()
    f32 = [np.ascontiguousarray(hp[0][:, 0], np.float32), np.ascontiguousarray(hp[0][:, 1], np.float32)]
    f32 += [np.ascontiguousarray(x, np.float32) for x in hp[1:]]
    cpu_s = time.perf_counter() - t
    res = {
        "metric": "staged particles/s (snapshot fp64 -> device fp32 SoA)", "value": n / ms * 1e3,
        "unit": "particles/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64->f32", "data": "synthetic uniform, generated in HBM",
        "config": {"workload": f"stage: {n:.0e} particles, positions (N,3) + h + 2 fields",
                   "particles": n},
        "roofline": {"bound": "hbm", "kernel": "k_stage", "achieved": round(bytes_alg / ms / 1e6, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(bytes_alg / ms / 1e6 / HBM_PEAK_GBS, 4), "traffic": None,
                     "bytes_alg_per_launch": bytes_alg},
        "host_path": {"particles": m, "seconds": round(host_s, 4),
                      "GB_per_s_pcie_inclusive": round(m * 48 / host_s / 1e9, 2)},
        "cpu_baseline": {"value": m / cpu_s, "unit": "particles/s", "cores": 1, "kind": "port",
                         "sample": f"NumPy column select + astype(float32) of {m} particles "
                                   "(the host-side conversion create_image performs)"},
    }
    print(json.dumps(res), flush=True)


def run_knn(args, dev):
    """h = distance to the 32nd nearest neighbour (the reference's
    scipy KDTree query, io/SWIFT/_SnapshotSWIFT.py:62-83) for N Plummer particles, inputs
    in HBM.  CPU baseline: scipy KDTree build + query (one thread, as the reference calls
    it) on a bounded random sample.

    Roofline (VALU): the search kernel evaluates squared distances -- fp32 ones in the
    curve-window pass (the prefilter; exact fp64 only for the few candidates) and fp64
    ones in the cell scans, fp32 ones (every lane of a wave) in the shared cell pass --
    counted in one untimed diagnostic call (ASP_KNN_COUNT), 8
    flops each; the time that work needs at the FP32 / FP64 vector peaks, over the search
    kernel's HIP-event time in the timed steps, is the fraction."""
    import numpy as np
    import torch
    from asp_amd import _lib
    from asp_amd.device import stats
    from asp_amd.knn import knn_smoothing_lengths
    from asp_amd.plummer import plummer_torch
    d = plummer_torch(args.n, seed=0, h_law="pixel", extent=4.0, grid=64, device=dev)
    pos = torch.stack([d["x"], d["y"], d["z"]], dim=1).double().contiguous()
    del d
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        knn_smoothing_lengths(pos, 32)
    torch.cuda.synchronize()
    local = dev.index or 0
    _lib.profile(local, True)
    t = time.perf_counter()
    for _ in range(args.steps):
        h = knn_smoothing_lengths(pos, 32)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / args.steps * 1e3
    prof = {k: v for k, v in _lib.profile_read(local).items() if v[1]}
    _lib.profile(local, False)
    ok = bool(torch.isfinite(h).all().item()) and float(h.min().item()) > 0
    # untimed: the distances the search evaluates (one atomic per lane while counting)
    os.environ["ASP_KNN_COUNT"] = "1"
    try:
        h2 = knn_smoothing_lengths(pos, 32)
        torch.cuda.synchronize()
        st = stats(local)
    finally:
        del os.environ["ASP_KNN_COUNT"]
    same = bool(torch.equal(h, h2))
    # window (fp32), cell scans (fp64), the shared cell pass's entries (fp32, every lane)
    e32, e64 = float(st["evals"]), float(st["evals_small"])
    eshared = float(st["evals_gather"]) * 64
    e32 += eshared
    s_ms = prof["knn_search"][0] / max(1, prof["knn_search"][1]) if "knn_search" in prof else None
    roof = None
    if s_ms:
        t_peak = (e32 * DIST_FLOPS / (VALU_PEAK_TFLOPS * 1e12)
                  + e64 * DIST_FLOPS / (VALU_F64_PEAK_TFLOPS * 1e12))
        flops = (e32 + e64) * DIST_FLOPS
        roof = {"bound": "valu", "kernel": "knn_search",
                "achieved": round(flops / (s_ms * 1e-3) / 1e12, 3),
                "peak": round(flops / t_peak / 1e12, 3), "unit": "TFLOP/s",
                "frac": round(t_peak / (s_ms * 1e-3), 4),
                "distances_fp32": int(e32), "distances_fp64": int(e64),
                "distances_shared_pass": int(eshared),
                "topk_insertions_per_particle": round(float(st["evals_wide"]) / args.n, 1),
                "distances_per_particle": round((e32 + e64) / args.n, 1),
                "flops_per_distance": DIST_FLOPS,
                "kernel_ms_per_step": round(s_ms, 4),
                "peak_note": f"work-weighted peak: fp32 distances at {VALU_PEAK_TFLOPS}, fp64 "
                             f"at {VALU_F64_PEAK_TFLOPS} TFLOP/s; frac = time at those peaks "
                             f"/ the search kernel's event time"}
    res = {
        "metric": "k-NN smoothing lengths/s (k = 32, fp64, bit-exact vs scipy KDTree)",
        "value": args.n / ms * 1e3, "unit": "particles/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic Plummer sphere (a=1, seed 0) generated in HBM",
        "config": {"workload": f"knn: {args.n:.0e} particles, k = 32", "particles": args.n},
        "stages": {k: {"ms_per_launch": a / b, "launches": b} for k, (a, b) in prof.items()},
        "output_ok": ok and same,
    }
    if roof is not None:
        res["roofline"] = roof
    if args.cpu_baseline != "off":
        from scipy.spatial import KDTree
        m = min(args.n, 1 << 20)
        sample = pos[torch.randperm(args.n, device=dev)[:m]].cpu().numpy()
        t = time.perf_counter()
        KDTree(sample).query(sample, k=32)
        cpu_s = time.perf_counter() - t
        res["cpu_baseline"] = {"value": m / cpu_s, "unit": "particles/s", "cores": 1,
                               "kind": "reference",
                               "sample": f"scipy KDTree build + query(k=32) of {m} random "
                                         f"particles of the set (the reference's call)"}
    print(json.dumps(res), flush=True)


def run_ion(args, dev):
    """per-particle ion masses m * X * 10^f_ion(log10 n_H, log10 T, z)
    for an ion column map -- the reference's IonisationTableBase.evaluate_at_redshift
    (data_structures/_IonisationTable.py:54-58, scipy RegularGridInterpolator) fused with
    the mass product, inputs in HBM.  Table: HM01-shaped 41 x 141 x 49 fp64 (synthetic
    values; the HDF5 tables are not in the repo).  Algorithmic bytes per particle: 16 (n_H,
    T) + 16 (m, X) + 8 (out) = 40 B; the table stays in cache.  CPU baseline: the
    reference's call (scipy RGI at a redshift, one thread) on a bounded sample."""
    import numpy as np
    import torch
    from asp_amd.ionisation import IonisationTable, ion_masses
    n = args.n
    rng = np.random.default_rng(0)
    shape = (41, 141, 49)
    axes = [np.linspace(-8.0, 0.0, shape[0]), np.linspace(2.0, 9.0, shape[1]),
            np.concatenate([np.linspace(0.0, 1.0, 21), np.linspace(1.1, 9.0, 28)])]
    table = rng.uniform(-12.0, 0.0, shape)
    tab = IonisationTable(table, *axes, redshift_input_index=2)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    state = torch.rand((n, 2), generator=g, device=dev, dtype=torch.float64)
    state[:, 0] = state[:, 0] * 9.0 - 8.5          # a few points outside the table -> -inf
    state[:, 1] = state[:, 1] * 7.0 + 2.0
    m = torch.rand(n, generator=g, device=dev, dtype=torch.float64) + 0.5
    X = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 0.2 + 0.6
    z = 2.25
    torch.cuda.synchronize()

    def step():
        return tab._run(state, 2, z, 2, m, X)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / args.steps * 1e3
    bytes_alg = n * 40
    k = min(n, 1 << 16)
    chk = out[:k].cpu().numpy()
    s_h = state[:k].cpu().numpy()
    from scipy.interpolate import RegularGridInterpolator
    rgi = RegularGridInterpolator(axes, table, bounds_error=False, fill_value=-np.inf)
    P = np.empty((k, 3))
    P[:, :2] = s_h
    P[:, 2] = z
    want = (m[:k].cpu().numpy() * X[:k].cpu().numpy()) * 10.0 ** rgi(P)
    ok = bool(np.allclose(chk, want, rtol=4.5e-16, atol=0))
    res = {
        "metric": "ion masses/s (m * X * f_ion from a 3-D ionisation table, fp64)",
        "value": n / ms * 1e3, "unit": "particles/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic gas states and HM01-shaped table (41x141x49), generated in HBM",
        "config": {"workload": f"ion: {n:.0e} particles, HM01-shaped table at z = {z}",
                   "particles": n},
        "roofline": {"bound": "hbm", "kernel": "k_table_slab", "achieved": round(bytes_alg / ms / 1e6, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(bytes_alg / ms / 1e6 / HBM_PEAK_GBS, 4), "traffic": None,
                     "bytes_alg_per_launch": bytes_alg},
        "output_ok": ok,
    }
    if args.cpu_baseline != "off":
        c = min(n, 1 << 22)
        s_c = state[:c].cpu().numpy()
        mc, Xc = m[:c].cpu().numpy(), X[:c].cpu().numpy()
        t = time.perf_counter()
        Pc = np.empty((c, 3))
        Pc[:, :2] = s_c
        Pc[:, 2] = z
        (mc * Xc) * 10.0 ** rgi(Pc)
        cpu_s = time.perf_counter() - t
        res["cpu_baseline"] = {"value": c / cpu_s, "unit": "particles/s", "cores": 1,
                               "kind": "reference",
                               "sample": f"scipy RegularGridInterpolator at a redshift (the "
                                         f"reference's call) + mass product on {c} particles"}
    print(json.dumps(res), flush=True)


def pair_work(u, v, h, G, ext, kernel, world, dev):
    """Untimed: the map's exact included pairs (the indicator kernel's per-pixel neighbour
    counts, summed; every pixel's count is exact in fp32 below 2^24) and the (pixel,
    particle) lane-slots the deposit kernels spend (the library's ASP_COUNT_EVALS
    diagnostic), of this rank's particles."""
    import torch
    import torch.distributed as dist
    from asp_amd.device import project2d, stats
    ones = torch.ones_like(h)
    cnt, _ = project2d(u, v, h, ones, image_size=(G, G), extent=ext, kernel="indicator")
    os.environ["ASP_COUNT_EVALS"] = "1"
    try:
        project2d(u, v, h, ones, image_size=(G, G), extent=ext, kernel=kernel)
        torch.cuda.synchronize()
        st = stats(dev.index or 0)
    finally:
        del os.environ["ASP_COUNT_EVALS"]
    del world, dist  # per rank: priced against this rank's own kernel time
    return [float(cnt.double().sum().item()), float(st["evals"]), float(st["evals_small"]),
            float(st["evals_gather"]), float(st["evals_wide"])]


def valu_roofline(valu, kernel, nout, dom, dom_ms, pm_stage):
    """The compute bound of SURVEY §8(d): included pairs x algorithmic flops per pair over
    the dominant kernel's time, against the FP32 vector peak (157.3 TFLOPS)."""
    pairs, evals, ev_small, ev_gather, ev_wide = valu
    F = pair_flops(kernel, nout)
    tflops = pairs * F / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else 0.0
    r = {"bound": "valu", "kernel": dom, "achieved": round(tflops, 3), "peak": VALU_PEAK_TFLOPS,
         "unit": "TFLOP/s", "frac": round(tflops / VALU_PEAK_TFLOPS, 4),
         "included_pairs": int(pairs), "evaluated_lane_pairs": int(evals),
         "evaluated_per_included": round(evals / pairs, 3) if pairs else None,
         "evaluated_split": {"small_mid": int(ev_small), "gather": int(ev_gather),
                             "wide": int(ev_wide)},
         "flops_per_pair": F, "pairs_per_s": pairs / (dom_ms * 1e-3) if dom_ms > 0 else None,
         "note": "pairs and flops of the whole map (all deposit kernels) over the dominant "
                 "kernel's time: an upper bound on that kernel's rate"}
    if pm_stage and "SQ_INSTS_VALU" in pm_stage and pairs:
        r["valu_lane_instr_per_pair"] = round(pm_stage["SQ_INSTS_VALU"] * 64 / pairs, 3)
        r["valu_lane_instr_source"] = "SQ_INSTS_VALU of the dominant kernel (PMC pass) x 64"
    return r


def workload_tag(n, grid, world, rows):
    """BASELINE.json configs: [1] 10^7 -> 2048^2 surface density, [2] 10^8 -> 4096^2
    weighted map (the metric's), [3] the same Z-slab-decomposed on N GPUs with one grid
    collective; the image-row decomposition is NOT configs[3] ("cfg4-rows"); anything
    else is a custom size."""
    if n == 100_000_000 and grid == 4096:
        return "cfg3" if world == 1 else ("cfg4-rows" if rows else "cfg4")
    if n == 10_000_000 and grid == 2048:
        return "cfg2"
    return "custom"


def output_check(out0, out1, a0, a1, ratio, world=1, gathered_ratio=False):
    """Size-independent sanity of the timed map (the parity proper is tests/): finite,
    non-negative component sums (W >= 0, m > 0), and for the mass-weighted map every pixel a
    weighted MEAN of particle temperatures -- inside [min T, max T] wherever sum m W > 0,
    exactly 0 elsewhere."""
    import torch
    lo = hi = None
    if ratio:  # the collective first: every rank reaches it whatever its own checks say
        t = a0 / a1
        rng = torch.stack([-t.min(), t.max()]).double()
        if world > 1:  # the reduced map averages every rank's particles
            import torch.distributed as dist
            dist.all_reduce(rng, op=dist.ReduceOp.MAX)
        lo, hi = -float(rng[0].item()), float(rng[1].item())
    if not bool(torch.isfinite(out0).all().item()):
        return False
    if not ratio:
        return bool((out0 >= 0).all().item()) and float(out0.sum().item()) > 0
    if gathered_ratio:  # reduce_scatter_gather: out0 is the all-gathered ratio map, out1
        out1 = out0     # this rank's own (unreduced) component: coverage from out0 itself
    if not bool(torch.isfinite(out1).all().item()) or not bool((out1 >= 0).all().item()):
        return False
    cov = out1 > 0
    inside = (out0[cov] >= lo * (1 - 1e-5)) & (out0[cov] <= hi * (1 + 1e-5))
    return (bool(cov.any().item()) and bool(inside.all().item())
            and bool((out0[~cov] == 0).all().item()))


def main():
    args = parse()
    if args.deterministic and args.map == "weighted" and args.workload == "map":
        log("bench: --deterministic needs --map surface (a ratio of fixed-point components "
            "is imprecise in kernel-tail pixels; the library refuses it, DESIGN.md §4)")
        sys.exit(2)
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    local = local % max(1, torch.cuda.device_count())  # 1-GPU rehearsal of N ranks
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    backend_label = None
    if world > 1:
        backend = os.environ.get("ASP_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        backend_label = "RCCL" if backend == "nccl" else f"{backend} (rehearsal, not RCCL)"
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal only (several ranks sharing one GPU cannot use RCCL)
            dist.init_process_group(backend)
    from asp_amd import _lib
    from asp_amd.device import project2d, stats
    from asp_amd.distributed import project2d_sharded, zslab_bounds
    from asp_amd.plummer import plummer_torch

    if args.workload == "cube":
        return run_cube(args, world, rank, local, dev)
    if args.workload == "stage":
        return run_stage(args, dev)
    if args.workload == "ion":
        return run_ion(args, dev)
    if args.workload == "knn":
        return run_knn(args, dev)
    G, extent = args.grid, 4.0
    ext = (-extent, extent, -extent, extent)
    t0 = time.time()
    d = plummer_torch(args.n, seed=0, h_law=args.h_law, extent=extent, grid=G, device=dev)
    if args.order == "cell":  # cell-ordered input (the particles' tile, Morton order)
        tx = ((d["x"] + extent) * (G / (2 * extent))).long().clamp(0, G - 1) >> 6
        ty = ((d["y"] + extent) * (G / (2 * extent))).long().clamp(0, G - 1) >> 6
        key = torch.zeros_like(tx)
        for b in range(12):  # interleave the tile coordinates' bits
            key |= ((tx >> b) & 1) << (2 * b + 1) | ((ty >> b) & 1) << (2 * b)
        perm = torch.argsort(key)
        d = {k: v[perm].contiguous() for k, v in d.items()}
        del tx, ty, key, perm
    R = None  # --decomp rows: the row-slab bounds
    partition_ms = None  # --decomp rows: the timed all-to-all from the reader's split
    rows_got = None
    if world > 1:
        from asp_amd.distributed import exchange_rows, row_slabs, slab_cost
        if args.decomp == "rows":
            # The reader's split (_SnapshotEAGLE.py:120-130): a contiguous 1/W of the
            # particles per rank, with no spatial order.  The row bounds balance the union
            # of all ranks' particles (one all-reduce of a row histogram), then ONE
            # all-to-all sends every particle to the ranks whose rows its 2h footprint
            # reaches -- timed: the per-snapshot cost the row decomposition adds.
            lo_, hi_ = args.n * rank // world, args.n * (rank + 1) // world
            d = {k: v[lo_:hi_].contiguous() for k, v in d.items()}
            w = None if args.slab_weight == "count" else slab_cost(d["x"], d["y"], d["h"], ext, 2 * extent / G)
            R = row_slabs(G, world, d["x"], ext[:2], weights=w, group=dist.group.WORLD)
            del w
            cols = [d["x"], d["y"], d["h"]] + ([(d["m"] * d["T"]).contiguous(), d["m"]]
                                               if args.map == "weighted" else [d["m"]])
            torch.cuda.synchronize()
            dist.barrier()
            t_ex = time.perf_counter()
            rows_got = exchange_rows(cols, d["x"], d["h"], u_extent=ext[:2], nx=G, bounds=R)
            torch.cuda.synchronize()
            pt = torch.tensor([time.perf_counter() - t_ex], dtype=torch.float64, device=dev)
            dist.all_reduce(pt, op=dist.ReduceOp.MAX)
            partition_ms = float(pt.item()) * 1e3
            del cols, d
            d = {"x": rows_got[0], "y": rows_got[1], "h": rows_got[2]}
        else:
            # Z-slabs: any reader split sums to the same map, so no exchange is needed; the
            # slabs (equal modelled work) only balance the ranks
            w = None if args.slab_weight == "count" else slab_cost(d["x"], d["y"], d["h"], ext, 2 * extent / G)
            e = zslab_bounds(d["z"], world, weights=w)
            keep = (d["z"] >= e[rank]) & (d["z"] < e[rank + 1])
            del w
            d = {k: v[keep].contiguous() for k, v in d.items()}
    u, v, h = d["x"], d["y"], d["h"]
    if rows_got is not None:  # the routed columns as exchanged
        a0, a1 = rows_got[3], (rows_got[4] if args.map == "weighted" else None)
        del rows_got
    elif args.map == "weighted":
        a0, a1 = (d["m"] * d["T"]).contiguous(), d["m"]
        del d["z"], d["T"]
    else:
        a0, a1 = d["m"], None
        del d["z"], d["T"]
    n_local = u.shape[0]
    torch.cuda.synchronize()
    if not args.quiet:
        log(f"[rank {rank}] data ready: {n_local} particles in {time.time() - t0:.1f}s")

    ratio = args.map == "weighted"
    # both component maps in one allocation: N > 1 sums them with ONE RCCL collective.
    # N > 1 double-buffers them: the collective of map i (RCCL's stream) overlaps the
    # binning + deposit of map i + 1 (compute stream); map i + 2 reuses map i's buffer
    # only after its collective (stream-ordered wait).
    # Consecutive maps alternate between --streams HIP streams (each with its own output
    # buffer; the library gives each stream its own workspace slot): the binning of map
    # i + 1 runs beside the deposit of map i.  The timed region uses
    # --streams (default 1); a second timed region uses --overlap-streams (default 2).
    gate_env = os.environ.get("ASP_SCATTER_GATE")  # set by the caller: kept as is

    def set_gate(n):
        """ASP_SCATTER_GATE for a region on n streams (auto: small shares only)."""
        if gate_env is None:
            os.environ["ASP_SCATTER_GATE"] = "1" if (n > 1 and n_local <= 20_000_000) else "0"
        return n > 1 and os.environ.get("ASP_SCATTER_GATE", "0") not in ("", "0")

    stream_sets = {}

    def stream_set(n):
        if n not in stream_sets:
            stream_sets[n] = ([torch.cuda.current_stream(dev)] if n == 1 else
                              [torch.cuda.Stream(device=dev) for _ in range(n)])
        return stream_sets[n]

    # auto: one stream on one GPU (the roofline's kernel durations are then the kernels'
    # own); two on N > 1, where the line is a scaling point and a rank's share is small
    # (1.25e7: 0.618 -> 0.538 ms gated, profiles/r05/seq_main/).  The second, overlapped
    # region runs on one GPU only: at N > 1 the timed region itself already overlaps maps.
    ns = args.streams if args.streams > 0 else (1 if world == 1 else 2)
    nso = args.overlap_streams if (args.overlap_streams > 1 and world == 1) else 0
    mode = {"ns": ns, "streams": stream_set(ns)}
    gated = set_gate(ns)
    nbuf = max(ns, nso, 2 if (world > 1 and args.pipeline) else 1)
    bufs = [torch.empty((2 if a1 is not None else 1, G, G), dtype=torch.float32, device=dev)
            for _ in range(nbuf)]
    pending = [None]
    it = [0]
    last = [None]  # the last completed map's (out0, out1) as the collective returns them

    if R is not None:  # row slabs: this rank's rows, then the ratio map gathered
        rmax = max(R[i + 1] - R[i] for i in range(world))
        my_rows = R[rank + 1] - R[rank]
        if args.rows_gather == "all":  # all-gather (equal sizes: slabs padded to rmax)
            sends = [torch.zeros((rmax, G), dtype=torch.float32, device=dev) for _ in range(nbuf)]
            fulls = [torch.empty((world * rmax, G), dtype=torch.float32, device=dev)
                     for _ in range(nbuf)]
        else:  # to rank 0 over point-to-point sends of the exact slabs (the reduce's analogue)
            fulls = [torch.empty((G, G), dtype=torch.float32, device=dev) for _ in range(nbuf)]
            sends = [f[R[rank]:R[rank + 1]] for f in fulls]

    class _Gathered:  # the gather of one map's row slabs, waited for stream-ordered
        def __init__(self, works, full, comp):
            self.works, self.full, self.comp = works, full, comp

        def wait(self):
            for w in self.works:
                w.wait()
            self.works = []
            return self.full, self.comp

    def gather_rows(b):
        """Post the gather of buffer b's ratio map: all-gather, or p2p slabs to rank 0."""
        if args.rows_gather == "all":
            return [dist.all_gather_into_tensor(fulls[b], sends[b], async_op=True)]
        if rank != 0:
            ops = [dist.P2POp(dist.isend, sends[b], 0)]
        else:
            ops = [dist.P2POp(dist.irecv, fulls[b][R[r]:R[r + 1]], r) for r in range(1, world)]
        return dist.batch_isend_irecv(ops)

    def step(pipelined=world > 1 and args.pipeline):
        k = it[0]
        it[0] += 1
        maps = bufs[k % nbuf]
        o0, o1 = maps[0], (maps[1] if a1 is not None else None)
        with torch.cuda.stream(mode["streams"][k % mode["ns"]]):
            if R is not None:
                # this rank's rows (ratio formed locally: its rows' sums are complete), then
                # ONE all-gather of the single map -- no grid reduction
                s0 = sends[k % nbuf][:my_rows]
                s1 = o1[:my_rows] if o1 is not None else None
                project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext, kernel=args.kernel,
                          ratio=ratio, out0=s0, out1=s1, deterministic=args.deterministic,
                          rows=(R[rank], R[rank + 1]))
                p = _Gathered(gather_rows(k % nbuf), fulls[k % nbuf], s1)
                if not pipelined:
                    last[0] = p.wait()
            elif world > 1:
                p = project2d_sharded(u, v, h, a0, a1, image_size=(G, G), extent=ext,
                                      kernel=args.kernel, ratio=ratio, op=args.op, out0=o0,
                                      out1=o1, deterministic=args.deterministic,
                                      async_op=pipelined)
            else:
                last[0] = project2d(u, v, h, a0, a1, image_size=(G, G), extent=ext,
                                    kernel=args.kernel, ratio=ratio, out0=o0, out1=o1,
                                    deterministic=args.deterministic)
        if world > 1 and not (R is not None and not pipelined):
            if pipelined:
                if pending[0] is not None:
                    # map k - 1's collective: the stream that next writes its buffer (map
                    # k - 1 + nbuf) waits for it -- stream-ordered, no host block
                    with torch.cuda.stream(mode["streams"][(k - 1 + nbuf) % mode["ns"]]):
                        last[0] = pending[0].wait()
                pending[0] = p
            else:
                last[0] = p

    def drain():
        if pending[0] is not None:
            with torch.cuda.stream(mode["streams"][(it[0] - 1) % mode["ns"]]):
                last[0] = pending[0].wait()
            pending[0] = None

    # The warm-up maps carry HIP events around every stage (the library's asp_profile): they
    # name the dominant kernel.  The timed steps then carry events around THAT kernel only
    # (asp_profile_stages), on the stream it runs on: its duration, and so the roofline,
    # comes from the timed steps themselves, while the other stages' event pairs -- about
    # 4-5 us each between dependent launches, 9 % of a 1.25e7-particle share's step and
    # 2 % of the 10^8 map (round 6, profiles/r06/t5/) -- stay out of the timed region.  The
    # per-stage breakdown comes from a separate region after it (every stage marked).
    # The first warm-up map runs unmarked: it loads the kernels' code objects and runs the
    # record-placement trials, whose times would make any stage look dominant.
    step()
    drain()
    torch.cuda.synchronize()
    _lib.profile(local, args.stage_events)
    for _ in range(max(1, args.warmup - 1)):
        step()
    drain()
    torch.cuda.synchronize()
    warm = {k: v for k, v in _lib.profile_read(local).items() if v[1]}
    dom = max(warm, key=lambda k: warm[k][0]) if warm else None  # most device time
    if args.stage_events and dom is not None:
        _lib.profile(local, True, stages=[dom])
    else:
        _lib.profile(local, False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t
    out0, out1 = last[0]
    prof = _lib.profile_read(local)  # timed region: the dominant stage's events
    _lib.profile(local, False)
    launched = {k: v for k, v in prof.items() if v[1]}
    if not launched or dom not in launched:
        log("bench: no stage events in the timed region (--no-stage-events): no roofline")
        launched = {"none": (0.0, 0)}
        dom = "none"
    # N > 1: the single-map LATENCY as well (each map's collective completed before the
    # next map starts), beside the overlapped throughput of the timed region
    latency_ms = None
    if nbuf > 1:
        k_lat = max(1, min(args.steps, 5))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tl = time.perf_counter()
        for _ in range(k_lat):
            step(pipelined=False)
            torch.cuda.synchronize()
        tt = torch.tensor([time.perf_counter() - tl], dtype=torch.float64, device=dev)
        if world > 1:
            dist.barrier()
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        latency_ms = float(tt.item()) / k_lat * 1e3
        out0, out1 = last[0]
    st = stats(local)
    valu = None
    if dom in COMPUTE_BOUND:
        valu = pair_work(u, v, h, G, ext, args.kernel, world, dev)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # reduce_scatter: out0 / out1 are this rank's reduced row slab (ratio formed there)
    if R is not None:  # the gathered row slabs -> the full map (rank 0; every rank: "all")
        if args.rows_gather == "all":
            out0 = torch.cat([out0[r * rmax:r * rmax + R[r + 1] - R[r]] for r in range(world)])
        elif rank != 0:
            out0 = out0[R[rank]:R[rank + 1]]  # (the rest of its buffer was never written)
        out1 = None
    ok = output_check(out0, out1, a0, a1, ratio, world,
                      gathered_ratio=world > 1 and (args.op == "reduce_scatter_gather"
                                                    or R is not None))
    # the per-stage breakdown: a separate region of maps with every stage marked (untimed)
    k_bd = max(1, min(args.steps, 10))
    breakdown = {}
    if args.stage_events:
        drain()
        torch.cuda.synchronize()
        _lib.profile(local, True)
        for _ in range(k_bd):
            step()
        drain()
        torch.cuda.synchronize()
        breakdown = {k: v for k, v in _lib.profile_read(local).items() if v[1]}
        _lib.profile(local, False)
    overlapped = None
    if nso:
        # Second timed region: the same maps alternating between nso streams (throughput of
        # the overlapped pipeline; no stage events, so the kernels run undisturbed).  Its
        # kernels share the CUs with the other stream's, so their durations say nothing
        # about any one kernel: the roofline above is the sequential region's.
        drain()
        torch.cuda.synchronize()
        mode["ns"], mode["streams"] = nso, stream_set(nso)
        gated_o = set_gate(nso)
        for _ in range(args.warmup):
            step()
        drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        to = time.perf_counter()
        for _ in range(args.steps):
            step()
        drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tt = torch.tensor([time.perf_counter() - to], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el_o = float(tt.item())
        o0, o1 = last[0]
        if R is not None:
            if args.rows_gather == "all":
                o0 = torch.cat([o0[r * rmax:r * rmax + R[r + 1] - R[r]] for r in range(world)])
            elif rank != 0:
                o0 = o0[R[rank]:R[rank + 1]]
            o1 = None
        ok_o = output_check(o0, o1, a0, a1, ratio, world,
                            gathered_ratio=world > 1 and (args.op == "reduce_scatter_gather"
                                                          or R is not None))
        overlapped = {"streams": nso, "scatter_gate": gated_o,
                      "ms_per_step": round(el_o / args.steps * 1e3, 4),
                      "value": round(G * G * args.steps / el_o / 1e6, 3), "unit": "Mpixels/s",
                      "output_ok": ok_o,
                      "note": f"a second timed region of {args.steps} maps (after {args.warmup} "
                              f"warm-up maps) alternating between {nso} HIP streams, each with "
                              "its own workspace slot and output buffer: map i + 1's binning "
                              "and scatter run beside map i's deposit.  Throughput of the "
                              "overlapped pipeline; 'value' and the roofline are the "
                              "sequential region's"}
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    ms_step = elapsed / args.steps * 1e3
    mpix = G * G * args.steps / elapsed / 1e6
    pps = args.n * args.steps / elapsed
    nout = 2 if a1 is not None else 1
    b_p = 4 * (3 + nout)  # u, v, h + one property per output map
    bytes_alg = n_local * b_p + nout * G * G * 4
    stages = {k: {"ms_per_launch": (ms / n if n else 0.0), "launches": n,
                  "ms_per_step": ms / k_bd}
              for k, (ms, n) in breakdown.items() if n}
    # Dominant kernel = most device time over the timed steps, its duration per step from
    # the same HIP events (one launch per step unless the map runs as windows / batches).
    dom_ms = launched[dom][0] / args.steps
    achieved = bytes_alg / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic = None
    traffic_src = None
    pm_stage = None
    try:
        with open(args.pmc) as f:
            pm = json.load(f)
        # per-rank traffic: keyed on THIS rank's particle count (a profile of the shard)
        key = f"n{n_local}_g{G}_{args.kernel}_{args.h_law}_{args.map}"
        if key in pm and dom in pm[key]:
            pm_stage = pm[key][dom]
            traffic = pm_stage.get("hbm_bytes_per_launch")
            traffic_src = pm[key].get("source")
    except (OSError, ValueError, KeyError):
        pass
    cfg_tag = workload_tag(args.n, G, world, R is not None)
    res = {
        "metric": METRIC, "value": round(mpix, 3), "unit": "Mpixels/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic Plummer sphere (a=1, M=1, seed 0) generated in HBM",
        "config": {"workload": f"{cfg_tag}: {args.n:.0e} particles -> {G}^2 "
                               f"{'mass-weighted temperature' if ratio else 'surface density'} "
                               f"map, {args.kernel}, {args.h_law}-scale h, fp32"
                               + ((f", Z-slab x{world} + {backend_label} {args.op}"
                                   if R is None else
                                   f", image row slabs x{world} + {backend_label} "
                                   + ("all-gather" if args.rows_gather == "all"
                                      else "gather to rank 0"))
                                  if world > 1 else ""),
                   "particles": args.n, "grid": G, "kernel": args.kernel, "h_law": args.h_law,
                   "map": args.map, **({"order": "cell"} if args.order == "cell" else {}),
                   "parallelism": (f"zslab{world}" if R is None else f"rows{world}")
                   if world > 1 else "single",
                   **({"backend": backend_label, "decomp": args.decomp,
                       **({"row_bounds": R} if R is not None else {})} if world > 1 else {}),
                   "accumulation": "int64 fixed point" if args.deterministic else "fp64",
                   "collective_overlap": world > 1 and args.pipeline,
                   "streams": ns, "scatter_gate": gated,
                   **({"slab_weight": args.slab_weight,
                       "collective": args.op if R is None else
                       ("all_gather" if args.rows_gather == "all" else "p2p_gather"),
                       "partition": ("Z-slab split of the generated particles before the "
                                     "timed region (only balances the ranks: any reader "
                                     "split sums to the same map, so none is needed)"
                                     if R is None else
                                     "from a reader split (a contiguous 1/W per rank), one "
                                     "all-to-all routes every particle to the ranks whose "
                                     "rows its 2h footprint reaches "
                                     "(distributed.exchange_rows): once per snapshot, "
                                     "before the timed region, timed as partition_ms")}
                    if world > 1 else {})},
        **({"partition_ms": round(partition_ms, 3),
            "partition_note": "the rows decomposition's per-snapshot all-to-all (max over "
                              "ranks); amortised over the maps made from one snapshot"}
           if partition_ms is not None else {}),
        "particles_per_s": pps,
        **({"latency_ms_per_map": round(latency_ms, 4),
            "latency_note": "one map at a time, synchronised (no overlap of maps): binning + "
                            "deposit (+ collective) + ratio, max over ranks"}
           if latency_ms else {}),
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "bytes_alg_per_launch": bytes_alg,
                     "kernel_ms_per_step": round(dom_ms, 4),
                     "kernel_launches_timed": launched[dom][1],
                     "pipeline_frac": round(bytes_alg / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     **({"concurrency_note": f"maps alternate between {ns} HIP streams: this "
                         "kernel's launches run beside the other stream's kernels (the "
                         "previous map's deposit), so its per-launch time includes sharing "
                         "the CUs and HBM; pipeline_frac (the whole map per step) is the "
                         "measure of the overlapped pipeline"} if ns > 1 else {})},
        **({"overlapped": overlapped} if overlapped else {}),
        "stages": stages,
        "stages_note": f"per-stage HIP-event times of {k_bd} further maps after the timed region "
                       "(every stage marked); the timed region marks only the roofline's kernel",
        "records_per_particle": round(st["records"] / max(1, n_local), 4),
        "work_items": st["items"], "wide_particles": st["wide"], "large_records": st["large"],
        "output_ok": ok,
    }
    if valu is not None:  # compute-bound regime: the VALU roofline, the HBM one beside it
        res["roofline_hbm"] = res["roofline"]
        res["roofline"] = valu_roofline(valu, args.kernel, nout, dom, dom_ms, pm_stage)
        res["roofline"]["pipeline_frac"] = round(
            valu[0] * pair_flops(args.kernel, nout) / (ms_step * 1e-3) / 1e12 / VALU_PEAK_TFLOPS, 4)
    # A fraction of a physical peak above 1 is a measurement error (e.g. events that timed
    # waiting): refuse to publish it.
    for key in ("roofline", "roofline_hbm"):
        fr = res.get(key, {}).get("frac")
        if fr is not None and fr > 1.0:
            log(f"bench: {key}.frac = {fr} > 1 for kernel {res[key].get('kernel')!r} -- "
                f"not a valid measurement; no line printed")
            if world > 1:
                dist.destroy_process_group()
            sys.exit(4)
    want_cpu = args.cpu_baseline == "on" or (args.cpu_baseline == "auto" and world == 1)
    if want_cpu:
        try:
            res["cpu_baseline"] = cpu_baseline(args, extent)
        except Exception as exc:  # a baseline failure must not hide the GPU number
            res["cpu_baseline"] = {"error": repr(exc)}
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if ok is False:
        log("bench: the timed map FAILED its output check")
        sys.exit(3)


if __name__ == "__main__":
    main()
