"""Multi-GPU projection: particles sharded by Z-slab, one RCCL collective on the grid.

One process per GPU (``torch.distributed``, backend "nccl" = RCCL over xGMI).  The
projection is linear in the particles and particles along the line of sight are
independent, so every rank projects ITS particles onto the FULL grid and a single sum
over ranks gives the map.  No halo exchange is needed for 2-D maps.

The reference's own decomposition is compatible: its snapshot readers already split
particles across MPI ranks (io/EAGLE/_SnapshotEAGLE.py:120-130); this works for ANY
particle split, Z-slabs are what the benchmark uses.

Collective choice (per-link bound ring on point-to-point xGMI): ``"reduce"`` to ``dst``
(default; one 64 MiB fp32 map per output at 4096^2), ``"allreduce"`` when every rank needs
the map, ``"reduce_scatter"`` for a row-slab-distributed map (each rank keeps nx/W rows).
"""
from __future__ import annotations

from . import _lib
from .device import project2d


def slab_cost(u, v, h, extent, pitch: float, binning_pairs: float = 1000.0):
    """Per-particle work model for slab balancing, in units of one (pixel, particle) pair:
    ``binning_pairs`` plus the footprint's pixels inside the image, ``(2h / pitch)^2``
    clipped to the image's extent on each axis (0 for a particle whose footprint misses
    it).  The constant is a fit to the per-slab times of tools/slab_balance.py at 10^8
    particles -> 4096^2, physical h: a particle costs ~1000 pairs' worth
    beyond its footprint area (binning, the gather's 8 x 16-pixel granularity, the K6
    wide list); at pixel-scale h every particle weighs the same and the edges are the
    equal-count ones."""
    import torch
    x_min, x_max, y_min, y_max = (float(e) for e in extent)
    r = 2.0 * h.double().abs()
    ud, vd = u.double(), v.double()
    wx = (torch.minimum(ud + r, torch.full_like(ud, x_max)) -
          torch.maximum(ud - r, torch.full_like(ud, x_min))).clamp(min=0.0)
    wy = (torch.minimum(vd + r, torch.full_like(vd, y_max)) -
          torch.maximum(vd - r, torch.full_like(vd, y_min))).clamp(min=0.0)
    return binning_pairs + (wx / float(pitch)) * (wy / float(pitch))


def zslab_bounds(z, world_size: int, sample: int = 1 << 20, seed: int = 0, weights=None):
    """Z-slab edges from a random subsample of z (device tensor): equal particle counts,
    or with ``weights`` (one per particle, e.g. :func:`slab_cost`) equal summed weight --
    at physical h the pair work per particle grows as h^2, so equal counts leave the core
    slabs with far more work than the outer ones.

    Returns a list of world_size + 1 floats (first -inf, last +inf).
    """
    import torch
    n = z.shape[0]
    if n == 0 or world_size == 1:
        return [float("-inf")] + [float("inf")] * world_size
    g = torch.Generator(device=z.device)
    g.manual_seed(seed)
    k = min(n, sample)
    idx = torch.randint(0, n, (k,), generator=g, device=z.device)
    s, order = torch.sort(z[idx])
    edges = [float("-inf")]
    if weights is None:
        for r in range(1, world_size):
            edges.append(float(s[(k * r) // world_size]))
    else:
        c = torch.cumsum(weights[idx][order].double(), 0)
        tot = float(c[-1])
        targets = torch.tensor([tot * r / world_size for r in range(1, world_size)],
                               dtype=torch.float64, device=z.device)
        pos = torch.searchsorted(c, targets).clamp(max=k - 1)
        edges += [float(s[int(i)]) for i in pos.tolist()]
    edges.append(float("inf"))
    return edges


def _adjacent(o0, o1):
    """A 1-D view over both maps when out1 directly follows out0 in one allocation."""
    if o1 is None or o0.dtype != o1.dtype or o0.device != o1.device:
        return None
    n = o0.numel()
    if o1.numel() != n or o1.data_ptr() != o0.data_ptr() + n * o0.element_size():
        return None
    base = o0.view(-1)
    try:
        import torch
        return torch.as_strided(base, (2 * n,), (1,))
    except Exception:  # pragma: no cover
        return None


class PendingMap:
    """A sharded map whose collective may still be in flight (``async_op=True``).

    ``wait()`` makes the caller's current stream wait for the collective (the host is not
    blocked on RCCL), forms the ratio map where requested, and returns ``(out0, out1)``.
    Until then the buffers must not be reused: the next projection into them has to be
    enqueued after ``wait()`` (bench.py double-buffers the component maps so the RCCL
    sum of map i overlaps the binning and deposit of map i + 1).
    """

    def __init__(self, outs, works, ratio_here, gather=None, single=False, host_ok=False):
        self._outs = outs
        self._works = works
        self._ratio = ratio_here
        self._gather = gather  # (full-size destination, group): all-gather map 0's slabs
        self._single = single  # reduce_scatter_gather: (out0, None) on every world size
        self._host_ok = host_ok  # an injected projector may hand back host maps
        self._done = False

    def wait(self):
        if not self._done:
            for w in self._works:
                w.wait()
            if self._ratio:
                import torch
                o0, o1 = self._outs
                dev = o0.device
                if not o0.is_cuda:  # host maps of an injected projector (the CPU tests)
                    if not self._host_ok:
                        raise RuntimeError("the projector's maps must be device tensors")
                    o0.copy_(torch.where(o1 != 0, o0 / torch.where(o1 != 0, o1, 1), 0))
                else:
                    _lib.check(_lib.lib().asp_ratio(_lib.ptr(o0), _lib.ptr(o1), o0.numel(),
                                                    dev.index or 0,
                                                    torch.cuda.current_stream(dev).cuda_stream))
            if self._gather is not None:
                import torch.distributed as dist
                full, group = self._gather
                dist.all_gather_into_tensor(full, self._outs[0].contiguous(), group=group)
                self._outs = [full]
            self._done = True
        if self._single:
            return self._outs[0], None
        return self._outs[0], (self._outs[1] if len(self._outs) > 1 else None)


def project2d_sharded(u, v, h, a0, a1=None, *, image_size, extent, chunk_size: int = 64,
                      kernel="cubic", ratio: bool = False, op: str = "reduce", dst: int = 0,
                      group=None, out0=None, out1=None, projector=None,
                      deterministic: bool = False, async_op: bool = False):
    """Project this rank's particles, then combine the grids over ``group``.

    Returns ``(out0, out1)``: the full map(s) on ``dst`` (``op="reduce"``), on every rank
    (``"allreduce"``), or this rank's row slab (``"reduce_scatter"``; requires
    nx % world_size == 0).  ``"reduce_scatter_gather"``: reduce-scatter, the ratio (or the
    single map) formed per row slab, then ONE all-gather of that map into ``out0`` on
    every rank -- returns ``(out0, None)``.  With ``ratio`` the weighted map is formed
    after the sum.
    ``async_op=True`` returns a :class:`PendingMap` instead, whose ``wait()`` completes the
    collective (stream-ordered) and the ratio.
    ``projector`` replaces the local projection (tests drive the collective logic on CPU
    ranks with the oracle through it); the default is the HIP path.
    """
    import torch
    import torch.distributed as dist
    if ratio and a1 is None:
        raise ValueError("ratio needs a1")
    if ratio and deterministic:
        raise ValueError("ratio=True cannot use the deterministic fixed point (DESIGN.md §4)")
    if op not in ("reduce", "allreduce", "reduce_scatter", "reduce_scatter_gather"):
        raise ValueError(f"unknown op {op!r}")
    if op == "reduce_scatter_gather" and a1 is not None and not ratio:
        # one map is gathered: two component maps would need two all-gathers
        raise ValueError("reduce_scatter_gather gathers ONE map: with a1 it needs ratio=True")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    nx = int(image_size[0])
    if op.startswith("reduce_scatter") and world > 1 and nx % world:
        raise ValueError("reduce_scatter needs nx divisible by the world size")
    proj = project2d if projector is None else projector
    kw = {"deterministic": True} if deterministic else {}
    o0, o1 = proj(u, v, h, a0, a1, image_size=image_size, extent=extent,
                  chunk_size=chunk_size, kernel=kernel, ratio=False, out0=out0, out1=out1, **kw)
    outs = [o0] if o1 is None else [o0, o1]
    works = []
    fused = _adjacent(o0, o1)  # both maps in one buffer: one collective of 2 maps
    if world > 1:
        if op.startswith("reduce_scatter"):
            res = []
            for t in outs:
                part = torch.empty((nx // world, t.shape[1]), dtype=t.dtype, device=t.device)
                works.append(dist.reduce_scatter_tensor(part, t, op=dist.ReduceOp.SUM,
                                                        group=group, async_op=True))
                res.append(part)
            outs = res
        else:
            for t in ([fused] if fused is not None else outs):
                if op == "reduce":
                    works.append(dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM, group=group,
                                             async_op=True))
                else:
                    works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group,
                                                 async_op=True))
    ratio_here = ratio and (op != "reduce" or rank == dst or world == 1)
    gather = None
    if op == "reduce_scatter_gather" and world > 1:
        # each rank forms the ratio (or the single map) of ITS row slab, then one
        # all-gather of that one map: 2 maps reduce-scattered + 1 map gathered on the wire
        # instead of 2 maps reduced to one rank and the ratio there
        gather = (o0, group)
    pending = PendingMap(outs, works, ratio_here, gather,
                         single=op == "reduce_scatter_gather", host_ok=projector is not None)
    return pending if async_op else pending.wait()


def project2d_sharded_host(positions, h, a0, a1=None, *, projection_axis=2, image_size,
                           extent, chunk_size: int = 64, kernel="cubic", ratio: bool = False,
                           op: str = "reduce", dst: int = 0, group=None, device=None,
                           out0=None, out1=None, projector=None, deterministic: bool = False,
                           async_op: bool = False):
    """The reader -> stage -> project -> collective chain from each rank's OWN float64
    host arrays, as the reference's readers hand them out under their MPI split
    (io/EAGLE/_SnapshotEAGLE.py:120-130: any particle split is fine; a Z-slab split
    balances the work).  The arrays go through pinned bounce buffers to the rank's GPU
    (asp_project2d_f64 with ASP_F_DEVICE_OUTPUTS: the fp64 values stay resident for the
    exact decisions), the map stays on the device and :func:`project2d_sharded`'s
    collective sums it over ``group``.  ``projector`` replaces the local projection (the
    CPU tests inject the oracle; its signature is :func:`project2d_f64_local`'s)."""
    import torch
    if device is None:
        device = torch.cuda.current_device() if projector is None else 0

    def local(_u, _v, _h, _a0, _a1, *, image_size, extent, chunk_size, kernel, ratio, out0,
              out1, **kw):
        f = project2d_f64_local if projector is None else projector
        return f(positions, h, a0, a1, projection_axis=projection_axis, image_size=image_size,
                 extent=extent, chunk_size=chunk_size, kernel=kernel, out0=out0, out1=out1,
                 device=device, **kw)

    return project2d_sharded(None, None, None, a0, a1, image_size=image_size, extent=extent,
                             chunk_size=chunk_size, kernel=kernel, ratio=ratio, op=op, dst=dst,
                             group=group, out0=out0, out1=out1, projector=local,
                             deterministic=deterministic, async_op=async_op)


def project2d_f64_local(positions, h, a0, a1=None, *, projection_axis, image_size, extent,
                        chunk_size, kernel, out0, out1, device, deterministic=False):
    """One rank's fp64 host arrays -> its device map(s) (no ratio: formed after the sum)."""
    from .device import project2d_f64
    return project2d_f64(positions, h, a0, a1, projection_axis=projection_axis,
                         image_size=image_size, extent=extent, chunk_size=chunk_size,
                         kernel=kernel, out0=out0, out1=out1, device=device,
                         deterministic=deterministic, device_out=True)


# ---------------------------------------------------------------------------------------
# 3-D cube: voxel Z-slab ownership with footprint-halo duplication
# ---------------------------------------------------------------------------------------
def plane_slabs(nz: int, world_size: int):
    """Equal split of the nz voxel planes: rank r owns planes [K[r], K[r+1])."""
    return [(nz * r) // world_size for r in range(world_size + 1)]


def route_particles(z, h, z_extent, nz: int, world_size: int):
    """Owner-rank range [r0, r1] of every particle's plane footprint (r0 > r1: none).

    The plane range is a superset (one plane of slack each side) of the planes whose
    corners can lie within 2|h| of z; the device deposit decides every voxel exactly,
    so duplicates only cost bandwidth.
    """
    import torch
    z_min, z_max = (float(e) for e in z_extent)
    pz = (z_max - z_min) / nz
    zd, rad = z.double(), (2.0 * h.double()).abs()
    k0 = torch.floor((zd - rad - z_min) / pz) - 1
    k1 = torch.ceil((zd + rad - z_min) / pz) + 1
    ok = (rad > 0) & torch.isfinite(zd) & torch.isfinite(rad) & (k1 >= 0) & (k0 <= nz - 1)
    k0 = k0.clamp(0, nz - 1).long()
    k1 = k1.clamp(0, nz - 1).long()
    K = torch.tensor(plane_slabs(nz, world_size)[1:-1], device=z.device, dtype=torch.long)
    r0 = torch.searchsorted(K, k0, right=True)
    r1 = torch.searchsorted(K, k1, right=True)
    r0 = torch.where(ok, r0, torch.full_like(r0, world_size))
    r1 = torch.where(ok, r1, torch.full_like(r1, -1))
    return r0, r1


def exchange_halo(x, y, z, h, a, *, z_extent, nz: int, group=None):
    """All-to-all exchange: every rank receives every particle (from any rank) whose
    footprint reaches its plane slab.  Returns the received (x, y, z, h, a)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    r0, r1 = route_particles(z, h, z_extent, nz, world)
    packed = torch.stack([x, y, z, h, a], dim=1)
    parts, counts = [], []
    for d in range(world):
        sel = packed[(r0 <= d) & (r1 >= d)]
        parts.append(sel)
        counts.append(sel.shape[0])
    send = torch.cat(parts, dim=0).contiguous()
    scount = torch.tensor(counts, dtype=torch.int64, device=x.device)
    rcount = torch.empty_like(scount)
    dist.all_to_all_single(rcount, scount, group=group)
    rc = rcount.tolist()
    recv = torch.empty((sum(rc), 5), dtype=send.dtype, device=send.device)
    dist.all_to_all_single(recv.view(-1), send.view(-1), [c * 5 for c in rc],
                           [c * 5 for c in counts], group=group)
    return tuple(recv[:, c].contiguous() for c in range(5))


def project3d_sharded(x, y, z, h, a, *, cube_size, extent, kernel="cubic",
                      gather: str = "none", group=None, projector=None):
    """Cube on W ranks: rank r owns voxel planes [K[r], K[r+1]) of ``plane_slabs``.

    Any input split works (each rank passes ITS particles): one all-to-all moves each
    particle to every rank whose slab its footprint reaches (halo duplication), then each
    rank deposits its slab locally -- no reduction of the 512 MiB cube.  ``gather="none"``
    returns this rank's (nx, ny, K[r+1]-K[r]) slab; ``"all"`` all-gathers the full cube
    on every rank.  ``projector`` replaces the local deposit (CPU tests); default HIP.
    """
    import torch
    import torch.distributed as dist
    from .device import project3d
    proj = project3d if projector is None else projector
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    nx, ny, nz = (int(c) for c in cube_size)
    K = plane_slabs(nz, world)
    if world > 1:
        x, y, z, h, a = exchange_halo(x, y, z, h, a, z_extent=extent[4:6], nz=nz, group=group)
    local = proj(x, y, z, h, a, cube_size=cube_size, extent=extent, kernel=kernel,
                 planes=(K[rank], K[rank + 1]))
    if gather == "none" or world == 1:
        return local
    if gather != "all":
        raise ValueError(f"unknown gather {gather!r}")
    zmax = max(K[r + 1] - K[r] for r in range(world))
    pad = torch.zeros((nx, ny, zmax), dtype=local.dtype, device=local.device)
    pad[:, :, :local.shape[2]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([bufs[r][:, :, :K[r + 1] - K[r]] for r in range(world)], dim=2)


# ---------------------------------------------------------------------------------------
# 2-D map, image-plane alternative: row-slab ownership with footprint-halo duplication
# (SURVEY.md §8(e) / H2 "measure both"; the reference's own image chunks,
# _projector.py:89-111, distributed).  Rank r owns image rows [R[r], R[r+1]); every
# particle goes to each rank whose rows its 2h footprint reaches; each rank projects only
# its rows (asp_project2d_rows: fewer tiles binned per rank, no grid reduction at all).
# ---------------------------------------------------------------------------------------
def row_slabs(nx: int, world_size: int, u=None, u_extent=None, weights=None,
              sample: int = 1 << 22, seed: int = 0, group=None):
    """Row bounds R (world_size + 1 ints, R[0] = 0, R[-1] = nx, strictly increasing).
    Without ``u`` the rows are split evenly; with the particles' ``u`` (device or host
    tensor) and ``u_extent`` = (u_min, u_max) the split equalises the particle count -- or
    the summed ``weights`` -- per slab, at one-row granularity (a random subsample of up to
    2^22 decides; asp_project2d_rows takes any row range).  With ``group`` (an initialised
    process group) every rank passes ITS particles: the per-row histograms of all ranks'
    samples are summed (one all-reduce of nx words), so the bounds balance the union of
    the ranks' particles however the reader split them, and every rank gets the same R."""
    import torch
    W = int(world_size)
    if W <= 1:
        return [0, nx]
    if nx < W:
        raise ValueError(f"{nx} rows cannot make {W} row slabs")
    if group is not None and u is None:
        # every member must join the all-reduce below: a member without particles passes
        # an empty u (its histogram is zero), never None, or the others would hang
        raise ValueError("row_slabs with a group needs u on every rank (an empty tensor if "
                         "the rank holds no particles)")
    if u is None or (u.shape[0] == 0 and group is None):
        inner = [(nx * r) // W for r in range(1, W)]
    else:
        lo, hi = (float(e) for e in u_extent)
        per = torch.zeros(nx, dtype=torch.float64, device=u.device)
        if u.shape[0] > 0:
            g = torch.Generator(device=u.device)
            g.manual_seed(seed)
            k = min(u.shape[0], sample)
            idx = torch.randint(0, u.shape[0], (k,), generator=g, device=u.device)
            row = ((u[idx].double() - lo) / ((hi - lo) / nx)).floor().clamp(0, nx - 1).long()
            w = torch.ones(k, dtype=torch.float64, device=u.device) if weights is None \
                else weights[idx].double()
            # a rank's sample stands for all of its particles
            per.index_add_(0, row, w * (u.shape[0] / k))
        if group is not None:
            import torch.distributed as dist
            dist.all_reduce(per, op=dist.ReduceOp.SUM, group=group)
        c = torch.cumsum(per, 0)
        tot = float(c[-1])
        if not tot > 0:
            inner = [(nx * r) // W for r in range(1, W)]
        else:
            t = torch.tensor([tot * r / W for r in range(1, W)], dtype=torch.float64,
                             device=c.device)
            inner = [int(j) + 1 for j in torch.searchsorted(c, t).tolist()]
    R = [0]  # strictly increasing: bound i in [i, nx - W + i]
    for i, b in enumerate(inner, start=1):
        R.append(min(max(b, R[-1] + 1), nx - W + i))
    R.append(nx)
    return R


def route_rows(u, h, u_extent, nx: int, bounds):
    """Owner-rank range [r0, r1] of every particle's row footprint (r0 > r1: none): the
    rows whose corners can lie within 2|h| of u, with one row of slack each side (the
    device decides every pixel exactly, so duplicates only cost bandwidth)."""
    import torch
    u_min, u_max = (float(e) for e in u_extent)
    ps = (u_max - u_min) / nx
    ud, rad = u.double(), (2.0 * h.double()).abs()
    x0 = torch.floor((ud - rad - u_min) / ps) - 1
    x1 = torch.ceil((ud + rad - u_min) / ps) + 1
    ok = (rad > 0) & torch.isfinite(ud) & torch.isfinite(rad) & (x1 >= 0) & (x0 <= nx - 1)
    x0 = x0.clamp(0, nx - 1).long()
    x1 = x1.clamp(0, nx - 1).long()
    W = len(bounds) - 1
    K = torch.tensor(list(bounds[1:-1]), device=u.device, dtype=torch.long)
    r0 = torch.searchsorted(K, x0, right=True)
    r1 = torch.searchsorted(K, x1, right=True)
    r0 = torch.where(ok, r0, torch.full_like(r0, W))
    r1 = torch.where(ok, r1, torch.full_like(r1, -1))
    return r0, r1


def exchange_rows(cols, u, h, *, u_extent, nx: int, bounds, group=None):
    """All-to-all: every rank receives every particle (from any rank) whose footprint
    reaches its rows.  ``cols``: the per-particle float32 columns to move (u, v, h, a0[, a1])."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    r0, r1 = route_rows(u, h, u_extent, nx, bounds)
    k = len(cols)
    packed = torch.stack(list(cols), dim=1)
    parts, counts = [], []
    for d in range(world):
        sel = packed[(r0 <= d) & (r1 >= d)]
        parts.append(sel)
        counts.append(sel.shape[0])
    send = torch.cat(parts, dim=0).contiguous()
    scount = torch.tensor(counts, dtype=torch.int64, device=u.device)
    rcount = torch.empty_like(scount)
    dist.all_to_all_single(rcount, scount, group=group)
    rc = rcount.tolist()
    recv = torch.empty((sum(rc), k), dtype=send.dtype, device=send.device)
    dist.all_to_all_single(recv.view(-1), send.view(-1), [c * k for c in rc],
                           [c * k for c in counts], group=group)
    return tuple(recv[:, c].contiguous() for c in range(k))


def project2d_rowslab(u, v, h, a0, a1=None, *, image_size, extent, chunk_size: int = 64,
                      kernel="cubic", ratio: bool = False, bounds=None, group=None,
                      gather: str = "none", exchange: bool = True, out0=None, out1=None,
                      projector=None, deterministic: bool = False, dst: int = 0):
    """The map on W ranks by image rows: rank r owns rows [R[r], R[r+1]) of ``bounds``
    (default :func:`row_slabs` balanced on the particles' u).  With ``exchange`` every
    rank passes ITS particles (any split) and one all-to-all routes them to the owners of
    the rows their footprints reach; ``exchange=False`` when the caller already holds
    every particle reaching its rows.  Each rank projects its rows only
    (asp_project2d_rows) with the ratio formed locally -- its rows' sums are complete, so
    no grid collective runs.  ``gather="none"`` returns this rank's (rows, ny) slab(s);
    ``"all"`` all-gathers map 0 (the ratio map with ``ratio``) into the full (nx, ny) map
    on every rank and returns ``(full, None)``; ``"dst"`` sends every slab of map 0 to
    rank ``dst`` (point-to-point, exact slab sizes -- the analogue of the Z-slab path's
    reduce) and returns ``(full, None)`` there, ``(own slab, None)`` elsewhere.
    ``projector`` replaces the local projection (CPU tests); default the HIP path."""
    import torch
    import torch.distributed as dist
    if ratio and a1 is None:
        raise ValueError("ratio needs a1")
    if ratio and deterministic:
        raise ValueError("ratio=True cannot use the deterministic fixed point (DESIGN.md §4)")
    if gather not in ("none", "all", "dst"):
        raise ValueError(f"unknown gather {gather!r}")
    if gather != "none" and a1 is not None and not ratio:
        # one map is gathered: two component maps would need two gathers
        raise ValueError(f"gather={gather!r} gathers ONE map: with a1 it needs ratio=True")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    nx, ny = int(image_size[0]), int(image_size[1])
    if bounds is None:
        # every rank must agree: the row histogram of ALL ranks' particles (one
        # all-reduce), not one rank's sample -- a spatial reader split skews any one rank
        bounds = row_slabs(nx, world, u, extent[:2],
                           group=group if group is not None else dist.group.WORLD) \
            if world > 1 else [0, nx]
    if len(bounds) != world + 1 or bounds[0] != 0 or bounds[-1] != nx:
        raise ValueError(f"bounds must be {world + 1} row edges from 0 to nx, got {bounds}")
    if world > 1 and exchange:
        cols = (u, v, h, a0) if a1 is None else (u, v, h, a0, a1)
        got = exchange_rows(cols, u, h, u_extent=extent[:2], nx=nx, bounds=bounds, group=group)
        u, v, h, a0 = got[:4]
        a1 = got[4] if a1 is not None else None
    proj = project2d if projector is None else projector
    kw = {"deterministic": True} if deterministic else {}
    r0, r1 = bounds[rank], bounds[rank + 1]
    o0, o1 = proj(u, v, h, a0, a1, image_size=image_size, extent=extent, chunk_size=chunk_size,
                  kernel=kernel, ratio=ratio, out0=out0, out1=out1, rows=(r0, r1), **kw)
    if gather == "none" or world == 1:
        return o0, o1
    if gather == "dst":
        # P2POp peers are GLOBAL ranks; dst and r are ranks of `group`
        peer = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
        if rank != dst:
            dist.batch_isend_irecv([dist.P2POp(dist.isend, o0.contiguous(), peer(dst),
                                               group)])[0].wait()
            return o0, None
        full = torch.empty((nx, ny), dtype=o0.dtype, device=o0.device)
        full[r0:r1] = o0
        ops = [dist.P2POp(dist.irecv, full[bounds[r]:bounds[r + 1]], peer(r), group)
               for r in range(world) if r != dst]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return full, None
    rmax = max(bounds[r + 1] - bounds[r] for r in range(world))
    pad = torch.zeros((rmax, ny), dtype=o0.dtype, device=o0.device)
    pad[:r1 - r0] = o0
    full = torch.empty((world * rmax, ny), dtype=o0.dtype, device=o0.device)
    dist.all_gather_into_tensor(full, pad, group=group)
    return torch.cat([full[r * rmax:r * rmax + bounds[r + 1] - bounds[r]]
                      for r in range(world)], dim=0), None
