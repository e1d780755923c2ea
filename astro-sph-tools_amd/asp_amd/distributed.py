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


def zslab_bounds(z, world_size: int, sample: int = 1 << 20, seed: int = 0):
    """Equal-count Z-slab edges from a random subsample of z (device tensor).

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
    s = torch.sort(z[idx]).values
    edges = [float("-inf")]
    for r in range(1, world_size):
        edges.append(float(s[(k * r) // world_size]))
    edges.append(float("inf"))
    return edges


def project2d_sharded(u, v, h, a0, a1=None, *, image_size, extent, chunk_size: int = 64,
                      kernel="cubic", ratio: bool = False, op: str = "reduce", dst: int = 0,
                      group=None, out0=None, out1=None, projector=None,
                      deterministic: bool = False):
    """Project this rank's particles, then combine the grids over ``group``.

    Returns ``(out0, out1)``: the full map(s) on ``dst`` (``op="reduce"``), on every rank
    (``"allreduce"``), or this rank's row slab (``"reduce_scatter"``; requires
    nx % world_size == 0).  With ``ratio`` the weighted map is formed after the sum.
    ``projector`` replaces the local projection (tests drive the collective logic on CPU
    ranks with the oracle through it); the default is the HIP path.
    """
    import torch
    import torch.distributed as dist
    proj = project2d if projector is None else projector
    kw = {"deterministic": True} if deterministic else {}
    o0, o1 = proj(u, v, h, a0, a1, image_size=image_size, extent=extent,
                  chunk_size=chunk_size, kernel=kernel, ratio=False, out0=out0, out1=out1, **kw)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    outs = [o0] if o1 is None else [o0, o1]
    if world > 1:
        if op == "reduce":
            for t in outs:
                dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM, group=group)
        elif op == "allreduce":
            for t in outs:
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        elif op == "reduce_scatter":
            nx = int(image_size[0])
            if nx % world:
                raise ValueError("reduce_scatter needs nx divisible by the world size")
            res = []
            for t in outs:
                part = torch.empty((nx // world, t.shape[1]), dtype=t.dtype, device=t.device)
                dist.reduce_scatter_tensor(part, t, op=dist.ReduceOp.SUM, group=group)
                res.append(part)
            outs = res
        else:
            raise ValueError(f"unknown op {op!r}")
    if ratio:
        if o1 is None:
            raise ValueError("ratio needs a1")
        if op != "reduce" or rank == dst or world == 1:
            dev = outs[0].device
            _lib.check(_lib.lib().asp_ratio(_lib.ptr(outs[0]), _lib.ptr(outs[1]),
                                            outs[0].numel(), dev.index or 0,
                                            torch.cuda.current_stream(dev).cuda_stream))
    return outs[0], (outs[1] if len(outs) > 1 else None)
