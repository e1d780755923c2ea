"""Multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

Each rank keeps one Z-slab of the particles, projects it onto the full grid, and
``project2d_sharded`` combines the grids with one collective.  The local projection is
injected (the CPU oracle), so this checks the sharding and collective logic; the GPU
projection itself is covered by the -m gpu parity tests.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG_ROOT, REPO

G = 64
EXT = (-2.0, 2.0, -2.0, 2.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_projector(u, v, h, a0, a1, *, image_size, extent, chunk_size, kernel, ratio,
                      out0, out1):
    import pyoracle
    o0, o1 = pyoracle.project_scatter(u.numpy(), v.numpy(), h.numpy(), a0.numpy(),
                                      None if a1 is None else a1.numpy(), image_size,
                                      chunk_size, *extent, kernel=kernel)
    t0 = torch.from_numpy(o0.astype(np.float32))
    t1 = None if o1 is None else torch.from_numpy(o1.astype(np.float32))
    if out0 is not None:  # write into the caller's buffers, as the device path does
        out0.copy_(t0)
        t0 = out0
        if t1 is not None and out1 is not None:
            out1.copy_(t1)
            t1 = out1
    return t0, t1


def _data():
    import sys
    sys.path.insert(0, PKG_ROOT)
    from asp_amd.plummer import plummer
    p = plummer(4000, seed=2, h_law="physical")
    f = lambda a: torch.tensor(np.asarray(a, np.float32))  # noqa: E731
    return f(p["pos"][:, 0]), f(p["pos"][:, 1]), f(p["pos"][:, 2]), f(p["h"]), f(p["m"]), f(p["T"])


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from asp_amd.distributed import project2d_sharded, zslab_bounds
        x, y, z, h, m, T = _data()
        e = zslab_bounds(z, world)
        keep = (z >= e[rank]) & (z < e[rank + 1])
        sl = [t[keep].contiguous() for t in (x, y, h, m, T)]
        res = {}
        for op in ("reduce", "allreduce", "reduce_scatter"):
            o0, o1 = project2d_sharded(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                       image_size=(G, G), extent=EXT, chunk_size=16,
                                       kernel="cubic", op=op, projector=_oracle_projector)
            res[op] = (o0.numpy().copy(), o1.numpy().copy())
        # reduce-scatter + ONE all-gather: the ratio map of two components ...
        o0, o1 = project2d_sharded(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                   image_size=(G, G), extent=EXT, chunk_size=16, kernel="cubic",
                                   op="reduce_scatter_gather", ratio=True,
                                   projector=_oracle_projector, out0=torch.empty((G, G)),
                                   out1=torch.empty((G, G)))
        res["rsg_ratio"] = o0.numpy().copy()
        res["rsg_o1"] = o1
        # ... or a single map
        o0, o1 = project2d_sharded(sl[0], sl[1], sl[2], sl[3] * sl[4], None,
                                   image_size=(G, G), extent=EXT, chunk_size=16, kernel="cubic",
                                   op="reduce_scatter_gather", projector=_oracle_projector,
                                   out0=torch.empty((G, G)))
        res["rsg"] = o0.numpy().copy()
        try:  # two components but one gather: refused, not silently dropped
            project2d_sharded(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3], image_size=(G, G),
                              extent=EXT, chunk_size=16, kernel="cubic",
                              op="reduce_scatter_gather", projector=_oracle_projector)
            res["rsg_two_maps"] = "accepted"
        except ValueError:
            res["rsg_two_maps"] = "refused"
        maps = torch.empty((2, G, G))  # adjacent maps: one fused collective
        for op in ("reduce", "allreduce"):
            o0, o1 = project2d_sharded(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                       image_size=(G, G), extent=EXT, chunk_size=16,
                                       kernel="cubic", op=op, projector=_oracle_projector,
                                       out0=maps[0], out1=maps[1])
            res["fused_" + op] = (o0.numpy().copy(), o1.numpy().copy())
        # pipelined as bench.py runs N > 1: async collectives, double-buffered maps, map
        # i's collective completed (wait) only after map i + 1 has been projected
        bufs = [torch.full((2, G, G), float("nan")) for _ in range(2)]
        pend = None
        for i in range(3):
            b = bufs[i % 2]
            p = project2d_sharded(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                  image_size=(G, G), extent=EXT, chunk_size=16, kernel="cubic",
                                  op="allreduce", projector=_oracle_projector, out0=b[0],
                                  out1=b[1], async_op=True)
            if pend is not None:
                pend.wait()
            pend = p
        o0, o1 = pend.wait()
        assert o0.data_ptr() == bufs[0][0].data_ptr()
        res["pipelined"] = (o0.numpy().copy(), o1.numpy().copy(), bufs[1][0].numpy().copy())
        res["n_local"] = int(keep.sum())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_zslab_sharded_sum_world2():
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x, y, z, h, m, T = _data()
    full0, full1 = pyoracle.project_scatter(x.numpy(), y.numpy(), h.numpy(), (m * T).numpy(),
                                            m.numpy(), (G, G), 16, *EXT, kernel="cubic")
    assert out[0]["n_local"] + out[1]["n_local"] == x.numel()
    assert abs(out[0]["n_local"] - out[1]["n_local"]) < 0.1 * x.numel()
    tol = 1e-5 * np.abs(full0).max()
    np.testing.assert_allclose(out[0]["reduce"][0], full0, atol=tol, rtol=0)  # dst = 0
    np.testing.assert_allclose(out[0]["reduce"][1], full1, atol=1e-5 * np.abs(full1).max(), rtol=0)
    np.testing.assert_allclose(out[0]["fused_reduce"][0], full0, atol=tol, rtol=0)
    np.testing.assert_allclose(out[0]["fused_reduce"][1], full1, atol=1e-5 * np.abs(full1).max(),
                               rtol=0)
    for r in range(world):
        np.testing.assert_allclose(out[r]["fused_allreduce"][0], full0, atol=tol, rtol=0)
        np.testing.assert_allclose(out[r]["allreduce"][0], full0, atol=tol, rtol=0)
        np.testing.assert_allclose(out[r]["pipelined"][0], full0, atol=tol, rtol=0)
        np.testing.assert_allclose(out[r]["pipelined"][1], full1, atol=1e-5 * np.abs(full1).max(),
                                   rtol=0)
        np.testing.assert_allclose(out[r]["pipelined"][2], full0, atol=tol, rtol=0)
        rows = slice(r * G // world, (r + 1) * G // world)
        np.testing.assert_allclose(out[r]["reduce_scatter"][0], full0[rows], atol=tol, rtol=0)
        # reduce-scatter, then the one map all-gathered: the full map on every rank
        np.testing.assert_allclose(out[r]["rsg"], full0, atol=tol, rtol=0)
        cov = full1 > 1e-3 * full1.max()
        np.testing.assert_allclose(out[r]["rsg_ratio"][cov], (full0 / np.where(cov, full1, 1))[cov],
                                   rtol=1e-4)
        assert out[r]["rsg_o1"] is None and out[r]["rsg_two_maps"] == "refused"
    # the slabs really are partial maps: neither rank alone holds the full map
    assert not np.allclose(out[1]["reduce"][0], full0, atol=tol)


# ------------------------------------------- reader fp64 host arrays -> stage -> reduce
def _oracle_f64(positions, h, a0, a1, *, projection_axis, image_size, extent, chunk_size,
                kernel, out0, out1, device, deterministic=False):
    """The local projection of project2d_sharded_host on CPU: the oracle on the rank's own
    float64 host arrays (the GPU path is asp_project2d_f64 with ASP_F_DEVICE_OUTPUTS)."""
    import pyoracle
    from asp_amd._axes import reference_axes
    u, v, cu, cv = pyoracle._axes(positions, reference_axes(projection_axis))
    o0, o1 = pyoracle.project_scatter(u, v, h, a0, a1, image_size, chunk_size, *extent,
                                      kernel=kernel, cu=cu, cv=cv)
    t0 = torch.from_numpy(o0.astype(np.float32))
    t1 = None if o1 is None else torch.from_numpy(o1.astype(np.float32))
    return t0, t1


def _f64_data():
    import sys
    sys.path.insert(0, PKG_ROOT)
    from asp_amd.plummer import plummer
    rng = np.random.default_rng(9)
    p = plummer(3000, seed=4, h_law="physical")
    pos = p["pos"] * (1.0 + rng.uniform(-3e-9, 3e-9, p["pos"].shape))  # off the fp32 grid
    return pos, p["h"], p["m"], p["m"] * p["T"]


def _host_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from asp_amd.distributed import project2d_sharded_host
        pos, h, m, mT = _f64_data()
        # the reader's own split: every other particle (any split works for the sum)
        sel = slice(rank, None, world)
        res = {}
        for op in ("reduce", "allreduce"):
            o0, o1 = project2d_sharded_host(np.ascontiguousarray(pos[sel]), h[sel], mT[sel],
                                            m[sel], projection_axis=2, image_size=(G, G),
                                            extent=EXT, chunk_size=16, kernel="cubic", op=op,
                                            projector=_oracle_f64)
            res[op] = (o0.numpy().copy(), o1.numpy().copy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_from_fp64_host_arrays_world2():
    """Each rank hands its own raw-fp64 host arrays to project2d_sharded_host; the summed
    map equals the oracle over all particles (fp64 decisions on the same values)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pos, h, m, mT = _f64_data()
    full0, full1 = pyoracle.project_scatter(pos[:, 0], pos[:, 1], h, mT, m, (G, G), 16, *EXT,
                                            kernel="cubic")
    t0, t1 = 1e-5 * np.abs(full0).max(), 1e-5 * np.abs(full1).max()
    np.testing.assert_allclose(out[0]["reduce"][0], full0, atol=t0, rtol=0)
    np.testing.assert_allclose(out[0]["reduce"][1], full1, atol=t1, rtol=0)
    for r in range(world):
        np.testing.assert_allclose(out[r]["allreduce"][0], full0, atol=t0, rtol=0)
        np.testing.assert_allclose(out[r]["allreduce"][1], full1, atol=t1, rtol=0)


def test_pair_weighted_zslabs():
    """zslab_bounds with slab_cost weights: equal modelled work, not equal counts -- at
    physical h the core slabs hold fewer particles than the outer ones."""
    import sys
    sys.path.insert(0, PKG_ROOT)
    from asp_amd.distributed import slab_cost, zslab_bounds
    from asp_amd.plummer import plummer
    p = plummer(200_000, seed=3, h_law="physical")
    x, y, z = (torch.tensor(p["pos"][:, k]) for k in range(3))
    h = torch.tensor(p["h"])
    w = slab_cost(x, y, h, (-4.0, 4.0, -4.0, 4.0), 8.0 / 2048)
    for W in (2, 4, 8):
        e = zslab_bounds(z, W, weights=w)
        assert len(e) == W + 1 and e[0] == float("-inf") and e[-1] == float("inf")
        sums = [float(w[(z >= e[r]) & (z < e[r + 1])].sum()) for r in range(W)]
        counts = [int(((z >= e[r]) & (z < e[r + 1])).sum()) for r in range(W)]
        assert max(sums) / min(sums) < 1.10, sums
        if W == 8:
            assert max(counts) / min(counts) > 1.5, counts  # work balance != count balance
    e = zslab_bounds(z, 4)
    counts = [int(((z >= e[r]) & (z < e[r + 1])).sum()) for r in range(4)]
    assert max(counts) / min(counts) < 1.05


# --------------------------------------------------------------------------- 3-D cube
CUBE = (16, 12, 20)
CEXT = (-2.0, 2.0, -2.0, 2.0, -2.0, 2.0)


def _oracle_cube(x, y, z, h, a, *, cube_size, extent, kernel, planes):
    import pyoracle
    o = pyoracle.project3d(x.numpy(), y.numpy(), z.numpy(), h.numpy(), a.numpy(), cube_size,
                           extent, kernel=kernel, planes=planes)
    return torch.from_numpy(o.astype(np.float32))


def _cube_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from asp_amd.distributed import project3d_sharded
        x, y, z, h, m, T = _data()
        # an arbitrary (not Z-sorted) input split, as an MPI-split reader would give
        keep = (torch.arange(x.numel()) % world) == rank
        sl = [t[keep].contiguous() for t in (x, y, z, h, m)]
        slab = project3d_sharded(*sl, cube_size=CUBE, extent=CEXT, kernel="wendland_c2",
                                 projector=_oracle_cube)
        full = project3d_sharded(*sl, cube_size=CUBE, extent=CEXT, kernel="wendland_c2",
                                 gather="all", projector=_oracle_cube)
        q.put((rank, {"slab": slab.numpy().copy(), "full": full.numpy().copy()}))
    finally:
        dist.destroy_process_group()


def test_cube_plane_slabs_halo_exchange_world2():
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    from asp_amd.distributed import plane_slabs
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cube_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x, y, z, h, m, T = _data()
    ref = pyoracle.project3d(x.numpy(), y.numpy(), z.numpy(), h.numpy(), m.numpy(), CUBE, CEXT,
                             kernel="wendland_c2").astype(np.float32)
    K = plane_slabs(CUBE[2], world)
    tol = 1e-6 * np.abs(ref).max()
    for r in range(world):
        np.testing.assert_allclose(out[r]["slab"], ref[:, :, K[r]:K[r + 1]], atol=tol, rtol=1e-6)
        np.testing.assert_allclose(out[r]["full"], ref, atol=tol, rtol=1e-6)


# ------------------------------------------- 2-D row slabs (image-plane decomposition)
GR = 160  # rows split where the particle counts balance


def _oracle_rows(u, v, h, a0, a1, *, image_size, extent, chunk_size, kernel, ratio, out0,
                 out1, rows):
    """The local projection of project2d_rowslab on CPU: the oracle's map over the rank's
    (routed) particles, rows [rows[0], rows[1]) kept (the GPU path is asp_project2d_rows)."""
    import pyoracle
    o0, o1 = pyoracle.project_scatter(u.numpy(), v.numpy(), h.numpy(), a0.numpy(),
                                      None if a1 is None else a1.numpy(), image_size,
                                      chunk_size, *extent, kernel=kernel)
    r = slice(rows[0], rows[1])
    o0, o1 = o0[r], (None if o1 is None else o1[r])
    if ratio:
        o0 = np.where(o1 != 0, o0 / np.where(o1 != 0, o1, 1), 0.0)
    t0 = torch.from_numpy(np.ascontiguousarray(o0, np.float32))
    t1 = None if o1 is None else torch.from_numpy(np.ascontiguousarray(o1, np.float32))
    return t0, t1


def _rows_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from asp_amd.distributed import project2d_rowslab, route_rows, row_slabs
        x, y, z, h, m, T = _data()
        # an arbitrary input split (as a reader's MPI split): every other particle
        keep = (torch.arange(x.numel()) % world) == rank
        sl = [t[keep].contiguous() for t in (x, y, h, m, T)]
        res = {}
        slab, s1 = project2d_rowslab(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                     image_size=(GR, GR), extent=EXT, chunk_size=16,
                                     kernel="cubic", projector=_oracle_rows)
        res["slab"] = (slab.numpy().copy(), s1.numpy().copy())
        full, none = project2d_rowslab(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                       image_size=(GR, GR), extent=EXT, chunk_size=16,
                                       kernel="cubic", ratio=True, gather="all",
                                       projector=_oracle_rows)
        res["full_ratio"] = full.numpy().copy()
        res["none"] = none
        got, _ = project2d_rowslab(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                   image_size=(GR, GR), extent=EXT, chunk_size=16,
                                   kernel="cubic", ratio=True, gather="dst",
                                   projector=_oracle_rows)
        res["dst"] = got.numpy().copy()
        # the bounds project2d_rowslab balanced: the all-reduced row histogram of every
        # rank's own particles (the same on both ranks)
        R = row_slabs(GR, world, sl[0], EXT[:2], group=dist.group.WORLD)
        res["bounds"] = R
        r0, r1 = route_rows(x, h, EXT[:2], GR, R)
        res["routed"] = int(((r0 <= rank) & (r1 >= rank)).sum())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_rowslab_world2():
    """Row-slab ownership (H2): the all-to-all routes each particle to the ranks whose rows
    its footprint reaches; each rank's slab equals the oracle's full map on those rows,
    the ratio is formed locally, and the all-gathered ratio map is the full one."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x, y, z, h, m, T = _data()
    full0, full1 = pyoracle.project_scatter(x.numpy(), y.numpy(), h.numpy(), (m * T).numpy(),
                                            m.numpy(), (GR, GR), 16, *EXT, kernel="cubic")
    R = out[0]["bounds"]
    assert R == out[1]["bounds"] and R[0] == 0 and R[-1] == GR and 0 < R[1] < GR
    t0, t1 = 1e-5 * np.abs(full0).max(), 1e-5 * np.abs(full1).max()
    cov = full1 > 1e-3 * full1.max()
    want_ratio = np.where(full1 != 0, full0 / np.where(full1 != 0, full1, 1), 0.0)
    for r in range(world):
        rows = slice(R[r], R[r + 1])
        np.testing.assert_allclose(out[r]["slab"][0], full0[rows], atol=t0, rtol=0)
        np.testing.assert_allclose(out[r]["slab"][1], full1[rows], atol=t1, rtol=0)
        np.testing.assert_allclose(out[r]["full_ratio"][cov], want_ratio[cov], rtol=1e-4)
        assert out[r]["none"] is None
    np.testing.assert_allclose(out[0]["dst"][cov], want_ratio[cov], rtol=1e-4)  # on rank 0
    assert out[1]["dst"].shape == (R[2] - R[1], GR)  # rank 1 keeps its own slab
    # every particle reaches some rank; the wide physical-h halo is duplicated, not all of it
    assert x.numel() <= out[0]["routed"] + out[1]["routed"] < 2 * x.numel()


def _rows_subgroup_worker(rank, world, port, q):
    """World 3; the row-slab map runs on the SUBGROUP {1, 2} (group ranks 0, 1 = global 1,
    2), each member holding one spatial half of the particles in x (a skewed reader split)."""
    import sys
    sys.path.insert(0, PKG_ROOT)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from asp_amd.distributed import project2d_rowslab, row_slabs
        grp = dist.new_group([1, 2])  # every rank creates it
        res = {}
        if rank in (1, 2):
            x, y, z, h, m, T = _data()
            # skewed split: group rank 0 gets x < 0, group rank 1 x >= 0
            keep = (x < 0) if rank == 1 else (x >= 0)
            sl = [t[keep].contiguous() for t in (x, y, h, m, T)]
            try:  # two maps but one gather: refused
                project2d_rowslab(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3], image_size=(GR, GR),
                                  extent=EXT, chunk_size=16, kernel="cubic", gather="all",
                                  group=grp, projector=_oracle_rows)
                res["refused"] = False
            except ValueError:
                res["refused"] = True
            res["bounds"] = row_slabs(GR, 2, sl[0], EXT[:2], group=grp)
            got, _ = project2d_rowslab(sl[0], sl[1], sl[2], sl[3] * sl[4], sl[3],
                                       image_size=(GR, GR), extent=EXT, chunk_size=16,
                                       kernel="cubic", ratio=True, gather="dst", dst=0,
                                       group=grp, projector=_oracle_rows)
            res["dst"] = got.numpy().copy()
        dist.barrier()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_rowslab_subgroup_global_peers_and_skewed_split():
    """The row-slab gather on a process subgroup sends to / receives from the members'
    GLOBAL ranks (world 3, group {1, 2}, dst = group rank 0 = global rank 1); the row bounds
    balance the UNION of the members' particles although each holds one spatial half (one
    rank's sample alone would put the bound at an edge of its own half); and two component
    maps with one gather are refused."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_subgroup_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == {}
    assert out[1]["refused"] and out[2]["refused"]
    R = out[1]["bounds"]
    assert R == out[2]["bounds"]
    x, y, z, h, m, T = _data()
    # the union's median row: the bound must sit near it (equal counts per slab)
    rows = np.floor((x.numpy().astype(np.float64) - EXT[0]) / ((EXT[1] - EXT[0]) / GR))
    rows = np.clip(rows, 0, GR - 1)
    frac_below = float(np.mean(rows < R[1]))
    assert 0.45 < frac_below < 0.55, (R, frac_below)
    full0, full1 = pyoracle.project_scatter(x.numpy(), y.numpy(), h.numpy(), (m * T).numpy(),
                                            m.numpy(), (GR, GR), 16, *EXT, kernel="cubic")
    cov = full1 > 1e-3 * full1.max()
    want = np.where(full1 != 0, full0 / np.where(full1 != 0, full1, 1), 0.0)
    np.testing.assert_allclose(out[1]["dst"][cov], want[cov], rtol=1e-4)  # the full map
    assert out[2]["dst"].shape == (R[2] - R[1], GR)                       # its own slab
