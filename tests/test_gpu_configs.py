"""BASELINE configs[3] and configs[4] exercised through the HIP path on one MI355X.

* cfg5 (10^8 -> 512^3 density cube): the full 512^3 cube (16384 bricks, the per-call
  maximum) from 10^6 physical-h Plummer particles against the CPU restatement
  ``oracle_project3d`` -- voxel neighbour counts bit-exact, density within the bar of
  tests/test_gpu_parity.py;
* cfg5's decomposition: the 8 voxel-plane slabs of
  ``distributed.plane_slabs`` each deposited from the particles ``route_particles`` sends
  to that slab (halo duplication), concatenated: counts equal to the full cube's
  bit-for-bit, density equal to the fp32 rounding of the fp64 sums;
* cfg4's decomposition: the eight work-weighted Z-slab shards of a 2 x 10^6-particle
  4096^2 mass-weighted map (``zslab_bounds(z, 8, weights=slab_cost(...))``, the edges
  ``bench.py --gpus 8`` uses), each projected by the HIP path alone and summed on the host
  as the RCCL reduce would: counts bit-exact against ``project_scatter`` over all
  particles, both components and the ratio within the bar;
* the image-row alternative (``bench.py --decomp rows``): the same map's eight
  row slabs (``row_slabs``), each projected by ``asp_project2d_rows`` from only the
  particles ``route_rows`` sends it, the ratio formed locally, the slabs concatenated as
  the gather assembles them: counts bit-exact, components and ratio within the bar
  against ``project_scatter`` over all particles.

The reference has no cube and no multi-GPU path; the cube's parity
is pinned by its CPU restatement (tests/test_cube_oracle.py), the map's by the goldens.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_map_close, assert_ratio_close

pytestmark = pytest.mark.gpu

CUBE = (512, 512, 512)
EXT3 = (-4.0, 4.0, -4.0, 4.0, -4.0, 4.0)


@pytest.fixture(scope="module")
def cube_particles():
    """10^6 physical-h Plummer particles, float32-representable (the cube's entry point
    takes float32 arrays; the oracle gets the same values in float64)."""
    from asp_amd.plummer import plummer
    p = plummer(1_000_000, seed=11, h_law="physical")
    f = lambda a: np.asarray(a, np.float32).astype(np.float64)  # noqa: E731
    x, y, z = (f(p["pos"][:, c]) for c in range(3))
    return x, y, z, f(p["h"]), f(p["m"])


@pytest.fixture(scope="module")
def cube_full(gpu, cube_particles):
    """The whole 512^3 cube on the GPU: (counts, density) as float32 host arrays."""
    import torch
    from asp_amd.device import project3d
    x, y, z, h, m = (torch.from_numpy(a.astype(np.float32)).cuda() for a in cube_particles)
    ones = torch.ones_like(h)
    cnt = project3d(x, y, z, h, ones, cube_size=CUBE, extent=EXT3, kernel="indicator")
    cnt = cnt.cpu().numpy()
    den = project3d(x, y, z, h, m, cube_size=CUBE, extent=EXT3, kernel="wendland_c2")
    den = den.cpu().numpy()
    return cnt, den


def test_cfg5_512_cube_vs_oracle(gpu, oracle, cube_particles, cube_full):
    from asp_amd.device import stats
    x, y, z, h, m = cube_particles
    cnt, den = cube_full
    want = oracle.project3d(x, y, z, h, np.ones_like(h), CUBE, EXT3, kernel="indicator")
    assert np.array_equal(cnt, want), f"{np.count_nonzero(cnt != want)} voxel counts differ"
    pairs = float(want.sum())
    del want
    assert pairs > 1e9  # physical h: ~10^3 voxels per particle
    ref = oracle.project3d(x, y, z, h, m, CUBE, EXT3, kernel="wendland_c2")
    assert_map_close(den, ref)
    assert stats(0)["tiles"] == 16384  # every brick of the cube in one call


def test_cfg5_plane_slabs_compose(gpu, cube_particles, cube_full):
    """8 voxel-plane slabs, each from the particles routed to it (what project3d_sharded
    deposits on rank r of 8), concatenated == the full cube."""
    import torch
    from asp_amd.device import project3d
    from asp_amd.distributed import plane_slabs, route_particles
    x, y, z, h, m = (torch.from_numpy(a.astype(np.float32)).cuda() for a in cube_particles)
    cnt_full, den_full = cube_full
    W = 8
    K = plane_slabs(CUBE[2], W)
    r0, r1 = route_particles(z, h, EXT3[4:6], CUBE[2], W)
    cnts, dens, routed = [], [], 0
    for r in range(W):
        keep = (r0 <= r) & (r1 >= r)
        routed += int(keep.sum())
        s = [t[keep].contiguous() for t in (x, y, z, h, m)]
        ones = torch.ones_like(s[3])
        c = project3d(*s[:4], ones, cube_size=CUBE, extent=EXT3, kernel="indicator",
                      planes=(K[r], K[r + 1]))
        d = project3d(*s[:4], s[4], cube_size=CUBE, extent=EXT3, kernel="wendland_c2",
                      planes=(K[r], K[r + 1]))
        cnts.append(c.cpu().numpy())
        dens.append(d.cpu().numpy())
    assert routed > x.shape[0]  # halo particles were duplicated into neighbouring slabs
    cnt = np.concatenate(cnts, axis=2)
    assert np.array_equal(cnt, cnt_full), f"{np.count_nonzero(cnt != cnt_full)} voxels differ"
    den = np.concatenate(dens, axis=2)
    # the same particles and pairs per voxel; only the fp64 accumulation order differs
    assert np.array_equal(den != 0, den_full != 0)
    np.testing.assert_allclose(den, den_full, rtol=2.5e-7, atol=0)


def test_cfg4_eight_zslab_shards_summed(gpu, oracle):
    """cfg4 rehearsal on one GPU: 2 x 10^6 raw-fp64 Plummer particles, pixel-scale h,
    4096^2 mass-weighted Wendland map, split by the work-weighted Z-slab edges of 8 ranks;
    each shard projected alone (full grid, both components), the shards summed on the
    host, the ratio formed after the sum."""
    import torch
    from asp_amd.device import project2d_f64
    from asp_amd.distributed import slab_cost, zslab_bounds
    from asp_amd.plummer import plummer
    n, G, W = 2_000_000, 4096, 8
    ext = (-4.0, 4.0, -4.0, 4.0)
    p = plummer(n, seed=23, h_law="pixel", grid=G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    zt = torch.from_numpy(pos[:, 2]).cuda()
    w = slab_cost(torch.from_numpy(pos[:, 0]).cuda(), torch.from_numpy(pos[:, 1]).cuda(),
                  torch.from_numpy(h).cuda(), ext, 2 * ext[1] / G)
    e = zslab_bounds(zt, W, weights=w)
    assert len(e) == W + 1
    s0 = np.zeros((G, G))
    s1 = np.zeros((G, G))
    cnt = np.zeros((G, G))
    sizes = []
    for r in range(W):
        k = (pos[:, 2] >= e[r]) & (pos[:, 2] < e[r + 1])
        sizes.append(int(k.sum()))
        ps, hs = np.ascontiguousarray(pos[k]), h[k]
        c0, c1 = project2d_f64(ps, hs, (m * T)[k], m[k], image_size=(G, G), extent=ext,
                               kernel="wendland_c2")
        s0 += c0
        s1 += c1
        c, _ = project2d_f64(ps, hs, np.ones(hs.size), image_size=(G, G), extent=ext,
                             kernel="indicator")
        cnt += c
    assert sum(sizes) == n and min(sizes) > 0
    o0, o1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, m, (G, G), 64, *ext,
                                    kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = np.where(s1 != 0, s0 / s1, 0.0)
    assert_ratio_close(ratio, o0, o1)
    c_ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 64,
                                      *ext, kernel="indicator")
    assert np.array_equal(cnt, c_ref)


def test_cfg4_rows_eight_row_slabs_assembled(gpu, oracle):
    """The row-slab decomposition (``bench.py --decomp rows``) on one GPU: 2 x 10^6 Plummer
    particles at pixel-scale h, 4096^2 mass-weighted Wendland-C2 map, 8 row slabs; each
    slab projected from ITS routed particles only (asp_project2d_rows), its ratio formed
    locally, the slabs stitched as the reference stitches its chunks
    (_projector.py:111-117): neighbour counts bit-exact, both components and the ratio
    within the bar, against the oracle over ALL particles (not against the library's own
    full map)."""
    import torch
    from asp_amd.device import project2d
    from asp_amd.distributed import route_rows, row_slabs
    from asp_amd.plummer import plummer
    n, G, W = 2_000_000, 4096, 8
    ext = (-4.0, 4.0, -4.0, 4.0)
    p = plummer(n, seed=29, h_law="pixel", grid=G)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    x, y, h = f32(p["pos"][:, 0]), f32(p["pos"][:, 1]), f32(p["h"])
    a0, a1 = f32(p["m"] * p["T"]), f32(p["m"])
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    u, v, hh, A0, A1 = (dev(a) for a in (x, y, h, a0, a1))
    R = row_slabs(G, W, u, ext[:2])
    assert len(R) == W + 1 and R[0] == 0 and R[-1] == G
    r0, r1 = route_rows(u, hh, ext[:2], G, R)
    s0, s1, rr, cnt = (np.zeros((G, G), np.float64) for _ in range(4))
    routed = 0
    for r in range(W):
        k = (r0 <= r) & (r1 >= r)
        routed += int(k.sum())
        su, sv, sh, sa0, sa1 = (t[k].contiguous() for t in (u, v, hh, A0, A1))
        rows = (R[r], R[r + 1])
        kw = dict(image_size=(G, G), extent=ext, kernel="wendland_c2", rows=rows)
        c0, c1 = project2d(su, sv, sh, sa0, sa1, **kw)
        q0, q1 = project2d(su, sv, sh, sa0, sa1, ratio=True, **kw)
        c, _ = project2d(su, sv, sh, torch.ones_like(sh), image_size=(G, G), extent=ext,
                         kernel="indicator", rows=rows)
        sl = slice(*rows)
        s0[sl], s1[sl] = c0.cpu().numpy(), c1.cpu().numpy()
        rr[sl], cnt[sl] = q0.cpu().numpy(), c.cpu().numpy()
        # the weight map of the ratio call is the same sum (fp64 atomics: order may differ)
        np.testing.assert_allclose(q1.cpu().numpy(), s1[sl], rtol=1e-6, atol=0)
    assert n * 0.95 < routed < n * 1.05  # duplicates only where footprints cross a bound
    xd, yd, hd = (a.astype(np.float64) for a in (x, y, h))
    o0, o1 = oracle.project_scatter(xd, yd, hd, a0.astype(np.float64), a1.astype(np.float64),
                                    (G, G), 64, *ext, kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    assert_ratio_close(rr, o0, o1)
    c_ref, _ = oracle.project_scatter(xd, yd, hd, np.ones(n), None, (G, G), 64, *ext,
                                      kernel="indicator")
    assert np.array_equal(cnt, c_ref)
