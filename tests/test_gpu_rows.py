"""Row slabs (asp_project2d_rows, the image-plane decomposition of SURVEY.md §8(e) / H2):
the rows of one slab are exactly the whole map's rows -- neighbour counts bit-exact, int64
fixed-point maps bit-identical (a tile's records and scale do not depend on which rows
are asked for), fp64 maps within rounding -- and routing each slab only the particles
whose footprints reach it (distributed.route_rows) changes nothing.  (Particles over more
than 256 tiles take the wide path, whose fixed-point scale is shared by all wide
particles of a pass; a row window can make a particle narrow, so the bit-identity is
checked with the wide path off, ASP_WIDE_TILES, and the default within rounding.)"""
import pytest

pytestmark = pytest.mark.gpu


def _data(n, seed, h_law, grid):
    import torch
    from asp_amd.plummer import plummer_torch
    d = plummer_torch(n, seed=seed, h_law=h_law, extent=4.0, grid=grid, device="cuda")
    return d["x"], d["y"], d["h"], (d["m"] * d["T"]).contiguous(), d["m"]


@pytest.mark.parametrize("nx,ny,bounds,h_law", [
    (1024, 1024, [0, 192, 448, 1024], "physical"),
    (1000, 1024, [0, 64, 512, 960, 1000], "pixel"),
    (768, 640, [0, 384, 768], "physical"),
    (1000, 1024, [0, 100, 333, 334, 999, 1000], "physical"),  # any rows: tiles start at row_lo
])
def test_rows_equal_full_map(gpu, nx, ny, bounds, h_law, monkeypatch):
    import torch
    from asp_amd.device import project2d
    from asp_amd.distributed import route_rows
    u, v, h, a0, a1 = _data(300_000, 5, h_law, max(nx, ny))
    ext = (-4.0, 4.0, -3.0, 5.0)
    kw = dict(image_size=(nx, ny), extent=ext, kernel="wendland_c2")
    d0, d1 = project2d(u, v, h, a0, a1, deterministic=True, **kw)  # default wide path
    g0, g1 = project2d(u, v, h, a0, a1, **kw)
    cnt, _ = project2d(u, v, h, torch.ones_like(h), image_size=(nx, ny), extent=ext,
                       kernel="indicator")
    monkeypatch.setenv("ASP_WIDE_TILES", "1000000")
    f0, f1 = project2d(u, v, h, a0, a1, deterministic=True, **kw)
    for r in range(len(bounds) - 1):
        r0, r1 = bounds[r], bounds[r + 1]
        s0, s1 = project2d(u, v, h, a0, a1, deterministic=True, rows=(r0, r1), **kw)
        assert s0.shape == (r1 - r0, ny)
        # a window's tiles start at row_lo: tile-aligned windows have the full map's tiles
        # (same records, same fixed-point scale: bit-identical), others are within rounding
        aligned = r0 % 64 == 0 and (r1 % 64 == 0 or r1 == nx)
        if aligned:
            assert torch.equal(s0, f0[r0:r1]) and torch.equal(s1, f1[r0:r1])
        else:
            torch.testing.assert_close(s0, f0[r0:r1], rtol=1e-5, atol=1e-6 * float(f0.abs().max()))
            torch.testing.assert_close(s1, f1[r0:r1], rtol=1e-5, atol=1e-6 * float(f1.abs().max()))
        sc, _ = project2d(u, v, h, torch.ones_like(h), image_size=(nx, ny), extent=ext,
                          kernel="indicator", rows=(r0, r1))
        assert torch.equal(sc, cnt[r0:r1])
        monkeypatch.delenv("ASP_WIDE_TILES")
        e0, e1 = project2d(u, v, h, a0, a1, deterministic=True, rows=(r0, r1), **kw)
        torch.testing.assert_close(e0, d0[r0:r1], rtol=1e-5, atol=1e-6 * float(d0.abs().max()))
        torch.testing.assert_close(e1, d1[r0:r1], rtol=1e-5, atol=1e-6 * float(d1.abs().max()))
        w0, w1 = project2d(u, v, h, a0, a1, ratio=True, rows=(r0, r1), **kw)
        want = torch.where(g1[r0:r1] != 0, g0[r0:r1] / torch.where(g1[r0:r1] != 0, g1[r0:r1], 1), 0)
        torch.testing.assert_close(w1, g1[r0:r1], rtol=1e-5, atol=1e-6 * float(g1.abs().max()))
        cov = g1[r0:r1] > 1e-3 * float(g1.max())
        torch.testing.assert_close(w0[cov], want[cov], rtol=1e-4, atol=0)
        # only the particles routed to this slab
        edges = sorted({0, r0, r1, nx})
        q0, q1 = route_rows(u, h, ext[:2], nx, edges)
        mine = edges.index(r0)
        keep = (q0 <= mine) & (q1 >= mine)
        monkeypatch.setenv("ASP_WIDE_TILES", "1000000")
        k0, k1 = project2d(u[keep].contiguous(), v[keep].contiguous(), h[keep].contiguous(),
                           a0[keep].contiguous(), a1[keep].contiguous(), deterministic=True,
                           rows=(r0, r1), **kw)
        if aligned:
            assert torch.equal(k0, f0[r0:r1]) and torch.equal(k1, f1[r0:r1])
        else:
            assert torch.equal(k0, s0) and torch.equal(k1, s1)  # the same window's records
    torch.cuda.synchronize()


def test_rows_argument_errors(gpu):
    import torch
    from asp_amd.device import project2d
    u, v, h, a0, a1 = _data(1000, 1, "pixel", 256)
    for rows in ((128, 64), (0, 300), (-64, 64), (5, 5)):
        with pytest.raises(ValueError):
            project2d(u, v, h, a0, image_size=(256, 256), extent=(-4, 4, -4, 4), rows=rows)
