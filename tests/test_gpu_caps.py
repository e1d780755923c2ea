"""Arbitrary image sizes and particle counts through the HIP path.

The reference tiles ANY image (_projector.py:88-107).  The device pipeline holds at most
4096 GPU tiles of 64 x 64 pixels per pass, so larger images run as windows of whole tile
rows (asp_project2d.hip ``window_grid``): pixel corners, pitches (including the y-pitch
quirk S2, Δy = (y_max - y_min)/Nx) and the reference's chunk cull stay the whole image's.
Particle counts beyond one pass (32-bit indices and record cursors) run as batches that
accumulate into the same maps (``ASP_MAX_BATCH`` / ``ASP_MAX_RECORDS`` lower the limits
here so small inputs take those paths).

Bars as tests/test_gpu_parity.py: neighbour counts bit-exact against the oracle, values
|g - r| <= 2e-5 max|r| and <= 1e-4 |r| where |r| >= 1e-3 max|r|, zeros exact.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_map_close, assert_ratio_close

pytestmark = pytest.mark.gpu


def _plummer(n, seed, h_law, grid):
    from asp_amd.plummer import plummer
    return plummer(n, seed=seed, h_law=h_law, grid=grid)


def test_8192_square_map_windows(gpu, oracle):
    """8192^2 (16384 GPU tiles: four windows of 32 tile rows), pixel-scale h, weighted
    Wendland-C2 map from 2 x 10^6 raw-fp64 Plummer particles."""
    from asp_amd.device import stats
    from asp_amd.tools.projections import (create_image, create_weighted_image,
                                           indicator_kernel, wendland_c2_kernel)
    n, G = 2_000_000, 8192
    p = _plummer(n, 3, "pixel", G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    ext = (-4.0, 4.0, -4.0, 4.0)
    r, s0, s1 = create_weighted_image(pos, h, m, T, (G, G), 64, 2, *ext,
                                      kernel_func=wendland_c2_kernel, return_components=True)
    assert r.shape == (G, G) and r.dtype == np.float64
    assert stats(0)["tiles"] == 16384
    o0, o1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, m, (G, G), 64, *ext,
                                    kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    assert_ratio_close(r, o0, o1)
    del o0, o1, s0, s1, r
    cnt = create_image(pos, h, np.ones(n), (G, G), 64, 2, *ext, kernel_func=indicator_kernel)
    c_ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 64,
                                      *ext, kernel="indicator")
    assert np.array_equal(cnt, c_ref)
    # every window holds pairs: the seams at image rows 2048, 4096, 6144 are covered
    for x in (2047, 2048, 4095, 4096, 6143, 6144):
        assert cnt[x].sum() > 0


def test_6000x3000_nonsquare_mixed_axis(gpu, oracle):
    """Non-square 6000 x 3000 image (4418 GPU tiles: two windows) with the reference's
    mixed "y" spelling (pixel test on x/z, chunk cull on x/y) and a chunk size that does not
    divide the window rows (S2: Δy uses Nx = 6000)."""
    from asp_amd._axes import reference_axes
    from asp_amd.tools.projections import create_image, indicator_kernel
    rng = np.random.default_rng(31)
    n = 400_000
    pos = rng.normal(0, 0.7, (n, 3))
    h = rng.uniform(0.0005, 0.004, n)
    A = rng.uniform(0.5, 2.0, n)
    size, cs, ext = (6000, 3000), 48, (-2.5, 2.5, -1.3, 1.2)
    ax = reference_axes("y")
    u, v, cu, cv = oracle._axes(pos, ax)
    img = create_image(pos, h, A, size, cs, "y", *ext)
    ref, _ = oracle.project_scatter(u, v, h, A, None, size, cs, *ext, cu=cu, cv=cv)
    assert_map_close(img, ref)
    cnt = create_image(pos, h, np.ones(n), size, cs, "y", *ext, kernel_func=indicator_kernel)
    c_ref, _ = oracle.project_scatter(u, v, h, np.ones(n), None, size, cs, *ext,
                                      kernel="indicator", cu=cu, cv=cv)
    assert np.array_equal(cnt, c_ref)
    assert cnt[4095:4097].sum() > 0  # the window seam (tile row 64 = image row 4096)


@pytest.mark.parametrize("knob", [("ASP_MAX_BATCH", "70000"), ("ASP_MAX_RECORDS", "90000")])
def test_particle_batches_accumulate(gpu, oracle, monkeypatch, knob):
    """Batched passes (fixed-size particle batches, or halving while a pass would exceed
    the record limit) give the single-pass neighbour counts exactly and the map within the
    bar, the ratio formed after the last batch."""
    from asp_amd.tools.projections import (create_image, create_weighted_image,
                                           indicator_kernel, wendland_c2_kernel)
    n, G = 300_000, 512
    p = _plummer(n, 9, "physical", G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    ext = (-3.0, 3.0, -3.0, 3.0)
    monkeypatch.setenv(*knob)
    r, s0, s1 = create_weighted_image(pos, h, m, T, (G, G), 64, 2, *ext,
                                      kernel_func=wendland_c2_kernel, return_components=True)
    cnt = create_image(pos, h, np.ones(n), (G, G), 64, 2, *ext, kernel_func=indicator_kernel)
    r1 = create_weighted_image(pos, h, m, T, (G, G), 64, 2, *ext, kernel_func=wendland_c2_kernel)
    monkeypatch.delenv(knob[0])
    o0, o1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, m, (G, G), 64, *ext,
                                    kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    assert_ratio_close(r, o0, o1)
    assert_ratio_close(r1, o0, o1)  # the fused-ratio request, batched
    c_ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 64,
                                      *ext, kernel="indicator")
    assert np.array_equal(cnt, c_ref)
