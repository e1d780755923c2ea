"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors and
the CPU oracle on identical inputs.

Bars (stated here):
* neighbour sets, per-pixel neighbour counts, bin (chunk) membership: BIT-EXACT;
* pixel values (fp32 accumulation vs the fp64 reference):
    |g - r| <= 2e-5 * max|r|   everywhere, and
    |g - r| <= 1e-4 * |r|      where |r| >= 1e-3 * max|r|;
  pixels where the reference is exactly 0 are exactly 0.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ABS_TOL = 2e-5
REL_TOL = 1e-4


def assert_map_close(g, r, abs_tol=ABS_TOL, rel_tol=REL_TOL):
    g = np.asarray(g, np.float64)
    r = np.asarray(r, np.float64)
    assert g.shape == r.shape
    assert np.all(g[r == 0] == 0), "pixels that are 0 in the reference must be exactly 0"
    m = np.max(np.abs(r)) if r.size else 0.0
    if m == 0:
        assert np.all(g == 0)
        return
    err = np.abs(g - r)
    assert err.max() <= abs_tol * m, f"max abs err {err.max() / m:.3e} x max"
    big = np.abs(r) >= 1e-3 * m
    rel = err[big] / np.abs(r[big])
    assert rel.max() <= rel_tol, f"max rel err {rel.max():.3e}"


def assert_ratio_close(r, o0, o1, abs_tol=ABS_TOL, rel_tol=REL_TOL):
    """Weighted map r = s0 / s1 against the reference components o0, o1: zeros exact, and
    the error within what the component bar allows to propagate into the quotient,
    |dr| <= (abs_tol max|o0| + |r| abs_tol max|o1|) / o1 + 2 rel_tol |r| (a pixel whose
    weight comes only from pairs at the kernel's edge has tiny o1)."""
    r = np.asarray(r, np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        want = np.where(o1 != 0, o0 / o1, 0.0)
    np.testing.assert_array_equal(r == 0, want == 0)
    cov = o1 != 0
    bound = ((abs_tol * np.abs(o0).max() + np.abs(want[cov]) * abs_tol * np.abs(o1).max())
             / np.abs(o1[cov]) + 2 * rel_tol * np.abs(want[cov]))
    err = np.abs(r[cov] - want[cov])
    assert np.all(err <= bound), f"ratio error {np.max(err / bound):.3f} x its bound"


def g3():
    g = golden("g3_plummer_1e4_256.npz")
    return (g["pos"].astype(np.float64), g["h"].astype(np.float64), g["A"].astype(np.float64),
            tuple(g["size"]), int(g["cs"]), tuple(g["ext"]), g["img"])


# ------------------------------------------------------------------ golden vectors
def test_g1_kernel_eval_on_device(gpu):
    from asp_amd.tools.projections import quartic_spline_kernel
    g = golden("g1_kernel_table.npz")
    w = quartic_spline_kernel(g["r"], g["h"])
    assert np.array_equal(w == 0, g["w"] == 0)
    np.testing.assert_allclose(w, g["w"], rtol=4e-16 * 8, atol=0)
    with pytest.raises(ValueError):
        quartic_spline_kernel(g["r"].astype(np.float32), g["h"])


@pytest.mark.parametrize("case", list(range(11)))
def test_g2_hand_cases(gpu, case):
    from asp_amd.tools.projections import create_image
    g = golden("g2_hand_cases.npz")
    c = {k: g[f"c{case}_{k}"] for k in ("pos", "h", "A", "size", "cs", "axis", "ext", "img")}
    from asp_amd import CoordinateAxes
    # the fixture ran the reference with its enum member (an int would mean Z there)
    img = create_image(c["pos"].reshape(-1, 3), c["h"], c["A"], tuple(c["size"]), int(c["cs"]),
                       CoordinateAxes(int(c["axis"])), *c["ext"])
    assert img.dtype == np.float64 and img.shape == c["img"].shape
    assert_map_close(img, c["img"])
    assert np.array_equal(img != 0, c["img"] != 0)


def test_g3_plummer_cubic(gpu):
    from asp_amd import CoordinateAxes
    from asp_amd.tools.projections import create_image
    pos, h, A, size, cs, ext, ref = g3()
    img = create_image(pos, h, A, size, cs, CoordinateAxes.Z, *ext)
    assert_map_close(img, ref)


def test_g3_neighbour_counts_bitexact(gpu, oracle):
    """Indicator kernel: per-pixel neighbour counts and index checksums, bit-exact."""
    from asp_amd.tools.projections import create_image, indicator_kernel
    pos, h, A, size, cs, ext, ref = g3()
    ones = np.ones_like(h)
    cnt = create_image(pos, h, ones, size, cs, 2, *ext, kernel_func=indicator_kernel)
    want = oracle.create_image(pos, h, ones, size, cs, 2, *ext, kernel="indicator")
    assert np.array_equal(cnt, want)
    assert np.array_equal(cnt != 0, ref != 0)
    ids = (np.arange(h.size) % 4096).astype(np.float64)
    chk = create_image(pos, h, ids, size, cs, 2, *ext, kernel_func=indicator_kernel)
    want = oracle.create_image(pos, h, ids, size, cs, 2, *ext, kernel="indicator")
    assert np.array_equal(chk, want)


def test_g4_chunk_membership_bitexact(gpu):
    import ctypes as C
    from asp_amd import _lib
    pos, h, A, size, cs, ext, _ = g3()
    g = golden("g4_tile_membership.npz")
    u, v, hh = (np.ascontiguousarray(a, np.float32) for a in (pos[:, 0], pos[:, 1], h))
    out = [np.empty(u.size, np.int32) for _ in range(4)]
    _lib.check(_lib.lib().asp_chunk_ranges(_lib.ptr(u), _lib.ptr(v), _lib.ptr(hh), u.size,
                                           *map(float, ext), size[0], size[1], cs,
                                           *[_lib.ptr(o, _lib._i32) for o in out], 0, 0, None))
    cx0, cx1, cy0, cy1 = out
    ncx, ncy = g["n_chunks"]
    offs = g["offsets"]
    for cx in range(ncx):
        for cy in range(ncy):
            k = cx * ncy + cy
            got = np.nonzero((cx0 <= cx) & (cx <= cx1) & (cy0 <= cy) & (cy <= cy1))[0]
            assert np.array_equal(got, g["index"][offs[k]:offs[k + 1]]), (cx, cy)
    del C


def gpu_neighbours(u, v, h, ext, size, cs, pixels):
    from asp_amd import _lib
    u, v, h = (np.ascontiguousarray(a, np.float32) for a in (u, v, h))
    pix = np.ascontiguousarray(pixels, np.int64)
    offs = np.zeros(pix.size + 1, np.int64)
    tot = np.zeros(1, np.int64)
    cap = max(1, 64 * u.size)
    idx = np.empty(cap, np.int32)
    _lib.check(_lib.lib().asp_pixel_neighbours(
        _lib.ptr(u), _lib.ptr(v), _lib.ptr(h), u.size, *map(float, ext), size[0], size[1], cs,
        _lib.ptr(pix, _lib._i64), pix.size, _lib.ptr(offs, _lib._i64), _lib.ptr(idx, _lib._i32),
        cap, _lib.ptr(tot, _lib._i64), 0))
    assert tot[0] <= cap
    return offs, idx[:tot[0]]


def test_g5_neighbour_sets_bitexact(gpu):
    pos, h, A, size, cs, ext, _ = g3()
    g = golden("g5_neighbours.npz")
    offs, idx = gpu_neighbours(pos[:, 0], pos[:, 1], h, ext, size, cs, g["pixels"])
    assert np.array_equal(offs, g["offsets"]) and np.array_equal(idx, g["index"])


def test_g6_wendland(gpu):
    from asp_amd.tools.projections import create_image, wendland_c2_kernel
    pos, h, A, size, cs, ext, _ = g3()
    ref = golden("g6_wendland_c2.npz")["img"]
    img = create_image(pos, h, A, size, cs, 2, *ext, kernel_func=wendland_c2_kernel)
    assert_map_close(img, ref)


def test_g7_axes_permutation_nonsquare(gpu):
    from asp_amd import CoordinateAxes
    from asp_amd.tools.projections import create_image
    g = golden("g7_axes_permuted.npz")
    pos, h, A = (g[k].astype(np.float64) for k in ("pos", "h", "A"))
    ext = tuple(g["ext"])
    for ax in CoordinateAxes:
        assert_map_close(create_image(pos, h, A, (64, 64), 8, ax, *ext), g[f"img_{ax.value}"])
    p = g["perm"]
    assert_map_close(create_image(pos[p], h[p], A[p], (64, 64), 8, "z", *ext), g["img_z_perm"])
    assert_map_close(create_image(pos, h, A, (48, 64), 16, 2, *ext), g["img_ns_48x64_c16"])
    assert_map_close(create_image(pos, h, A, (64, 40), 7, 2, *ext), g["img_ns_64x40_c7"])


# ------------------------------------------------------------------ oracle, wider cases
def plummer_f32(n, seed, h_law="physical", grid=None, extent=4.0):
    from asp_amd.plummer import plummer
    p = plummer(n, seed=seed, h_law=h_law, grid=grid, extent=extent)
    return {k: np.asarray(v, np.float32).astype(np.float64) for k, v in p.items()}


@pytest.mark.parametrize("n,G,h_law,kernel", [(200_000, 512, "physical", "cubic"),
                                              (300_000, 1024, "pixel", "wendland_c2"),
                                              (50_000, 300, "physical", "wendland_c2")])
def test_plummer_vs_oracle(gpu, oracle, n, G, h_law, kernel):
    from asp_amd.tools.projections import (create_image, indicator_kernel,
                                           quartic_spline_kernel, wendland_c2_kernel)
    p = plummer_f32(n, seed=n, h_law=h_law, grid=G)
    ext = (-4.0, 4.0, -4.0, 4.0)
    kf = {"cubic": quartic_spline_kernel, "wendland_c2": wendland_c2_kernel}[kernel]
    img = create_image(p["pos"], p["h"], p["m"], (G, G), 64, 2, *ext, kernel_func=kf)
    ref, _ = oracle.project_scatter(p["pos"][:, 0], p["pos"][:, 1], p["h"], p["m"], None, (G, G),
                                    64, *ext, kernel=kernel)
    assert_map_close(img, ref)
    cnt = create_image(p["pos"], p["h"], np.ones(n), (G, G), 64, 2, *ext,
                       kernel_func=indicator_kernel)
    want, _ = oracle.project_scatter(p["pos"][:, 0], p["pos"][:, 1], p["h"], np.ones(n), None,
                                     (G, G), 64, *ext, kernel="indicator")
    assert np.array_equal(cnt, want)


def test_boundary_pairs_exact(gpu, oracle):
    """Particles placed at (and 1-4 ulp around) distance exactly 2h from pixel corners:
    the fp32 test alone would misjudge some of these; the fp64 band path must not."""
    from asp_amd.tools.projections import create_image, indicator_kernel
    rng = np.random.default_rng(3)
    G = 64
    ext = (-1.0, 1.0, -1.0, 1.0)
    ps = 2.0 / G
    n = 20000
    xi = rng.integers(4, G - 4, n)
    yi = rng.integers(4, G - 4, n)
    h = np.float32(ps) * rng.choice([0.5, 0.75, 1.0, 1.25, 1.5], n).astype(np.float32)
    ang = rng.uniform(0, 2 * np.pi, n)
    X = -1.0 + xi * ps
    Y = -1.0 + yi * ps
    u = (X + 2.0 * h * np.cos(ang)).astype(np.float32)
    v = (Y + 2.0 * h * np.sin(ang)).astype(np.float32)
    k = rng.integers(-4, 5, n).astype(np.float32)
    u = (u + k * np.spacing(u)).astype(np.float32)
    axis_aligned = rng.random(n) < 0.3  # exact 2h offsets along one axis
    u[axis_aligned] = (X[axis_aligned] + 2.0 * h[axis_aligned]).astype(np.float32)
    v[axis_aligned] = Y[axis_aligned].astype(np.float32)
    pos = np.stack([u, v, np.zeros(n, np.float32)], 1).astype(np.float64)
    h64 = h.astype(np.float64)
    ones = np.ones(n)
    cnt = create_image(pos, h64, ones, (G, G), 8, 2, *ext, kernel_func=indicator_kernel)
    want = oracle.create_image(pos, h64, ones, (G, G), 8, 2, *ext, kernel="indicator")
    assert np.array_equal(cnt, want)
    ids = (np.arange(n) % 4096).astype(np.float64)
    chk = create_image(pos, h64, ids, (G, G), 8, 2, *ext, kernel_func=indicator_kernel)
    want = oracle.create_image(pos, h64, ids, (G, G), 8, 2, *ext, kernel="indicator")
    assert np.array_equal(chk, want)


def test_weighted_map(gpu, oracle):
    from asp_amd.tools.projections import create_weighted_image, wendland_c2_kernel
    p = plummer_f32(100_000, seed=9, h_law="pixel", grid=512)
    ext = (-4.0, 4.0, -4.0, 4.0)
    T = p["T"]
    r, s0, s1 = create_weighted_image(p["pos"], p["h"], p["m"], T, (512, 512), 64, 2, *ext,
                                      kernel_func=wendland_c2_kernel, return_components=True)
    a0 = (p["m"] * T).astype(np.float32).astype(np.float64)  # what the wrapper feeds
    o0, o1 = oracle.project_scatter(p["pos"][:, 0], p["pos"][:, 1], p["h"], a0, p["m"],
                                    (512, 512), 64, *ext, kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    ratio = create_weighted_image(p["pos"], p["h"], p["m"], T, (512, 512), 64, 2, *ext,
                                  kernel_func=wendland_c2_kernel)
    with np.errstate(divide="ignore", invalid="ignore"):
        want = np.where(o1 != 0, o0 / o1, 0.0)
    np.testing.assert_array_equal(ratio == 0, want == 0)
    np.testing.assert_allclose(ratio, want, rtol=2e-4, atol=0)


def test_wide_particles(gpu, oracle):
    """Huge smoothing lengths (wide path, > kWideTiles GPU tiles), large ones (gather path:
    clipped boxes >= 1024 pixels) and small ones (lane / wave paths) mixed."""
    from asp_amd.tools.projections import create_image, indicator_kernel
    rng = np.random.default_rng(5)
    n = 3000
    pos = np.asarray(rng.uniform(-1, 1, (n, 3)), np.float32).astype(np.float64)
    h = np.asarray(rng.uniform(0.0025, 0.01, n), np.float32).astype(np.float64)
    h[:40] = np.asarray(rng.uniform(0.3, 2.0, 40), np.float32)
    h[40:400] = np.asarray(rng.uniform(0.01, 0.06, 360), np.float32)
    A = np.asarray(rng.uniform(0.5, 1.5, n), np.float32).astype(np.float64)
    G = 2048
    ext = (-1.0, 1.0, -1.0, 1.0)
    img = create_image(pos, h, A, (G, G), 32, 2, *ext)
    ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, A, None, (G, G), 32, *ext)
    assert_map_close(img, ref)
    cnt = create_image(pos, h, np.ones(n), (G, G), 32, 2, *ext, kernel_func=indicator_kernel)
    want, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 32,
                                     *ext, kernel="indicator")
    assert np.array_equal(cnt, want)
    from asp_amd.device import stats
    assert stats(0)["wide"] > 0


def test_split_tile_items(gpu, oracle):
    """A dense clump puts > 1 work item on one tile (atomic tile merge path)."""
    from asp_amd.tools.projections import create_image
    rng = np.random.default_rng(8)
    n = 40_000
    pos = np.asarray(rng.normal(0, 0.01, (n, 3)), np.float32).astype(np.float64)
    h = np.full(n, 0.004)
    A = np.asarray(rng.uniform(0.5, 1.5, n), np.float32).astype(np.float64)
    G = 512
    ext = (-1.0, 1.0, -1.0, 1.0)
    img = create_image(pos, h, A, (G, G), 64, 2, *ext)
    from asp_amd.device import stats
    s = stats(0)
    assert s["items"] > s["tiles"] // 64  # some tile was split
    ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, A, None, (G, G), 64, *ext)
    assert_map_close(img, ref)


def test_edge_cases(gpu):
    from asp_amd.tools.projections import create_image
    z = create_image(np.zeros((0, 3)), np.zeros(0), np.zeros(0), (8, 8), 4, 2, -1, 1, -1, 1)
    assert z.shape == (8, 8) and not z.any()
    img = create_image([[0.0, 0, 0], [np.nan, 0, 0], [0.2, 0.2, 0]], [0.0, 0.3, 0.3],
                       [1.0, 1.0, 1.0], (8, 8), 4, 2, -1, 1, -1, 1)
    only = create_image([[0.2, 0.2, 0]], [0.3], [1.0], (8, 8), 4, 2, -1, 1, -1, 1)
    assert np.array_equal(img, only)  # h = 0 and NaN particles contribute nothing
    assert create_image([[0, 0, 0]], [0.5], [1.0], (4, 4), -3, 2, -1, 1, -1, 1).sum() == 0
    with pytest.raises(ValueError):
        create_image([[0, 0, 0]], [0.5], [1.0], (4, 4), 0, 2, -1, 1, -1, 1)
    with pytest.raises(TypeError):  # kernel_func must be callable
        create_image([[0, 0, 0]], [0.5], [1.0], (4, 4), 4, 2, -1, 1, -1, 1, kernel_func=3.0)
    with pytest.raises(ValueError):
        create_image([[0, 0, 0]], [0.5], [1.0], (4, 4), 4, 2, 1, -1, -1, 1)


def test_device_api_ratio_accumulate(gpu, oracle):
    import torch
    from asp_amd.device import project2d
    p = plummer_f32(50_000, seed=4, h_law="pixel", grid=256)
    t = {k: torch.tensor(p[k], dtype=torch.float32, device="cuda") for k in ("h", "m", "T")}
    u = torch.tensor(p["pos"][:, 0], dtype=torch.float32, device="cuda")
    v = torch.tensor(p["pos"][:, 1], dtype=torch.float32, device="cuda")
    ext = (-4.0, 4.0, -4.0, 4.0)
    a0 = t["m"] * t["T"]
    o0, o1 = project2d(u, v, t["h"], a0, t["m"], image_size=(256, 256), extent=ext,
                       kernel="wendland_c2")
    # accumulate: project the two halves into the same maps
    half = u.shape[0] // 2
    s0 = torch.zeros_like(o0)
    s1 = torch.zeros_like(o1)
    for sl in (slice(0, half), slice(half, None)):
        project2d(u[sl].contiguous(), v[sl].contiguous(), t["h"][sl].contiguous(),
                  a0[sl].contiguous(), t["m"][sl].contiguous(), image_size=(256, 256),
                  extent=ext, kernel="wendland_c2", accumulate=True, out0=s0, out1=s1)
    torch.cuda.synchronize()
    assert_map_close(s0.cpu().numpy(), o0.cpu().numpy().astype(np.float64), abs_tol=1e-6,
                     rel_tol=1e-5)
    r, _ = project2d(u, v, t["h"], a0, t["m"], image_size=(256, 256), extent=ext,
                     kernel="wendland_c2", ratio=True)
    o0n, o1n = o0.cpu().numpy().astype(np.float64), o1.cpu().numpy().astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        want = np.where(o1n != 0, o0n / o1n, 0.0)
    np.testing.assert_allclose(r.cpu().numpy(), want, rtol=1e-6)


def test_bitwise_deterministic_and_permutation_invariant(gpu, oracle):
    """ASP_F_DETERMINISTIC (int64 fixed point): repeated runs AND permuted inputs give
    bit-identical maps (the reference itself varies by summation order, S11), within the
    stated tolerance of the reference."""
    from asp_amd.tools.projections import create_image, create_weighted_image
    p = plummer_f32(300_000, seed=12, h_law="physical")
    ext = (-4.0, 4.0, -4.0, 4.0)
    kw = dict(deterministic=True)
    a = create_image(p["pos"], p["h"], p["m"], (512, 512), 64, 2, *ext, **kw)
    b = create_image(p["pos"], p["h"], p["m"], (512, 512), 64, 2, *ext, **kw)
    perm = np.random.default_rng(1).permutation(p["h"].size)
    c = create_image(p["pos"][perm], p["h"][perm], p["m"][perm], (512, 512), 64, 2, *ext, **kw)
    assert np.array_equal(a, b) and np.array_equal(a, c)
    # two fixed-point component maps (no ratio: DESIGN.md §4 -- the library refuses a
    # fixed-point ratio map) are bitwise permutation invariant as well
    from asp_amd.device import project2d_f64
    mT = p["m"] * p["T"]
    kw2 = dict(image_size=(512, 512), extent=ext, chunk_size=64, deterministic=True)
    w1 = project2d_f64(p["pos"], p["h"], mT, p["m"], **kw2)
    w2 = project2d_f64(p["pos"][perm], p["h"][perm], mT[perm], p["m"][perm], **kw2)
    assert np.array_equal(w1[0], w2[0]) and np.array_equal(w1[1], w2[1])
    with pytest.raises(ValueError):
        create_weighted_image(p["pos"], p["h"], p["m"], p["T"], (512, 512), 64, 2, *ext, **kw)
    ref, _ = oracle.project_scatter(p["pos"][:, 0], p["pos"][:, 1], p["h"], p["m"], None,
                                    (512, 512), 64, *ext)
    assert_map_close(a, ref)


def test_record_placement_trials(gpu, oracle, monkeypatch):
    """Record-buffer placement trials (a freshly allocated record buffer: the call's
    scatter is run into several candidate buffers and the fastest kept) leave
    the deterministic maps bit-identical and the neighbour counts exact -- wide particles
    and split tiles included (the wide-list cursor is reset before every trial)."""
    from asp_amd import _lib
    from asp_amd.tools.projections import create_image, create_weighted_image
    from asp_amd.tools.projections import indicator_kernel
    p = plummer_f32(300_000, seed=21, h_law="physical")
    ext = (-4.0, 4.0, -4.0, 4.0)
    from asp_amd.device import project2d_f64
    mT = p["m"] * p["T"]
    kw = dict(image_size=(512, 512), extent=ext, chunk_size=64, deterministic=True)
    monkeypatch.setenv("ASP_PLACEMENT_TRIALS", "0")
    _lib.check(_lib.lib().asp_release(0))
    a = project2d_f64(p["pos"], p["h"], mT, p["m"], **kw)
    monkeypatch.setenv("ASP_PLACEMENT_TRIALS", "4")
    monkeypatch.setenv("ASP_PLACEMENT_MIN_MB", "0")
    _lib.check(_lib.lib().asp_release(0))
    b = project2d_f64(p["pos"], p["h"], mT, p["m"], **kw)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    _lib.check(_lib.lib().asp_release(0))
    cnt = create_image(p["pos"], p["h"], np.ones_like(p["h"]), (512, 512), 64, 2, *ext,
                       kernel_func=indicator_kernel)
    want, _ = oracle.project_scatter(p["pos"][:, 0], p["pos"][:, 1], p["h"], np.ones_like(p["h"]),
                                     None, (512, 512), 64, *ext, kernel="indicator")
    assert np.array_equal(cnt, want)
    _lib.check(_lib.lib().asp_release(0))


def test_default_vs_deterministic_modes(gpu):
    """fp64 and int64 accumulation agree to fp32 rounding on the same inputs."""
    from asp_amd.tools.projections import create_image
    p = plummer_f32(200_000, seed=13, h_law="pixel", grid=1024)
    ext = (-4.0, 4.0, -4.0, 4.0)
    a = create_image(p["pos"], p["h"], p["m"], (1024, 1024), 64, 2, *ext)
    b = create_image(p["pos"], p["h"], p["m"], (1024, 1024), 64, 2, *ext, deterministic=True)
    assert_map_close(b, a, abs_tol=1e-6, rel_tol=1e-5)


@pytest.mark.parametrize("gmin,area", [("5", "20"), ("12", "20"), ("65", "1073741824"),
                                       ("65", "20"), ("65", "6")])
def test_large_stream_threshold(gpu, oracle, gmin, area, monkeypatch):
    """Records whose box clipped to a tile spans >= gather_min pixels on both axes, or at
    least gather_area pixels, go to the large stream and are GATHERED (K4g: register
    sums); the rest are swept or deposited lane-per-record (K4).  Any thresholds must give
    the same neighbour counts (bit-exact) and values within tolerance: 5 sends almost
    every non-small box to K4g, 65 with the area test off none, 65 with area 20 only the
    thin slivers of large discs clipped at tile edges, area 6 also most small boxes.
    Tiles holding both streams are split items merged by K5."""
    from asp_amd.device import stats
    from asp_amd.tools.projections import create_image, create_weighted_image, indicator_kernel
    monkeypatch.setenv("ASP_GATHER_MIN", gmin)
    monkeypatch.setenv("ASP_GATHER_AREA", area)
    rng = np.random.default_rng(11)
    n = 6000
    pos = rng.normal(0, 0.4, (n, 3))
    h = rng.uniform(0.002, 0.08, n)
    A = rng.uniform(0.5, 1.5, n)
    T = rng.uniform(1.0, 3.0, n)
    G, ext = 512, (-1.0, 1.0, -1.0, 1.0)
    cnt = create_image(pos, h, np.ones(n), (G, G), 64, 2, *ext, kernel_func=indicator_kernel)
    large = stats(0)["large"]
    assert (large == 0) == (gmin == "65" and int(area) > 1 << 20)
    want, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 64,
                                     *ext, kernel="indicator")
    assert np.array_equal(cnt, want)
    r, s0, s1 = create_weighted_image(pos, h, A, T, (G, G), 64, 2, *ext, return_components=True)
    w0, w1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, A * T, A, (G, G), 64, *ext)
    assert_map_close(s0, w0)
    assert_map_close(s1, w1)
    from asp_amd.device import project2d_f64
    d0, d1 = project2d_f64(pos, h, A * T, A, image_size=(G, G), extent=(-1.0, 1.0, -1.0, 1.0),
                           chunk_size=64, deterministic=True)
    assert_map_close(d0, w0)
    assert_map_close(d1, w1)


def test_speculative_scatter_grow_and_reuse(gpu, oracle, monkeypatch):
    """The scatter is enqueued before the host reads the record count, against the buffers
    an earlier call left (project2d): a call needing MORE records / wide
    slots than those buffers hold must fall back (kernel leaves, host grows, relaunches),
    one needing fewer must reuse them.  Same bit-exact bar either way."""
    from asp_amd.device import stats
    from asp_amd.tools.projections import create_image, indicator_kernel
    monkeypatch.setenv("ASP_WIDE_TILES", "16")
    G, ext = 512, (-4.0, 4.0, -4.0, 4.0)
    for n, seed, wide in ((20_000, 31, 0), (400_000, 32, 0), (60_000, 33, 0), (90_000, 34, 40),
                          (700_000, 35, 60), (30_000, 36, 0)):
        p = plummer_f32(n, seed=seed, h_law="pixel", grid=G)
        h = p["h"]
        h[:wide] = np.float32(2.0)  # 2h = half the extent: > 16 of the 8 x 8 tiles -> wide
        cnt = create_image(p["pos"], h, np.ones(n), (G, G), 64, 2, *ext,
                           kernel_func=indicator_kernel)
        want, _ = oracle.project_scatter(p["pos"][:, 0], p["pos"][:, 1], h, np.ones(n), None,
                                         (G, G), 64, *ext, kernel="indicator")
        assert np.array_equal(cnt, want), (n, seed)
        assert stats(0)["records"] >= n // 2 and stats(0)["wide"] >= 0.9 * wide  # some miss the map


@pytest.mark.parametrize("n", [4_099, 250_003])
def test_unaligned_inputs_and_ragged_batches(gpu, oracle, n):
    """Count and scatter load U consecutive particles per lane with one vector load when
    the arrays are 16-B aligned, and fall back to scalar loads otherwise (views that start
    one float into an allocation) and for the ragged last batch.  Both load paths feed the
    same particles to the same (workgroup, tile) runs: int64 fixed-point maps are
    bit-identical, and match the oracle within the stated tolerance."""
    import torch
    from asp_amd.device import project2d
    p = plummer_f32(n, seed=21, h_law="pixel", grid=512)
    ext = (-4.0, 4.0, -4.0, 4.0)
    cols = [p["pos"][:, 0], p["pos"][:, 1], p["h"], p["m"] * p["T"], p["m"]]
    aligned = [torch.tensor(c, dtype=torch.float32, device="cuda") for c in cols]
    shifted = []
    for c in cols:  # same values, storage offset of one float (4-B aligned only)
        buf = torch.empty(n + 1, dtype=torch.float32, device="cuda")
        buf[1:] = torch.tensor(c, dtype=torch.float32, device="cuda")
        shifted.append(buf[1:])
    assert shifted[0].data_ptr() % 16 != 0
    kw = dict(image_size=(512, 512), extent=ext, kernel="wendland_c2", deterministic=True)
    a0, a1 = project2d(*aligned, **kw)
    b0, b1 = project2d(*shifted, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a0, b0) and torch.equal(a1, b1)
    ref, _ = oracle.project_scatter(cols[0], cols[1], p["h"], cols[4], None, (512, 512), 64,
                                    *ext, kernel="wendland_c2")
    assert_map_close(a1.cpu().numpy(), ref)


# ------------------------------------------------------------------ kernel_func plugin
def wendland_c2_numpy(r, h):
    """The same NumPy callable tests/golden/make_golden.py handed the reference for G6."""
    r = np.asarray(r, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64)
    q = r / h
    t = np.clip(1.0 - 0.5 * q, 0.0, None)
    return np.where(q < 2.0, 21.0 / (16.0 * np.pi * h ** 3) * t ** 4 * (1.0 + 2.0 * q), 0.0)


def test_plugin_g6_generic_callable(gpu, monkeypatch):
    """G6 (the reference run with a NumPy Wendland-C2 through its kernel_func plugin
    point, _projector.py:86 / .pyx:33) reproduced by handing create_image the same
    Python callable: the device produces the neighbour pairs and the reference's fp64
    r, the callable runs on the host.  Small pair batches force several device calls."""
    from asp_amd.tools.projections import _plugin, create_image
    monkeypatch.setattr(_plugin, "MAX_PAIRS", 1 << 22)
    pos, h, A, size, cs, ext, _ = g3()
    ref = golden("g6_wendland_c2.npz")["img"]
    calls = []

    def kern(r, hh):
        calls.append(r.size)
        return wendland_c2_numpy(r, hh)

    img = create_image(pos, h, A, size, cs, 2, *ext, kernel_func=kern)
    assert len(calls) > 1
    np.testing.assert_allclose(img, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    assert np.array_equal(img != 0, ref != 0)


def test_plugin_matches_native_kernels(gpu):
    """A Python restatement of the cubic spline through the plugin path equals the
    native kernel within the fp32 bar, on G3 (the reference's own output) and on a
    weighted map."""
    from asp_amd.tools.projections import create_image, create_weighted_image, quartic_spline_kernel

    def cubic(r, hh):
        q = r / hh
        w = np.where(q < 1.0, 1 - 1.5 * q ** 2 + 0.75 * q ** 3,
                     np.where(q < 2.0, 0.25 * (2 - q) ** 3, 0.0))
        return w / (np.pi * hh ** 3)

    pos, h, A, size, cs, ext, ref = g3()
    img = create_image(pos, h, A, size, cs, 2, *ext, kernel_func=cubic)
    np.testing.assert_allclose(img, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    T = np.linspace(1.0, 2.0, h.size)
    r1 = create_weighted_image(pos, h, A, T, size, cs, 2, *ext, kernel_func=cubic)
    r2 = create_weighted_image(pos, h, A, T, size, cs, 2, *ext, kernel_func=quartic_spline_kernel)
    np.testing.assert_allclose(r1, r2, rtol=2e-5)


def test_plugin_per_pixel_mode_is_the_reference(gpu):
    """kernel_func_mode="per_pixel": one call per pixel in the reference's chunk order, on
    the pixel's pairs in particle order (empty arrays included, S15), summed by np.sum as
    .pyx:34 -- G6 (the reference's own output for this callable) reproduced BIT FOR BIT."""
    from asp_amd.tools.projections import create_image
    pos, h, A, size, cs, ext, _ = g3()
    ref = golden("g6_wendland_c2.npz")["img"]
    seen = []

    def kern(r, hh):
        seen.append(r.size)
        return wendland_c2_numpy(r, hh)

    img = create_image(pos, h, A, size, cs, 2, *ext, kernel_func=kern,
                       kernel_func_mode="per_pixel")
    assert len(seen) == size[0] * size[1]  # every pixel (empty ones too: S15)
    np.testing.assert_array_equal(img, ref)


def test_plugin_bins_once_many_batches(gpu, monkeypatch):
    """The plug-in session stages and bins once and emits >= 4 tile-range batches from the
    resident records; deterministic=True (pairs in particle order per pixel) makes the map
    bitwise reproducible and equal to the per-batch-free result within rounding."""
    from asp_amd.tools.projections import _plugin, create_image
    pos, h, A, size, cs, ext, _ = g3()
    ref = golden("g6_wendland_c2.npz")["img"]
    calls = []
    begins = []
    real = _plugin._Session.__init__

    def counting_init(self, *a, **k):
        begins.append(1)
        real(self, *a, **k)

    monkeypatch.setattr(_plugin._Session, "__init__", counting_init)
    monkeypatch.setattr(_plugin, "MAX_PAIRS", 1 << 18)

    def kern(r, hh):
        calls.append(r.size)
        return wendland_c2_numpy(r, hh)

    a = create_image(pos, h, A, size, cs, 2, *ext, kernel_func=kern, deterministic=True)
    assert len(begins) == 1 and len(calls) >= 4
    b = create_image(pos, h, A[::-1].copy()[::-1], size, cs, 2, *ext, kernel_func=kern,
                     deterministic=True)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(a, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def test_plugin_zero_particles(gpu):
    """An empty particle set through the plug-in session (nothing is binned: the emit must
    not read records that were never written): zero maps in both modes, and per_pixel
    still calls the callable once per pixel with empty arrays, as the reference does."""
    from asp_amd.tools.projections import create_image, create_weighted_image
    pos, h, A = np.zeros((0, 3)), np.zeros(0), np.zeros(0)
    seen = []

    def kern(r, hh):
        seen.append(r.size)
        return wendland_c2_numpy(r, hh)

    ext = (-1.0, 1.0, -1.0, 1.0)
    img = create_image(pos, h, A, (96, 80), 32, 2, *ext, kernel_func=kern,
                       kernel_func_mode="per_pixel")
    assert img.shape == (96, 80) and not img.any()
    assert len(seen) == 96 * 80 and not any(seen)
    seen.clear()
    img = create_image(pos, h, A, (96, 80), 32, 2, *ext, kernel_func=kern)
    assert img.shape == (96, 80) and not img.any() and not seen
    w = create_weighted_image(pos, h, A, A, (70, 70), 32, 2, *ext, kernel_func=kern)
    assert not w.any()


def test_plugin_sessions_release_everything(gpu):
    """Every plug-in session owns a workspace with a side stream, events and pinned
    buffers; closing it must release them all (asp_pairs_end).  Hundreds of sessions in a
    row stay correct and leave the device usable."""
    from asp_amd.tools.projections import create_image
    pos, h, A, size, cs, ext, ref = g3()
    sub = slice(0, 500)
    first = None
    for _ in range(300):
        img = create_image(pos[sub], h[sub], A[sub], (64, 64), 32, 2, *ext,
                           kernel_func=lambda r, hh: wendland_c2_numpy(r, hh),
                           deterministic=True)  # pairs in particle order: bitwise sums
        if first is None:
            first = img
        np.testing.assert_array_equal(img, first)
    assert first.any()
