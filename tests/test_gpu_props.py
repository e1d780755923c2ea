"""Several property maps from ONE binning (asp_project2d_props / _props_f64, create_images):
each map equals the single-property projection of the same particles -- the same
neighbour sets (indicator maps exact), values equal up to fp64 summation order -- for 1 to
6 properties (odd counts included), at pixel and physical h (gathered large stream,
wide particles, split tiles), and through the reference-style host API."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b):
    import torch
    torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-7 * float(b.abs().max()) + 1e-30)


@pytest.mark.parametrize("h_law,G,k,wide", [("pixel", 512, 6, None), ("physical", 512, 3, "16"),
                                            ("physical", 1024, 5, None), ("pixel", 256, 4, None)])
def test_props_equal_single_maps(gpu, h_law, G, k, wide, monkeypatch):
    import torch
    from asp_amd.device import project2d, project2d_props, stats
    from asp_amd.plummer import plummer_torch
    if wide:
        monkeypatch.setenv("ASP_WIDE_TILES", wide)
    d = plummer_torch(200_000, seed=7, h_law=h_law, extent=4.0, grid=G, device="cuda")
    u, v, h, m, T = d["x"], d["y"], d["h"], d["m"], d["T"]
    props = [m, (m * T).contiguous(), torch.ones_like(m), T, (m * m).contiguous(),
             (T * 0.5 + 1.0).contiguous()][:k]
    kw = dict(image_size=(G, G), extent=(-4.0, 4.0, -4.0, 4.0), kernel="wendland_c2")
    outs = project2d_props(u, v, h, props, **kw)
    st = stats(0)
    if wide:
        assert st["wide"] > 0
    for a, o in zip(props, outs):
        want, _ = project2d(u, v, h, a, **kw)
        _close(o, want)
    # the same neighbour sets: the indicator kernel's counts, exact
    ones = torch.ones_like(m)
    cnts = project2d_props(u, v, h, [ones] * k, image_size=(G, G), extent=kw["extent"],
                           kernel="indicator")
    want, _ = project2d(u, v, h, ones, image_size=(G, G), extent=kw["extent"], kernel="indicator")
    for c in cnts:
        assert torch.equal(c, want)


def test_create_images_host_api(gpu, oracle):
    """create_images on the reader's raw float64 arrays = create_image per property (the
    fp64 decisions of asp_project2d_f64), and against the oracle within the value bar."""
    from asp_amd.tools.projections import create_image, create_images, indicator_kernel
    from test_gpu_parity import assert_map_close
    rng = np.random.default_rng(4)
    n = 30_000
    pos = rng.normal(0, 0.6, (n, 3))
    h = rng.uniform(0.01, 0.2, n)
    m = rng.uniform(0.5, 1.5, n)
    T = rng.uniform(1e3, 1e5, n)
    size, ext = (300, 200), (-2.0, 2.0, -2.0, 2.0)
    maps = create_images(pos, h, [m, m * T, np.ones(n)], size, 32, "y", *ext)
    for a, got in zip((m, m * T), maps):
        want = create_image(pos, h, a, size, 32, "y", *ext)
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-7 * np.abs(want).max())
    cnt = create_images(pos, h, [np.ones(n), np.ones(n), np.ones(n)], size, 32, 2, *ext,
                        kernel_func=indicator_kernel)
    want = create_image(pos, h, np.ones(n), size, 32, 2, *ext, kernel_func=indicator_kernel)
    for c in cnt:
        assert np.array_equal(c, want)
    o0, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, None, size, 32, *ext)
    mz = create_images(pos, h, [m * T, m], size, 32, 2, *ext)
    assert_map_close(mz[0], o0)


def test_props_argument_errors(gpu):
    import torch
    from asp_amd import _lib
    from asp_amd.device import project2d_props
    from asp_amd.plummer import plummer_torch
    d = plummer_torch(1000, seed=1, h_law="pixel", extent=4.0, grid=64, device="cuda")
    kw = dict(image_size=(64, 64), extent=(-4, 4, -4, 4))
    with pytest.raises(ValueError):
        project2d_props(d["x"], d["y"], d["h"], [d["m"]] * 7, **kw)
    with pytest.raises(ValueError):
        project2d_props(d["x"], d["y"], d["h"], [], **kw)
    P = _lib.ptr
    outs = [torch.empty((64, 64), device="cuda") for _ in range(3)]
    pa = (_lib._f * 3)(*[P(d["m"])] * 3)
    po = (_lib._f * 3)(*[P(o) for o in outs])
    rc = _lib.lib().asp_project2d_props(P(d["x"]), P(d["y"]), P(d["h"]), pa, 3, 1000, -4.0, 4.0,
                                        -4.0, 4.0, 64, 64, 64, 1,
                                        _lib.ASP_F_DEVICE_PTRS | _lib.ASP_F_RATIO, po, 0, None)
    assert rc == _lib.ASP_ERR_UNSUPPORTED


@pytest.mark.parametrize("nprops", [2, 5])
def test_sph_weighted_maps_vs_oracle(gpu, oracle, nprops):
    """asp_project2d_sph (north_star's mass/rho-weighted scatter over (x, y, z, h, m, rho,
    A)): map_k = sum_j (m_j / rho_j) A_kj W against the oracle on the composed property
    A' = A m / rho (fp64); the two-property ratio is the (m/rho)-weighted mean.  rho from
    the Plummer law, so the weights span orders of magnitude.  Reference getters:
    _SnapshotBase.py:833 (get_densities), the maps _projector.py:75-120."""
    import torch
    from asp_amd.device import project2d_props
    from asp_amd.plummer import plummer
    from test_gpu_parity import assert_map_close, assert_ratio_close
    G, ext = 512, (-3.0, 3.0, -3.0, 3.0)
    p = plummer(300_000, seed=13, h_law="physical")
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    x, y, h, m, T = (f32(a) for a in (p["pos"][:, 0], p["pos"][:, 1], p["h"], p["m"], p["T"]))
    rho = f32(p["rho"])
    props = [T, np.ones_like(T), f32(T * T * 1e-4), f32(1.0 + x * x), f32(np.abs(y))][:nprops]
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    kw = dict(image_size=(G, G), extent=ext, kernel="wendland_c2")
    outs = project2d_props(dev(x), dev(y), dev(h), [dev(a) for a in props], mass=dev(m),
                           density=dev(rho), **kw)
    d64 = lambda a: a.astype(np.float64)  # noqa: E731
    w = d64(m) / d64(rho)
    for a, o in zip(props, outs):
        want, _ = oracle.project_scatter(d64(x), d64(y), d64(h), d64(a) * w, None, (G, G), 64,
                                         *ext, kernel="wendland_c2")
        assert_map_close(o.cpu().numpy(), want)
    # rho omitted: mass-weighted sums
    mo = project2d_props(dev(x), dev(y), dev(h), [dev(props[0])], mass=dev(m), **kw)[0]
    want, _ = oracle.project_scatter(d64(x), d64(y), d64(h), d64(props[0]) * d64(m), None,
                                     (G, G), 64, *ext, kernel="wendland_c2")
    assert_map_close(mo.cpu().numpy(), want)
    if nprops == 2:  # the (m/rho)-weighted mean temperature
        q = project2d_props(dev(x), dev(y), dev(h), [dev(T), dev(np.ones_like(T))], mass=dev(m),
                            density=dev(rho), ratio=True, **kw)[0]
        o0, o1 = oracle.project_scatter(d64(x), d64(y), d64(h), d64(T) * w, w, (G, G), 64, *ext,
                                        kernel="wendland_c2")
        assert_ratio_close(q.cpu().numpy(), o0, o1)


def test_sph_weighted_f64_reader_arrays(gpu, oracle):
    """asp_project2d_sph_f64 on the reader's raw fp64 arrays (host): the weights formed in
    fp64 and rounded once; values against the oracle on A m / rho, neighbour sets those of
    the unweighted fp64 path (exact decisions), for a mixed axis spelling too."""
    from asp_amd.device import project2d_props_f64
    from test_gpu_parity import assert_map_close
    rng = np.random.default_rng(31)
    n = 40_000
    pos = rng.normal(0, 0.5, (n, 3))
    h = rng.uniform(0.005, 0.15, n)
    m = rng.uniform(0.5, 2.0, n)
    rho = np.exp(rng.uniform(-6, 3, n))
    A = rng.uniform(1e3, 1e6, n)
    G, ext = (384, 256), (-2.0, 2.0, -2.0, 2.0)
    for axis in (2, 0):
        maps = project2d_props_f64(pos, h, [A, np.ones(n)], projection_axis=axis, image_size=G,
                                   extent=ext, kernel="cubic", mass=m, density=rho)
        cols = {2: (0, 1), 0: (1, 2)}[axis]
        for a, got in zip((A, np.ones(n)), maps):
            want, _ = oracle.project_scatter(pos[:, cols[0]], pos[:, cols[1]], h, a * m / rho,
                                             None, G, 64, *ext, kernel="cubic")
            assert_map_close(got.cpu().numpy(), want)


def test_sph_f64_host_arrays_through_the_c_abi(gpu, oracle):
    """INTEGRATION.md §3's binding: asp_project2d_sph_f64 on the reader's HOST float64
    arrays (no device pointers; positions, h, m, rho and the property staged by the library),
    the map written to a host float32 buffer; ρ NULL gives the mass-weighted map."""
    import ctypes as C
    from asp_amd import _lib
    from test_gpu_parity import assert_map_close
    L = _lib.lib()
    rng = np.random.default_rng(5)
    n, G, ext = 20_000, (200, 160), (-1.5, 1.5, -1.5, 1.5)
    pos = rng.normal(0, 0.4, (n, 3))
    h = rng.uniform(0.01, 0.1, n)
    m = rng.uniform(0.5, 2.0, n)
    rho = np.exp(rng.uniform(-3, 3, n))
    A = rng.uniform(1.0, 10.0, n)
    d = lambda a: a.ctypes.data_as(_lib._d)  # noqa: E731
    for dens in (rho, None):
        img = np.zeros(G, np.float32)
        props = (_lib._d * 1)(d(A))
        outs = (_lib._f * 1)(img.ctypes.data_as(_lib._f))
        rc = L.asp_project2d_sph_f64(d(pos), d(h), d(m), d(dens) if dens is not None else None,
                                     props, 1, n, 2, *ext, G[0], G[1], 32, 0, 0, outs, 0, None)
        _lib.check(rc)
        w = m / dens if dens is not None else m
        want, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, A * w, None, G, 32, *ext,
                                         kernel="cubic")
        assert_map_close(img, want)
