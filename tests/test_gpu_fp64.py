"""GPU parity on raw float64 inputs and at BASELINE.json sizes.

create_image hands the reader's float64 arrays to asp_project2d_f64: float32 working
copies in HBM for the fast decision, the float64 originals for every pair inside the
error band.  So the neighbour sets are the reference's on the float64 inputs themselves
(_pixel_calculations.pyx:9, :30-31: double[:, :] input, strict <), not on their float32
roundings.  Bars as tests/test_gpu_parity.py: counts / index checksums bit-exact, values
|g - r| <= 2e-5 max|r| and <= 1e-4 |r| where |r| >= 1e-3 max|r|, zeros stay zero.
"""
import numpy as np
import pytest

from conftest import golden
from test_gpu_parity import assert_map_close, assert_ratio_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g10():
    return golden("g10_fp64_axes.npz")


def test_g10_plummer_raw_fp64(gpu, g10):
    from asp_amd.tools.projections import create_image, indicator_kernel
    pos, h, A = g10["plummer_pos"], g10["plummer_h"], g10["plummer_A"]
    size, cs, ext = tuple(g10["plummer_size"]), int(g10["plummer_cs"]), tuple(g10["plummer_ext"])
    assert_map_close(create_image(pos, h, A, size, cs, 2, *ext), g10["plummer_img"])
    n = h.size
    cnt = create_image(pos, h, np.ones(n), size, cs, 2, *ext, kernel_func=indicator_kernel)
    assert np.array_equal(cnt, g10["plummer_cnt"])
    ids = (np.arange(n) % 4093).astype(np.float64)
    chk = create_image(pos, h, ids, size, cs, 2, *ext, kernel_func=indicator_kernel)
    assert np.array_equal(chk, g10["plummer_ids"])


def test_g10_edge_pairs_fp64(gpu, g10):
    """Pairs at 2h +- a few fp64 ulps; > 1000 of them would flip if the inputs were
    rounded to float32 first.  Counts and index checksums bit-exact."""
    from asp_amd.tools.projections import create_image, indicator_kernel
    pos, h = g10["edge_pos"], g10["edge_h"]
    size, cs, ext = tuple(g10["edge_size"]), int(g10["edge_cs"]), tuple(g10["edge_ext"])
    n = h.size
    cnt = create_image(pos, h, np.ones(n), size, cs, 2, *ext, kernel_func=indicator_kernel)
    assert np.array_equal(cnt, g10["edge_cnt"])
    ids = (np.arange(n) % 4093).astype(np.float64)
    chk = create_image(pos, h, ids, size, cs, 2, *ext, kernel_func=indicator_kernel)
    assert np.array_equal(chk, g10["edge_ids"])
    # the same float64 values fed through the float32 entry point DO differ: the fp64
    # path is what makes the sets exact
    f32 = create_image(pos.astype(np.float32).astype(np.float64), h.astype(np.float32).astype(np.float64),
                       np.ones(n), size, cs, 2, *ext, kernel_func=indicator_kernel)
    assert not np.array_equal(f32, g10["edge_cnt"])


def test_g10_axis_spellings(gpu, g10):
    """Every axis spelling as the reference treats it, incl. the str "x" that culls on the
    Z columns but measures distances on the X ones (ASP_AXIS_CULL), on a non-square
    image."""
    from asp_amd import CoordinateAxes
    from asp_amd.tools.projections import create_image, indicator_kernel
    pos, h, A = g10["axes_pos"], g10["axes_h"], g10["axes_A"]
    size, cs, ext = tuple(g10["axes_size"]), int(g10["axes_cs"]), tuple(g10["axes_ext"])
    sp = {"enumX": CoordinateAxes.X, "enumY": CoordinateAxes.Y, "enumZ": CoordinateAxes.Z,
          "strx": "x", "stry": "y", "strz": "z", "strX": "X", "int0": 0, "int1": 1,
          "bytesx": b"x"}
    for key in g10["axes_keys"]:
        ax = sp[str(key)]
        assert_map_close(create_image(pos, h, A, size, cs, ax, *ext), g10[f"axes_img_{key}"])
        cnt = create_image(pos, h, np.ones(h.size), size, cs, ax, *ext,
                           kernel_func=indicator_kernel)
        assert np.array_equal(cnt, g10[f"axes_cnt_{key}"]), key


def _plummer(n, seed, h_law, grid):
    from asp_amd.plummer import plummer
    return plummer(n, seed=seed, h_law=h_law, grid=grid)


def test_baseline_cfg3_4096_weighted_wendland_pixel_h(gpu, oracle):
    """BASELINE configs[2]'s map (mass-weighted temperature, Wendland-C2, pixel-scale h)
    at its full 4096^2 grid with 2 x 10^6 raw-fp64 Plummer particles: 4096 GPU tiles,
    both map components and the ratio against the oracle on the same float64 arrays."""
    from asp_amd.device import stats
    from asp_amd.tools.projections import (create_image, create_weighted_image,
                                           indicator_kernel, wendland_c2_kernel)
    n, G = 2_000_000, 4096
    p = _plummer(n, 41, "pixel", G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    ext = (-4.0, 4.0, -4.0, 4.0)
    r, s0, s1 = create_weighted_image(pos, h, m, T, (G, G), 64, 2, *ext,
                                      kernel_func=wendland_c2_kernel, return_components=True)
    assert stats(0)["tiles"] == 4096
    o0, o1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, m, (G, G), 64, *ext,
                                    kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    assert_ratio_close(r, o0, o1)
    cnt = create_image(pos, h, np.ones(n), (G, G), 64, 2, *ext, kernel_func=indicator_kernel)
    c_ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 64,
                                      *ext, kernel="indicator")
    assert np.array_equal(cnt, c_ref)
    assert cnt.sum() > 5 * n  # ~7 pairs per particle at pixel-scale h


def test_baseline_cfg3_4096_deterministic_components(gpu, oracle):
    """The int64 fixed-point accumulation (ASP_F_DETERMINISTIC) on BASELINE configs[2]'s map
    (4096^2, Wendland-C2, pixel h, 2 x 10^6 raw-fp64 Plummer particles): both component maps
    (m T and m, two outputs, no ratio) against the oracle within the value bar, and bitwise
    reproducible under a permutation of the particles.  A RATIO map of fixed-point
    components is refused (ASP_ERR_INVALID / ValueError): pixels reached only by kernel
    tails keep a few fixed-point units of weight."""
    import torch
    from asp_amd.device import project2d, project2d_f64
    from asp_amd.tools.projections import create_weighted_image, wendland_c2_kernel
    n, G = 2_000_000, 4096
    p = _plummer(n, 41, "pixel", G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    ext = (-4.0, 4.0, -4.0, 4.0)
    kw = dict(image_size=(G, G), extent=ext, chunk_size=64, kernel="wendland_c2",
              deterministic=True)
    s0, s1 = project2d_f64(pos, h, m * T, m, **kw)
    o0, o1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, m, (G, G), 64, *ext,
                                    kernel="wendland_c2")
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)
    perm = np.random.default_rng(3).permutation(n)
    q0, q1 = project2d_f64(pos[perm], h[perm], (m * T)[perm], m[perm], **kw)
    assert np.array_equal(q0, s0) and np.array_equal(q1, s1)
    with pytest.raises(ValueError):
        create_weighted_image(pos, h, m, T, (G, G), 64, 2, *ext, kernel_func=wendland_c2_kernel,
                              deterministic=True)
    t = [torch.from_numpy(x.astype(np.float32)).cuda() for x in (pos[:1000, 0], pos[:1000, 1],
                                                               h[:1000], m[:1000] * T[:1000], m[:1000])]
    with pytest.raises(ValueError, match="DETERMINISTIC"):  # ASP_ERR_INVALID
        project2d(*t, image_size=(64, 64), extent=ext, kernel="wendland_c2", ratio=True,
                  deterministic=True)


def test_deterministic_components_physical_h(gpu, oracle):
    """The same components at physical h (gathered large stream and split tiles: every
    fixed-point deposit path)."""
    from asp_amd.device import project2d_f64, stats
    n, G = 400_000, 1024
    p = _plummer(n, 43, "physical", G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    ext = (-4.0, 4.0, -4.0, 4.0)
    s0, s1 = project2d_f64(pos, h, m * T, m, image_size=(G, G), extent=ext, chunk_size=64,
                           kernel="cubic", deterministic=True)
    st = stats(0)
    assert st["large"] > 0 and st["merges"] > 0
    o0, o1 = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m * T, m, (G, G), 64, *ext)
    assert_map_close(s0, o0)
    assert_map_close(s1, o1)


def test_baseline_cfg2_2048_cubic_physical_h(gpu, oracle):
    """BASELINE configs[1]'s map (surface density, cubic spline) at its full 2048^2 grid in
    the physical-h regime (~8.6e9 pairs from 10^6 raw-fp64 particles: the large stream /
    gathered deposit, wide particles and split tiles all run)."""
    from asp_amd.device import stats
    from asp_amd.tools.projections import create_image, indicator_kernel
    n, G = 1_000_000, 2048
    p = _plummer(n, 5, "physical", G)
    pos, h, m = p["pos"], p["h"], p["m"]
    ext = (-4.0, 4.0, -4.0, 4.0)
    img = create_image(pos, h, m, (G, G), 64, 2, *ext)
    st = stats(0)
    assert st["large"] > 0 and st["merges"] > 0
    ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, m, None, (G, G), 64, *ext,
                                    kernel="cubic")
    assert_map_close(img, ref)
    cnt = create_image(pos, h, np.ones(n), (G, G), 64, 2, *ext, kernel_func=indicator_kernel)
    c_ref, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, (G, G), 64,
                                      *ext, kernel="indicator")
    assert np.array_equal(cnt, c_ref)


def test_raw_fp64_nonsquare_mixed_axis_vs_oracle(gpu, oracle):
    """Larger raw-fp64 case on a non-square image with the reference's mixed "y" spelling
    (cull on x/y, pixel test on x/z) against the oracle: counts bit-exact, values within
    the bar."""
    from asp_amd._axes import reference_axes
    from asp_amd.tools.projections import create_image, indicator_kernel
    rng = np.random.default_rng(77)
    n = 200_000
    pos = rng.normal(0, 0.5, (n, 3))
    h = rng.uniform(0.001, 0.02, n)
    A = rng.uniform(0.5, 2.0, n)
    size, cs, ext = (384, 512), 48, (-1.5, 1.5, -1.2, 1.8)
    ax = reference_axes("y")
    assert ax == (1, 2)
    img = create_image(pos, h, A, size, cs, "y", *ext)
    u, v, cu, cv = oracle._axes(pos, ax)
    ref, _ = oracle.project_scatter(u, v, h, A, None, size, cs, *ext, cu=cu, cv=cv)
    assert_map_close(img, ref)
    cnt = create_image(pos, h, np.ones(n), size, cs, "y", *ext, kernel_func=indicator_kernel)
    c_ref, _ = oracle.project_scatter(u, v, h, np.ones(n), None, size, cs, *ext,
                                      kernel="indicator", cu=cu, cv=cv)
    assert np.array_equal(cnt, c_ref)


def test_host_inputs_device_outputs_pinned_staging(gpu):
    """Reader fp64 host arrays -> pinned bounce buffers (several 32 MiB pieces: 3e6
    particles = 72 MB of positions) -> device map (ASP_F_DEVICE_OUTPUTS, the RCCL-sum
    input of project2d_sharded_host): bit-identical to the host-output call, and to the
    same arrays handed over as device tensors."""
    import torch
    from asp_amd.device import project2d_f64
    rng = np.random.default_rng(5)
    n = 3_000_000
    pos = rng.normal(0, 0.6, (n, 3))
    h = rng.uniform(0.002, 0.01, n)
    a0, a1 = rng.uniform(0.5, 2.0, n), rng.uniform(0.5, 2.0, n)
    # fixed-point accumulation: bitwise reproducible, so the three calls must agree exactly
    kw = dict(image_size=(512, 384), extent=(-2.0, 2.0, -1.5, 1.5), kernel="wendland_c2",
              deterministic=True)
    r0, r1 = project2d_f64(pos, h, a0, a1, **kw)
    d0, d1 = project2d_f64(pos, h, a0, a1, device_out=True, **kw)
    assert d0.is_cuda and d1.is_cuda
    assert np.array_equal(d0.cpu().numpy(), r0) and np.array_equal(d1.cpu().numpy(), r1)
    t = [torch.from_numpy(x).cuda() for x in (pos, h, a0, a1)]
    e0, e1 = project2d_f64(*t, **kw)
    assert np.array_equal(e0.cpu().numpy(), r0) and np.array_equal(e1.cpu().numpy(), r1)


def test_sharded_host_arrays_single_rank_hip_path(gpu):
    """project2d_sharded_host through the real HIP path (a world-1 gloo group on the GPU
    box): the rank's fp64 host arrays -> pinned staging -> device maps -> collective ->
    ratio on the device; equal to project2d_f64 on the same arrays (fixed point: bitwise)."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from asp_amd.device import project2d_f64
    from asp_amd.distributed import project2d_sharded_host
    rng = np.random.default_rng(8)
    n = 400_000
    pos = rng.normal(0, 0.5, (n, 3))
    h = rng.uniform(0.003, 0.02, n)
    m, T = rng.uniform(0.5, 2.0, n), rng.uniform(1e3, 1e5, n)
    # fp64 accumulation: a ratio map of fixed-point components is refused
    kw = dict(image_size=(256, 256), extent=(-2.0, 2.0, -2.0, 2.0), chunk_size=64,
              kernel="wendland_c2")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        r, _ = project2d_sharded_host(pos, h, m * T, m, ratio=True, op="reduce", **kw)
    finally:
        dist.destroy_process_group()
    c0, c1 = project2d_f64(pos, h, m * T, m, **{k: v for k, v in kw.items()})
    want = np.where(c1 != 0, c0 / np.where(c1 != 0, c1, 1), 0).astype(np.float32)
    got = r.cpu().numpy()
    assert r.is_cuda
    # separate fp64-accumulated calls: LDS-atomic order moves the fp32 maps by an ulp or so
    np.testing.assert_array_equal(got == 0, want == 0)
    np.testing.assert_allclose(got, want, rtol=2e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("h_law,G", [("pixel", 4096), ("physical", 1024)])
def test_split_tile_scan_same_maps(gpu, monkeypatch, h_law, G):
    """The tile scan in two parts (ASP_SPLIT_SCAN, default on: tile starts on the map's
    stream, work items / merge list / dispatch order on the side stream beside the scatter)
    gives the one-launch scan's maps bit for bit in the deterministic (fixed-point) mode,
    small and mid items, gathered large stream and split tiles included."""
    from asp_amd.device import project2d_f64, stats
    n = 400_000
    p = _plummer(n, 47, h_law, G)
    pos, h, m, T = p["pos"], p["h"], p["m"], p["T"]
    kw = dict(image_size=(G, G), extent=(-4.0, 4.0, -4.0, 4.0), chunk_size=64, kernel="cubic",
              deterministic=True)
    monkeypatch.setenv("ASP_SPLIT_SCAN", "0")
    a0, a1 = project2d_f64(pos, h, m * T, m, **kw)
    one = stats(0)
    monkeypatch.setenv("ASP_SPLIT_SCAN", "1")
    b0, b1 = project2d_f64(pos, h, m * T, m, **kw)
    two = stats(0)
    assert np.array_equal(a0, b0) and np.array_equal(a1, b1)
    assert one["items"] == two["items"] and one["merges"] == two["merges"]
    if h_law == "physical":
        assert two["large"] > 0 and two["merges"] > 0
