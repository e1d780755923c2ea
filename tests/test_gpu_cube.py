"""GPU parity of the voxel cube (asp_project3d through the C-ABI) against the CPU
restatement oracle_project3d on identical (fp32-rounded) inputs.

Bars: per-voxel neighbour counts (indicator kernel) BIT-EXACT; values within the map's
fp32 tolerance (|g - r| <= 2e-5 max|r| everywhere, <= 1e-4 |r| where |r| >= 1e-3 max|r|);
voxels that are 0 in the oracle are exactly 0.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_map_close

pytestmark = pytest.mark.gpu

EXT = (-2.0, 2.0, -2.0, 2.0, -2.0, 2.0)


def _f32(*arrs):
    return [np.asarray(a, np.float32).astype(np.float64) for a in arrs]


def _plummer(n, seed, size):
    from asp_amd.plummer import plummer
    p = plummer(n, seed=seed, h_law="physical")
    x, y, z = (p["pos"][:, c] for c in range(3))
    return _f32(x, y, z, p["h"], p["m"])


@pytest.mark.parametrize("size", [(64, 64, 64), (40, 24, 70), (17, 33, 5)])
def test_cube_counts_bitexact(gpu, oracle, size):
    from asp_amd.tools.projections import create_cube, indicator_kernel
    x, y, z, h, m = _plummer(20000, 5, size)
    ones = np.ones_like(h)
    pos = np.stack([x, y, z], axis=1)
    g = create_cube(pos, h, ones, size, *EXT, kernel_func=indicator_kernel)
    r = oracle.project3d(x, y, z, h, ones, size, EXT, kernel="indicator")
    assert g.shape == r.shape == size
    assert np.array_equal(g, r), f"{np.count_nonzero(g != r)} voxels differ"


@pytest.mark.parametrize("kernel", ["cubic", "wendland_c2"])
def test_cube_density_matches_oracle(gpu, oracle, kernel):
    from asp_amd.tools.projections import create_cube, quartic_spline_kernel, wendland_c2_kernel
    kf = quartic_spline_kernel if kernel == "cubic" else wendland_c2_kernel
    size = (48, 56, 64)
    x, y, z, h, m = _plummer(30000, 6, size)
    g = create_cube(np.stack([x, y, z], 1), h, m, size, *EXT, kernel_func=kf)
    r = oracle.project3d(x, y, z, h, m, size, EXT, kernel=kernel)
    assert_map_close(g, r)


def test_cube_planes_compose(gpu):
    from asp_amd.tools.projections import create_cube
    size = (32, 32, 96)
    x, y, z, h, m = _plummer(20000, 7, size)
    pos = np.stack([x, y, z], 1)
    full = create_cube(pos, h, m, size, *EXT)
    parts = [create_cube(pos, h, m, size, *EXT, planes=p) for p in ((0, 31), (31, 33), (33, 96))]
    cat = np.concatenate(parts, axis=2)
    assert_map_close(cat, full, abs_tol=1e-6, rel_tol=1e-5)
    assert np.array_equal(cat != 0, full != 0)


def test_cube_large_particles_and_split_bricks(gpu, oracle):
    """Footprints spanning many bricks (wave sweeps), and bricks with enough records to
    be split over several work items (fp64 slab merge)."""
    from asp_amd.tools.projections import create_cube, indicator_kernel
    rng = np.random.default_rng(8)
    n = 6000
    x, y, z = _f32(*(rng.normal(0.0, 0.05, n) for _ in range(3)))  # dense core
    h, = _f32(rng.uniform(0.02, 0.05, n))
    bx, by, bz = _f32(*(rng.uniform(-1, 1, 20) for _ in range(3)))
    bh, = _f32(rng.uniform(0.3, 0.9, 20))
    x, y, z, h = (np.concatenate(t) for t in ((x, bx), (y, by), (z, bz), (h, bh)))
    size = (64, 64, 64)
    pos = np.stack([x, y, z], 1)
    ones = np.ones_like(h)
    g = create_cube(pos, h, ones, size, *EXT, kernel_func=indicator_kernel)
    r = oracle.project3d(x, y, z, h, ones, size, EXT, kernel="indicator")
    assert np.array_equal(g, r)
    m, = _f32(rng.uniform(0.5, 1.5, x.size))
    g = create_cube(pos, h, m, size, *EXT)
    r = oracle.project3d(x, y, z, h, m, size, EXT)
    assert_map_close(g, r)


def test_cube_edge_cases(gpu, oracle):
    from asp_amd.tools.projections import create_cube
    size = (20, 18, 40)
    z3 = np.zeros((0, 3))
    e = create_cube(z3, np.zeros(0), np.zeros(0), size, *EXT)
    assert e.shape == size and not e.any()
    # h = 0, non-finite and far-away particles contribute nothing
    pos = np.array([[0.0, 0.0, 0.0], [np.nan, 0, 0], [0, 0, np.inf], [50.0, 0, 0]])
    c = create_cube(pos, np.array([0.0, 0.5, 0.5, 0.5]), np.ones(4), size, *EXT)
    assert not c.any()
    # one particle whose footprint covers the whole cube
    pos = np.array([[0.1, -0.2, 0.05]])
    x, y, z, h, a = _f32(pos[:, 0], pos[:, 1], pos[:, 2], [3.0], [2.0])
    g = create_cube(np.stack([x, y, z], 1), h, a, size, *EXT)
    r = oracle.project3d(x, y, z, h, a, size, EXT)
    assert np.count_nonzero(r) > 0.5 * r.size
    assert_map_close(g, r)
    with pytest.raises(ValueError):
        create_cube(pos, [0.1], [1.0], size, 1.0, -1.0, *EXT[2:])
    with pytest.raises(NotImplementedError):  # one brick column of > 16384 bricks
        create_cube(pos, [0.1], [1.0], (16, 8192, 2048), *EXT)


def test_cube_device_api_accumulate(gpu):
    import torch
    from asp_amd.device import project3d
    from asp_amd.plummer import plummer_torch
    d = plummer_torch(50000, seed=3, h_law="physical", device="cuda:0")
    size, ext = (64, 64, 64), EXT
    c1 = project3d(d["x"], d["y"], d["z"], d["h"], d["m"], cube_size=size, extent=ext)
    c2 = project3d(d["x"], d["y"], d["z"], d["h"], d["m"], cube_size=size, extent=ext,
                   out=c1.clone(), accumulate=True)
    torch.cuda.synchronize()
    assert torch.allclose(c2, 2 * c1, rtol=1e-6, atol=0)
    # permutation of the input: same cube to fp32 rounding of the fp64 sums
    perm = torch.randperm(d["x"].numel(), device="cuda:0")
    c3 = project3d(*(d[k][perm].contiguous() for k in ("x", "y", "z", "h", "m")),
                   cube_size=size, extent=ext)
    assert torch.equal(c3 != 0, c1 != 0)
    assert torch.allclose(c3, c1, rtol=1e-5, atol=1e-6 * float(c1.abs().max()))


def test_cube_record_placement_trials(gpu, oracle, monkeypatch):
    """The placement trials of a fresh record buffer (the probe scatter run into several
    candidate buffers, the fastest kept holding the call's records) leave the voxel counts
    exact and the density within the bar."""
    from asp_amd import _lib
    from asp_amd.tools.projections import create_cube, indicator_kernel, wendland_c2_kernel
    size = (48, 48, 64)
    x, y, z, h, m = _plummer(30000, 9, size)
    pos = np.stack([x, y, z], axis=1)
    monkeypatch.setenv("ASP_PLACEMENT_TRIALS", "4")
    monkeypatch.setenv("ASP_PLACEMENT_MIN_MB", "0")
    _lib.check(_lib.lib().asp_release(0))
    ones = np.ones_like(h)
    g = create_cube(pos, h, ones, size, *EXT, kernel_func=indicator_kernel)
    assert np.array_equal(g, oracle.project3d(x, y, z, h, ones, size, EXT, kernel="indicator"))
    _lib.check(_lib.lib().asp_release(0))
    d = create_cube(pos, h, m, size, *EXT, kernel_func=wendland_c2_kernel)
    assert_map_close(d, oracle.project3d(x, y, z, h, m, size, EXT, kernel="wendland_c2"))
    _lib.check(_lib.lib().asp_release(0))


def test_cube_x_windows_beyond_16384_bricks(gpu, oracle):
    """A 640 x 512 x 512 cube (20480 bricks): two x windows of whole brick columns, each a
    pass over all particles; counts bit-exact and density within the bar across the seam."""
    from asp_amd.tools.projections import create_cube, indicator_kernel
    size = (640, 512, 512)
    x, y, z, h, m = _plummer(150_000, 12, size)
    pos = np.stack([x, y, z], 1)
    ext = (-3.0, 3.0, -2.4, 2.4, -2.4, 2.4)
    ones = np.ones_like(h)
    g = create_cube(pos, h, ones, size, *ext, kernel_func=indicator_kernel)
    r = oracle.project3d(x, y, z, h, ones, size, ext, kernel="indicator")
    assert np.array_equal(g, r), f"{np.count_nonzero(g != r)} voxels differ"
    seam = 16 * (16384 // (32 * 16))  # first x plane of the second window
    assert r[seam - 1].sum() > 0 and r[seam].sum() > 0
    del g, r
    d = create_cube(pos, h, m, size, *ext)
    assert_map_close(d, oracle.project3d(x, y, z, h, m, size, ext))


def test_cube_axis_beyond_32768_multibrick(gpu, oracle):
    """An elongated 40000 x 40 x 36 cube: particles near voxel 32768 and beyond, with
    footprints over several 16 x 16 x 32 bricks (the scatter's multi-brick deal).  Voxel
    bounds past 32767 used to be packed in 16-bit halves of a signed word;
    counts bit-exact and density within the bar against oracle_project3d."""
    from asp_amd.tools.projections import create_cube, indicator_kernel
    size = (40000, 40, 36)
    ext = (0.0, 4000.0, 0.0, 4.0, 0.0, 3.6)  # 0.1 per voxel on every axis
    rng = np.random.default_rng(17)
    n = 3000
    x = np.concatenate([rng.uniform(3200.0, 3400.0, n // 2), rng.uniform(3900.0, 4000.0, n // 2)])
    y = rng.uniform(0.0, 4.0, n)
    z = rng.uniform(0.0, 3.6, n)
    h = rng.uniform(0.3, 1.2, n)  # 2h of 6-24 voxels: several bricks per particle
    m = rng.uniform(0.5, 2.0, n)
    x, y, z, h, m = _f32(x, y, z, h, m)
    pos = np.stack([x, y, z], 1)
    ones = np.ones_like(h)
    g = create_cube(pos, h, ones, size, *ext, kernel_func=indicator_kernel)
    r = oracle.project3d(x, y, z, h, ones, size, ext, kernel="indicator")
    assert r[32768:].sum() > 0 and r[32000:32768].sum() > 0
    assert np.array_equal(g, r), f"{np.count_nonzero(g != r)} voxels differ"
    del g, r
    d = create_cube(pos, h, m, size, *ext)
    assert_map_close(d, oracle.project3d(x, y, z, h, m, size, ext))


@pytest.mark.parametrize("knob", [("ASP_MAX_BATCH", "7000"), ("ASP_MAX_RECORDS", "9000")])
def test_cube_particle_batches(gpu, oracle, monkeypatch, knob):
    from asp_amd.tools.projections import create_cube, indicator_kernel
    size = (40, 48, 64)
    x, y, z, h, m = _plummer(30000, 13, size)
    pos = np.stack([x, y, z], 1)
    monkeypatch.setenv(*knob)
    ones = np.ones_like(h)
    g = create_cube(pos, h, ones, size, *EXT, kernel_func=indicator_kernel)
    d = create_cube(pos, h, m, size, *EXT)
    monkeypatch.delenv(knob[0])
    assert np.array_equal(g, oracle.project3d(x, y, z, h, ones, size, EXT, kernel="indicator"))
    assert_map_close(d, oracle.project3d(x, y, z, h, m, size, EXT))


def test_cube_speculative_scatter_buffer_growth(gpu, oracle):
    """The cube scatter is enqueued before the host reads the record count when a record
    buffer is left from an earlier call (round 5): a small call, then one needing a larger
    buffer (the speculative launch must be a no-op, the buffer grows, the records are
    scattered again), then the small one again (fits: the speculative launch is the
    scatter).  Counts bit-exact each time."""
    from asp_amd import _lib
    from asp_amd.tools.projections import create_cube, indicator_kernel
    _lib.check(_lib.lib().asp_release(0))
    size = (48, 48, 48)
    for n, seed in ((5000, 11), (60000, 12), (5000, 13)):
        x, y, z, h, m = _plummer(n, seed, size)
        ones = np.ones_like(h)
        g = create_cube(np.stack([x, y, z], 1), h, ones, size, *EXT, kernel_func=indicator_kernel)
        r = oracle.project3d(x, y, z, h, ones, size, EXT, kernel="indicator")
        assert np.array_equal(g, r), (n, np.count_nonzero(g != r))
