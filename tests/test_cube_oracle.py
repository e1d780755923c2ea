"""The cube restatement (oracle/asp_oracle.c: oracle_project3d, oracle_voxel_neighbours).

The reference has no volumetric path, so the cube's parity is pinned by this
restatement alone ("parity unpinned by the reference").  These CPU tests
tie the C restatement to an independent NumPy brute force of the same definition and
to physical properties of an SPH density field.
"""
import numpy as np
import pytest

EXT = (-1.0, 1.0, -0.8, 1.2, -1.1, 0.9)


def _numpy_cube(x, y, z, h, a, size, ext, kernel, planes=None):
    """Brute force of the definition: every (particle, voxel) pair, fp64."""
    import pyoracle
    nx, ny, nz = size
    k_lo, k_hi = (0, nz) if planes is None else planes
    X = ext[0] + np.arange(nx) * ((ext[1] - ext[0]) / nx)
    Y = ext[2] + np.arange(ny) * ((ext[3] - ext[2]) / ny)
    Z = ext[4] + np.arange(k_lo, k_hi) * ((ext[5] - ext[4]) / nz)
    out = np.zeros((nx, ny, k_hi - k_lo))
    for p in range(x.size):
        dx = (x[p] - X)[:, None, None]
        dy = (y[p] - Y)[None, :, None]
        dz = (z[p] - Z)[None, None, :]
        r2 = dx * dx + dy * dy + dz * dz
        t = 2.0 * h[p]
        m = r2 < t * t
        if m.any():
            w = pyoracle.kernel_eval(kernel, np.sqrt(r2[m]), np.full(m.sum(), h[p]))
            out[m] += a[p] * w
    return out


def _particles(n, seed, hscale=0.12):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1.2, 1.2, n)
    y = rng.uniform(-1.0, 1.4, n)
    z = rng.uniform(-1.3, 1.1, n)
    h = rng.uniform(0.2, 1.0, n) * hscale
    a = rng.uniform(0.5, 2.0, n)
    return x, y, z, h, a


@pytest.mark.parametrize("kernel", ["cubic", "wendland_c2", "indicator"])
def test_cube_oracle_matches_bruteforce(oracle, kernel):
    x, y, z, h, a = _particles(300, 1)
    size = (12, 10, 14)
    got = oracle.project3d(x, y, z, h, a, size, EXT, kernel=kernel)
    ref = _numpy_cube(x, y, z, h, a, size, EXT, kernel)
    assert np.array_equal(got != 0, ref != 0)  # identical neighbour structure
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def test_cube_oracle_plane_slabs_compose(oracle):
    x, y, z, h, a = _particles(400, 2)
    size = (9, 11, 13)
    full = oracle.project3d(x, y, z, h, a, size, EXT)
    parts = [oracle.project3d(x, y, z, h, a, size, EXT, planes=(k0, k1))
             for k0, k1 in ((0, 4), (4, 5), (5, 13))]
    assert np.array_equal(np.concatenate(parts, axis=2), full)


def test_cube_oracle_neighbour_sets(oracle):
    x, y, z, h, a = _particles(500, 3, hscale=0.2)
    size = (8, 8, 8)
    rng = np.random.default_rng(0)
    vox = rng.choice(512, 40, replace=False)
    offs, idx = oracle.voxel_neighbours(x, y, z, h, size, EXT, vox)
    cnt = oracle.project3d(x, y, z, h, np.ones_like(h), size, EXT, kernel="indicator")
    assert np.array_equal(np.diff(offs), cnt.reshape(-1)[vox].astype(np.int64))
    # brute force membership for a few voxels
    nx, ny, nz = size
    for q in range(5):
        v = vox[q]
        i, j, k = v // (ny * nz), (v // nz) % ny, v % nz
        X = EXT[0] + i * ((EXT[1] - EXT[0]) / nx)
        Y = EXT[2] + j * ((EXT[3] - EXT[2]) / ny)
        Z = EXT[4] + k * ((EXT[5] - EXT[4]) / nz)
        r2 = (x - X) ** 2 + (y - Y) ** 2 + (z - Z) ** 2
        assert np.array_equal(np.nonzero(r2 < (2 * h) ** 2)[0], idx[offs[q]:offs[q + 1]])


def test_cube_oracle_density_integrates_to_mass(oracle):
    """Well-resolved particles (2h >> voxel) inside the box: sum(rho) dV = sum(m)."""
    rng = np.random.default_rng(4)
    n = 30
    x, y, z = (rng.uniform(-0.4, 0.4, n) for _ in range(3))
    h = np.full(n, 0.15)
    m = rng.uniform(0.5, 1.5, n)
    size = (48, 48, 48)
    ext = (-1.0, 1.0, -1.0, 1.0, -1.0, 1.0)
    for kernel in ("cubic", "wendland_c2"):
        rho = oracle.project3d(x, y, z, h, m, size, ext, kernel=kernel)
        dV = (2.0 / 48) ** 3
        assert abs(rho.sum() * dV / m.sum() - 1.0) < 2e-3


def test_cube_oracle_edge_cases(oracle):
    size = (6, 5, 7)
    x, y, z, h, a = (np.array([0.0]),) * 3 + (np.array([0.0]), np.array([1.0]))
    assert not oracle.project3d(x, y, z, h, a, size, EXT).any()  # h = 0: no neighbours
    far = oracle.project3d(np.array([50.0]), np.array([0.0]), np.array([0.0]),
                           np.array([0.1]), np.array([1.0]), size, EXT)
    assert not far.any()
    empty = oracle.project3d(np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0),
                             size, EXT)
    assert empty.shape == size and not empty.any()
