"""k-th nearest-neighbour smoothing lengths against the reference's
own dependency: scipy.spatial.KDTree (scipy 1.15.3 in this image), queried exactly as
io/SWIFT/_SnapshotSWIFT.py:62-83 does -- ``tree.query(pos, k)[0][:, k - 1]``.

Bar: BIT-EXACT fp64 (same Euclidean arithmetic; the k-th smallest distance is unique
whatever the tie order).  The CPU test pins the distance formula the device uses to
scipy's; the GPU tests compare the device with scipy on uniform, clustered, lattice (many
exact ties), duplicate-point and tiny inputs.
"""
import numpy as np
import pytest
from scipy.spatial import KDTree


def scipy_h(pos, k):
    d = KDTree(pos).query(pos, k=k)[0]
    return d if k == 1 else d[:, k - 1]


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


def brute_h(pos, k):
    """The device's definition: k-th smallest of ((dx^2 + dy^2) + dz^2), then sqrt."""
    d = pos[:, None, :] - pos[None, :, :]
    d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    return np.sqrt(np.sort(d2, axis=1)[:, k - 1])


@pytest.mark.parametrize("k", [1, 8, 32])
def test_distance_formula_is_scipys(k):
    """CPU: the brute-force restatement of the device's arithmetic is bit-identical to
    scipy's KDTree on random, clustered and lattice points."""
    rng = np.random.default_rng(1)
    sets = [rng.uniform(-3, 7, (400, 3)), rng.standard_normal((400, 3)) * np.array([1e-3, 2.0, 5.0]),
            np.stack(np.meshgrid(*[np.arange(7.0) * 0.3] * 3, indexing="ij"), -1).reshape(-1, 3)]
    for pos in sets:
        assert np.array_equal(bits(brute_h(pos, k)), bits(scipy_h(pos, k)))


def _plummer(n, seed):
    from asp_amd.plummer import plummer
    return plummer(n, seed=seed, h_law="pixel", grid=64)["pos"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform", "plummer", "lattice", "duplicates", "flat"])
def test_knn_bitexact_vs_scipy(gpu, kind):
    from asp_amd.knn import knn_smoothing_lengths
    rng = np.random.default_rng(2)
    if kind == "uniform":
        pos = rng.uniform(0.0, 25.0, (100_000, 3))
    elif kind == "plummer":
        pos = _plummer(100_000, 3)
    elif kind == "lattice":  # many exactly tied distances
        g = np.arange(40.0) * 0.5
        pos = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    elif kind == "duplicates":
        base = rng.uniform(0.0, 1.0, (3000, 3))
        pos = np.concatenate([base] * 12 + [rng.uniform(0.0, 1.0, (5000, 3))])
    else:  # all points in a plane, one axis of zero extent
        pos = np.concatenate([rng.uniform(0, 1, (50_000, 2)), np.full((50_000, 1), 3.0)], axis=1)
    for k in (32, 7):
        h = knn_smoothing_lengths(pos, k)
        assert np.array_equal(bits(h), bits(scipy_h(pos, k))), kind


@pytest.mark.gpu
def test_knn_small_and_edge_cases(gpu):
    from asp_amd.knn import knn_smoothing_lengths
    rng = np.random.default_rng(4)
    for n in (1, 2, 31, 32, 33, 100):
        pos = rng.uniform(0, 1, (n, 3))
        for k in (1, 32, 64):
            h = knn_smoothing_lengths(pos, k)
            want = scipy_h(pos, k) if k <= n else np.full(n, np.inf)
            assert np.array_equal(bits(h), bits(want)), (n, k)
    assert knn_smoothing_lengths(np.zeros((0, 3))).shape == (0,)
    with pytest.raises(ValueError):
        knn_smoothing_lengths(np.zeros((4, 3)), 65)


@pytest.mark.gpu
def test_knn_device_tensor_and_large(gpu):
    """2e6 Plummer particles (dense core + sparse halo), device-resident input."""
    import torch
    from asp_amd.knn import knn_smoothing_lengths
    pos = _plummer(2_000_000, 6)
    h = knn_smoothing_lengths(torch.from_numpy(pos).cuda(), 32)
    assert h.is_cuda
    want = KDTree(pos).query(pos, k=32, workers=-1)[0][:, 31]
    assert np.array_equal(bits(h.cpu().numpy()), bits(want))


@pytest.mark.gpu
def test_knn_fp32_window_prefilter_far_coordinates(gpu, monkeypatch):
    """The window pass's fp32 prefilter (asp_knn.hip wave_scan32) takes coordinates
    relative to each wave's first particle; its bound grows with the largest such offset.
    Clusters far from the origin (|x| ~ 1e6, separations ~1e-3) and a few remote outliers
    (1e9) stress that bound: the result must stay bit-identical to scipy and to the fp64
    window (ASP_KNN_F32=0)."""
    from asp_amd.knn import knn_smoothing_lengths
    rng = np.random.default_rng(7)
    pos = np.concatenate([rng.uniform(0.0, 1.0, (40_000, 3)) + np.array([1e6, -2e6, 5e5]),
                          rng.standard_normal((20_000, 3)) * 1e-3 + np.array([1e6, -2e6, 5e5]),
                          rng.uniform(-1e9, 1e9, (50, 3))])
    rng.shuffle(pos)
    want = scipy_h(pos, 32)
    h32 = knn_smoothing_lengths(pos, 32)
    monkeypatch.setenv("ASP_KNN_F32", "0")
    h64 = knn_smoothing_lengths(pos, 32)
    assert np.array_equal(bits(h32), bits(want))
    assert np.array_equal(bits(h64), bits(want))


@pytest.mark.gpu
@pytest.mark.parametrize("uq,mask,near,fill", [("0", "0", "0", "1"), ("0", "1", "0", "1"),
                                               ("32", "1", "0", "1"), ("56", "1", "0", "1"),
                                               ("64", "1", "0", "1"), ("56", "0", "0", "1"),
                                               ("0", "0", "1", "1"), ("64", "1", "1", "0")])
def test_knn_shared_cell_pass(gpu, monkeypatch, uq, mask, near, fill):
    """The search's switches off their defaults (the defaults -- shared cell pass over all
    lanes, bit-mask entry test, nearest-chunks-first window -- run in every other test):
    the shared cell pass at other lane quantiles (ASP_KNN_UNION, 0 = the per-lane cell pass
    of round 5), the 8-slot entry buffer (ASP_KNN_MASK=0), the window in array order
    (ASP_KNN_NEAR=0): bit-exact against scipy on
    every input kind, the far-coordinate clusters and 2e6 Plummer particles; the lanes the
    shared pass leaves out (looser radii) keep their own pass."""
    from asp_amd.knn import knn_smoothing_lengths
    monkeypatch.setenv("ASP_KNN_UNION", uq)
    monkeypatch.setenv("ASP_KNN_MASK", mask)
    monkeypatch.setenv("ASP_KNN_NEAR", near)
    monkeypatch.setenv("ASP_KNN_FILL", fill)
    rng = np.random.default_rng(11)
    g = np.arange(30.0) * 0.5
    sets = [rng.uniform(0.0, 25.0, (60_000, 3)), _plummer(200_000, 5),
            np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3),
            np.concatenate([rng.uniform(0.0, 1.0, (2000, 3))] * 10 + [rng.uniform(0.0, 1.0, (4000, 3))]),
            np.concatenate([rng.uniform(0, 1, (30_000, 2)), np.full((30_000, 1), 3.0)], axis=1),
            np.concatenate([rng.uniform(0.0, 1.0, (20_000, 3)) + np.array([1e6, -2e6, 5e5]),
                            rng.uniform(-1e9, 1e9, (50, 3))])]
    for pos in sets:
        for k in (32, 7):
            assert np.array_equal(bits(knn_smoothing_lengths(pos, k)), bits(scipy_h(pos, k))), (len(pos), k)
    pos = _plummer(2_000_000, 6)
    want = KDTree(pos).query(pos, k=32, workers=-1)[0][:, 31]
    assert np.array_equal(bits(knn_smoothing_lengths(pos, 32)), bits(want))
