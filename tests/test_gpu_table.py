"""GPU: ionisation-table interpolation (asp_table.hip, asp_table_interp3, through the C-ABI)
and the ion column map it feeds.

Bars: table values BIT-EXACT against the reference's own class run here (golden G9) and
against the oracle restatement / scipy RegularGridInterpolator on fresh inputs (-inf fill
outside the table, NaN for NaN input); ion masses m * X * 10^f within 2 ulp-scale
(rtol 4.5e-16 -- the device pow is not correctly rounded, NumPy's may differ by one ulp);
the ion column map meets the projector's map bar (test_gpu_parity.py) against the oracle
fed NumPy ion masses.
"""
import numpy as np
import pytest

from conftest import golden
from test_gpu_parity import assert_map_close

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


@pytest.fixture(scope="module")
def g9():
    return golden("g9_ion_table.npz")


@pytest.fixture(scope="module")
def table(gpu, g9):
    from asp_amd.ionisation import IonisationTable
    return IonisationTable(g9["table"], g9["g0"], g9["g1"], g9["g2"], redshift_input_index=2)


def test_g9_call_bit_exact(table, g9):
    assert np.array_equal(bits(table(g9["points3"])), bits(g9["out3"]))


def test_g9_at_redshift_bit_exact(table, g9):
    for z, want in zip(g9["redshifts"], g9["out2"]):
        assert np.array_equal(bits(table.evaluate_at_redshift(g9["points2"], float(z))), bits(want))


def test_table_accessors(table, g9):
    assert table.number_of_input_dimensions == 3
    assert np.array_equal(table.ionisation_fraction_table, g9["table"])
    assert np.array_equal(table.get_table_dimension(1), g9["g1"])


def test_large_fresh_bit_exact_device_tensors(gpu, oracle):
    """10^6 points on an HM01-sized table (e.g. 41 x 141 x 49), device tensors in and out."""
    import torch
    from asp_amd.ionisation import IonisationTable
    rng = np.random.default_rng(11)
    shape = (41, 141, 49)
    grids = [np.cumsum(rng.uniform(0.05, 0.2, n)) - 3.0 for n in shape]
    t = rng.uniform(-10.0, 0.0, shape)
    P = np.stack([rng.uniform(g[0] - 0.1, g[-1] + 0.1, 10 ** 6) for g in grids], axis=1)
    P[::997, 1] = np.nan
    tab = IonisationTable(t, *grids, redshift_input_index=2)
    got = tab(torch.from_numpy(P).cuda())
    assert got.is_cuda and got.dtype == torch.float64
    assert np.array_equal(bits(got.cpu().numpy()), bits(oracle.table_interp3(t, grids, P)))


def test_empty_and_errors(table):
    assert table(np.empty((0, 3))).shape == (0,)
    with pytest.raises(ValueError):
        table(np.zeros((4, 2)))
    from asp_amd.ionisation import IonisationTable
    with pytest.raises(IndexError):
        IonisationTable(np.zeros((2, 2, 2)), np.arange(2.0), np.arange(2.0))


def test_ion_masses_and_column_map(gpu, oracle, table, g9):
    from asp_amd.ionisation import ion_masses
    from asp_amd.tools.projections import create_image
    rng = np.random.default_rng(5)
    n = 20000
    pos = rng.uniform(0.0, 1.0, (n, 3))
    h = rng.uniform(0.005, 0.03, n)
    m = rng.uniform(0.5, 1.5, n)
    X = rng.uniform(0.6, 0.8, n)
    g0, g1 = g9["g0"], g9["g1"]
    nH = rng.uniform(g0[0], g0[-1], n)
    T = rng.uniform(g1[0], g1[-1], n)
    z = 2.25
    got = ion_masses(table, m, X, nH, T, z, table_is_log10=True)
    f = oracle.table_at_redshift(g9["table"], (g0, g9["g1"], g9["g2"]), np.stack([nH, T], 1), z)
    want = (m * X) * 10.0 ** f
    np.testing.assert_allclose(got, want, rtol=4.5e-16, atol=0)
    lin = ion_masses(table, m, X, nH, T, z, table_is_log10=False)
    assert np.array_equal(bits(lin), bits((m * X) * f))
    img = create_image(pos, h, got, (128, 128), 32, 2, 0.0, 1.0, 0.0, 1.0)
    ref = oracle.create_image(pos, h, want, (128, 128), 32, 2, 0.0, 1.0, 0.0, 1.0)
    assert_map_close(img, ref)


@pytest.mark.parametrize("zaxis", [0, 1, 2])
def test_at_redshift_any_axis_matches_restatement(gpu, oracle, zaxis):
    """The fixed axis anywhere (axis 2 goes through the LDS slab kernel, 0 / 1 through the
    global one), on a random table, random states and an HM01-sized slab."""
    from asp_amd.ionisation import IonisationTable
    rng = np.random.default_rng(100 + zaxis)
    shape = (41, 141, 49)
    grids = [np.cumsum(rng.uniform(0.05, 0.2, k)) for k in shape]
    t = rng.uniform(-10.0, 0.0, shape)
    tab = IonisationTable(t, *grids, redshift_input_index=zaxis)
    free = [d for d in range(3) if d != zaxis]
    P = np.stack([rng.uniform(grids[d][0] - 0.1, grids[d][-1] + 0.1, 300000) for d in free], 1)
    for z in (grids[zaxis][7], 0.5 * (grids[zaxis][3] + grids[zaxis][4]), grids[zaxis][-1],
              grids[zaxis][-1] + 1.0, np.nan):
        got = tab.evaluate_at_redshift(P, float(z))
        want = oracle.table_at_redshift(t, grids, P, float(z), zaxis=zaxis)
        assert np.array_equal(bits(got), bits(want)), (zaxis, z)


@pytest.mark.parametrize("ndim", [1, 2, 4, 5])
def test_nd_tables_bit_exact_vs_scipy(gpu, ndim):
    """IonisationTableBase takes any number of axes (_IonisationTable.py:31-49): 1, 2, 4 and
    5-D tables against scipy's RegularGridInterpolator (the reference's interpolator,
    linear, fill -inf), __call__ and evaluate_at_redshift, including points outside the
    table and NaN rows.  2-D also read-only (scipy's _evaluate_linear instead of its Cython
    fast path: a different arithmetic order, both reproduced)."""
    from scipy.interpolate import RegularGridInterpolator
    from asp_amd.ionisation import IonisationTable
    rng = np.random.default_rng(100 + ndim)
    shape = tuple(int(x) for x in rng.integers(3, 12 if ndim <= 2 else 7, ndim))
    grids = [np.cumsum(rng.uniform(0.05, 0.3, n)) - 1.0 for n in shape]
    t = rng.normal(size=shape)
    variants = [t]
    if ndim == 2:
        ro = t.copy()
        ro.flags.writeable = False
        variants.append(ro)
    P = np.stack([rng.uniform(g[0] - 0.1, g[-1] + 0.1, 50_000) for g in grids], axis=1)
    P[::331, 0] = np.nan
    for tab_arr in variants:
        ref = RegularGridInterpolator(grids, tab_arr, bounds_error=False, fill_value=-np.inf)
        tab = IonisationTable(tab_arr, *grids, redshift_input_index=ndim - 1)
        assert tab.number_of_input_dimensions == ndim
        assert np.array_equal(bits(tab(P)), bits(ref(P)))
        if ndim >= 2:
            z = float(grids[-1][1] + 0.37 * (grids[-1][2] - grids[-1][1]))
            full = np.concatenate([P[:, :-1], np.full((P.shape[0], 1), z)], axis=1)
            assert np.array_equal(bits(tab.evaluate_at_redshift(P[:, :-1], z)), bits(ref(full)))
