"""CPU: the ionisation-table restatement (oracle/pyoracle.py: table_interp3) against the
reference's own class run here (golden G9, tests/golden/make_golden_table.py) and against
scipy's RegularGridInterpolator (the reference's dependency) on fresh seeded inputs.
Bar: bit-exact (same fp64 operation order), -inf fill and NaN propagation included."""
import numpy as np
import pytest

from conftest import golden


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


@pytest.fixture(scope="module")
def g9():
    return golden("g9_ion_table.npz")


def test_restatement_matches_reference_call(oracle, g9):
    grids = (g9["g0"], g9["g1"], g9["g2"])
    got = oracle.table_interp3(g9["table"], grids, g9["points3"])
    assert np.array_equal(bits(got), bits(g9["out3"]))


def test_restatement_matches_reference_at_redshift(oracle, g9):
    grids = (g9["g0"], g9["g1"], g9["g2"])
    for z, want in zip(g9["redshifts"], g9["out2"]):
        got = oracle.table_at_redshift(g9["table"], grids, g9["points2"], float(z))
        assert np.array_equal(bits(got), bits(want))


def test_restatement_matches_scipy_fresh(oracle):
    from scipy.interpolate import RegularGridInterpolator
    rng = np.random.default_rng(7)
    grids = [np.cumsum(rng.uniform(0.01, 1.0, n)) for n in (31, 17, 12)]
    table = rng.standard_normal((31, 17, 12))
    P = np.stack([rng.uniform(g[0] - 0.3, g[-1] + 0.3, 20000) for g in grids], axis=1)
    want = RegularGridInterpolator(grids, table, bounds_error=False, fill_value=-np.inf)(P)
    assert np.array_equal(bits(oracle.table_interp3(table, grids, P)), bits(want))
