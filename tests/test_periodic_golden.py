"""CPU: the oracle's restatement of the reference's periodic-box helpers
(oracle/pyoracle.py pb_*) against the golden vectors G8, made by running the reference's
own function bodies (tests/golden/make_golden_periodic.py).  Bit-exact, sign of zero
included -- the restatement is what tests/test_gpu_stage.py checks the device against."""
import numpy as np
import pytest

from conftest import golden


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


@pytest.fixture(scope="module")
def g8():
    return golden("g8_periodic.npz")


@pytest.mark.parametrize("centred", [0, 1])
def test_wrap_and_shifts_match_reference(oracle, g8, centred):
    L, pos, c = float(g8["L"]), g8["pos"], g8["centre"]
    assert np.array_equal(bits(oracle.pb_wrap(pos, L, centred)), bits(g8[f"periodic_{centred}"]))
    assert np.array_equal(bits(g8[f"make_periodic_{centred}"]), bits(g8[f"periodic_{centred}"]))
    assert np.array_equal(bits(oracle.pb_shift(pos, c, L, "origin", centred)),
                          bits(g8[f"shift_origin_{centred}"]))
    assert np.array_equal(bits(oracle.pb_shift(pos, c, L, "centre", centred)),
                          bits(g8[f"shift_centre_{centred}"]))


def test_displacement_and_distance_match_reference(oracle, g8):
    L = float(g8["L"])
    assert np.array_equal(bits(oracle.pb_displacement(g8["frm"], g8["to"], L)), bits(g8["disp"]))
    assert np.array_equal(bits(oracle.pb_displacement(g8["one"], g8["to"], L)), bits(g8["disp_one"]))
    assert np.array_equal(bits(oracle.pb_distance(g8["frm"], g8["to"], L)), bits(g8["dist"]))
    assert np.array_equal(bits(oracle.pb_distance(g8["frm"], g8["to"], L, True)), bits(g8["dist2"]))
    assert np.array_equal(bits(oracle.pb_distance(g8["one"], g8["to"], L)), bits(g8["dist_one"]))
    assert bits(oracle.pb_distance(g8["one"], g8["to"][0], L)) == bits(g8["dist_vec"])


def test_reference_wraps_once(g8):
    """The reference wraps by ONE box width: coordinates more than a box out stay out."""
    L = float(g8["L"])
    p = g8["periodic_0"]
    assert (p >= 0).mean() < 1.0 and np.all(p < 2 * L) and np.all(p >= -L)


def test_staging_images_restatement(oracle):
    """Periodic images: a particle inside the box within reach 2|h| of a face gets one copy
    per crossed face (and the corner copy); none far from the faces or with h = 0."""
    L = 10.0
    pos = np.array([[0.5, 5.0, 1.0], [9.7, 9.8, 1.0], [5.0, 5.0, 1.0], [0.1, 0.1, 0.0],
                    [12.0, 5.0, 0.0]])
    h = np.array([0.3, 0.2, 0.3, 0.0, 0.3])
    u, v, hh, a = oracle.stage_particles(pos, h, [np.arange(5.0)], 2, L=L, shift=None,
                                         images=True)
    assert u.size == 5 + 1 + 3          # particle 0: one copy; particle 1: x, y and corner
    got = sorted(zip(u[5:].tolist(), v[5:].tolist(), a[5:].tolist()))
    want = sorted([(10.5, 5.0, 0.0), (np.float32(9.7) - 10.0, 9.8, 1.0),
                   (9.7, np.float32(9.8) - 10.0, 1.0),
                   (np.float32(9.7) - 10.0, np.float32(9.8) - 10.0, 1.0)])
    np.testing.assert_allclose(np.array(got), np.array(want), rtol=0, atol=1e-5)
