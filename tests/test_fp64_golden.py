"""G10 (raw float64 inputs, every axis spelling) on the CPU: the oracle restatement and
the host-side axis resolution against the reference's own outputs
(tests/golden/make_golden_f64.py ran the reference).  Bit-exact: the oracle repeats the
reference's fp64 operation order and NumPy's pairwise sum."""
import numpy as np
import pytest

from conftest import golden


@pytest.fixture(scope="module")
def g10():
    return golden("g10_fp64_axes.npz")


def test_inputs_are_not_float32_representable(g10):
    for k in ("plummer_pos", "plummer_h", "axes_pos"):
        a = g10[k]
        assert not np.any(a.astype(np.float32).astype(np.float64) == a)
    assert int(g10["edge_f32_flips"]) > 1000  # float32 rounding would flip these pairs


def test_oracle_plummer_raw_fp64(g10, oracle):
    pos, h, A = g10["plummer_pos"], g10["plummer_h"], g10["plummer_A"]
    size, cs, ext = tuple(g10["plummer_size"]), int(g10["plummer_cs"]), tuple(g10["plummer_ext"])
    assert np.array_equal(oracle.create_image(pos, h, A, size, cs, 2, *ext), g10["plummer_img"])
    n = h.size
    assert np.array_equal(oracle.create_image(pos, h, np.ones(n), size, cs, 2, *ext,
                                              kernel="indicator"), g10["plummer_cnt"])
    ids = (np.arange(n) % 4093).astype(np.float64)
    assert np.array_equal(oracle.create_image(pos, h, ids, size, cs, 2, *ext, kernel="indicator"),
                          g10["plummer_ids"])


def test_oracle_edge_pairs(g10, oracle):
    pos, h = g10["edge_pos"], g10["edge_h"]
    size, cs, ext = tuple(g10["edge_size"]), int(g10["edge_cs"]), tuple(g10["edge_ext"])
    n = h.size
    assert np.array_equal(oracle.create_image(pos, h, np.ones(n), size, cs, 2, *ext,
                                              kernel="indicator"), g10["edge_cnt"])
    ids = (np.arange(n) % 4093).astype(np.float64)
    assert np.array_equal(oracle.create_image(pos, h, ids, size, cs, 2, *ext, kernel="indicator"),
                          g10["edge_ids"])
    # the scatter restatement decides the same pairs
    cnt, _ = oracle.project_scatter(pos[:, 0], pos[:, 1], h, np.ones(n), None, size, cs, *ext,
                                    kernel="indicator")
    assert np.array_equal(cnt, g10["edge_cnt"])


def _spelling(key):
    from asp_amd import CoordinateAxes
    return {"enumX": CoordinateAxes.X, "enumY": CoordinateAxes.Y, "enumZ": CoordinateAxes.Z,
            "strx": "x", "stry": "y", "strz": "z", "strX": "X", "int0": 0, "int1": 1,
            "bytesx": b"x"}[key]


def test_reference_axes_resolution():
    from asp_amd import CoordinateAxes
    from asp_amd._axes import reference_axes
    assert reference_axes(CoordinateAxes.X) == (0, 0)
    assert reference_axes(CoordinateAxes.Y) == (1, 1)
    assert reference_axes(CoordinateAxes.Z) == (2, 2)
    assert reference_axes("x") == (0, 2) and reference_axes("y") == (1, 2)
    assert reference_axes("X") == (2, 2) and reference_axes(" x") == (2, 2)
    assert reference_axes(0) == (2, 2) and reference_axes(1) == (2, 2)
    assert reference_axes(b"x") == (2, 2)


def test_oracle_axes_spellings(g10, oracle):
    """Mixed cull / pixel columns (str "x"), ints and bytes as the reference handles them,
    resolved by reference_axes and restated by the oracle: bit-exact."""
    from asp_amd._axes import reference_axes
    pos, h, A = g10["axes_pos"], g10["axes_h"], g10["axes_A"]
    size, cs, ext = tuple(g10["axes_size"]), int(g10["axes_cs"]), tuple(g10["axes_ext"])
    for key in g10["axes_keys"]:
        ax = reference_axes(_spelling(str(key)))
        assert np.array_equal(oracle.create_image(pos, h, A, size, cs, ax, *ext),
                              g10[f"axes_img_{key}"]), key
        assert np.array_equal(oracle.create_image(pos, h, np.ones(h.size), size, cs, ax, *ext,
                                                  kernel="indicator"), g10[f"axes_cnt_{key}"]), key
    # the spellings really differ: "x" (mixed) is neither the X nor the Z map
    assert not np.array_equal(g10["axes_img_strx"], g10["axes_img_enumX"])
    assert not np.array_equal(g10["axes_img_strx"], g10["axes_img_enumZ"])
    assert np.array_equal(g10["axes_img_int0"], g10["axes_img_enumZ"])
