"""GPU: the §8(f) rows either side of the projection path (asp_stage.hip, through the C-ABI).

Bars: the periodic helpers and the fp64 -> fp32 staging are BIT-EXACT (the reference's
golden vectors G8; NumPy's astype(float32) via the oracle restatement); the staged
periodic images equal the restatement's as a set (the device appends them in an
unspecified order); periodic maps meet the projector's map bar (test_gpu_parity.py)
against the oracle run on the restated staged set.
"""
import numpy as np
import pytest

from conftest import golden
from test_gpu_parity import assert_map_close

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


@pytest.fixture(scope="module")
def g8():
    return golden("g8_periodic.npz")


@pytest.mark.parametrize("centred", [False, True])
def test_periodic_helpers_match_reference(gpu, g8, centred):
    from asp_amd.tools import calculate_periodic, make_periodic, shift_centre, shift_origin
    L, pos, c, k = float(g8["L"]), g8["pos"], g8["centre"], int(centred)
    assert np.array_equal(bits(calculate_periodic(pos, L, centred)), bits(g8[f"periodic_{k}"]))
    mp = pos.copy()
    assert make_periodic(mp, L, centred) is None
    assert np.array_equal(bits(mp), bits(g8[f"make_periodic_{k}"]))
    assert np.array_equal(bits(shift_origin(pos, c, L, centred)), bits(g8[f"shift_origin_{k}"]))
    assert np.array_equal(bits(shift_centre(pos, c, L, centred)), bits(g8[f"shift_centre_{k}"]))


def test_wrapped_displacement_distance_match_reference(gpu, g8):
    from asp_amd.tools import calculate_wrapped_displacement, calculate_wrapped_distance
    L = float(g8["L"])
    assert np.array_equal(bits(calculate_wrapped_displacement(g8["frm"], g8["to"], L)), bits(g8["disp"]))
    assert np.array_equal(bits(calculate_wrapped_displacement(g8["one"], g8["to"], L)),
                          bits(g8["disp_one"]))
    assert np.array_equal(bits(calculate_wrapped_distance(g8["frm"], g8["to"], L)), bits(g8["dist"]))
    assert np.array_equal(bits(calculate_wrapped_distance(g8["frm"], g8["to"], L, True)),
                          bits(g8["dist2"]))
    assert np.array_equal(bits(calculate_wrapped_distance(g8["one"], g8["to"], L)),
                          bits(g8["dist_one"]))
    d = calculate_wrapped_distance(g8["one"], g8["to"][0], L)
    assert isinstance(d, np.float64) and bits(d) == bits(g8["dist_vec"])


def test_periodic_helpers_device_tensors(gpu, g8):
    """float64 tensors on the GPU stay there, same bits."""
    import torch
    from asp_amd.tools import shift_centre
    L = float(g8["L"])
    t = torch.from_numpy(g8["pos"]).cuda()
    r = shift_centre(t, torch.from_numpy(g8["centre"]).cuda(), L)
    assert r.is_cuda and np.array_equal(bits(r.cpu().numpy()), bits(g8["shift_centre_0"]))


def _plummer(n, seed):
    from asp_amd.plummer import plummer
    p = plummer(n, seed=seed, h_law="knn32")
    return p["pos"], p["h"], p["m"], p["T"]


@pytest.mark.parametrize("axis", [0, 1, 2])
def test_stage_bitexact_host_and_device(gpu, oracle, axis):
    import torch
    from asp_amd.stage import stage_particles
    pos, h, m, T = _plummer(20000, 4)
    want = oracle.stage_particles(pos, h, [m, m * T], axis)
    u, v, hf, (a0, a1) = stage_particles(pos, h, m, m * T, projection_axis=axis)
    for g, w in zip((u, v, hf, a0, a1), want):
        assert g.dtype == torch.float32 and np.array_equal(g.cpu().numpy().view(np.uint32),
                                                           w.view(np.uint32))
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (pos, h, m)]
    u, v, hf, (a0,) = stage_particles(*dev, projection_axis=axis)
    for g, w in zip((u, v, hf, a0), want):
        assert np.array_equal(g.cpu().numpy().view(np.uint32), w.view(np.uint32))


def _as_set(cols):
    a = np.stack([c.view(np.uint32) for c in cols], axis=1)
    return a[np.lexsort(a.T[::-1])]


@pytest.mark.parametrize("shift,centred", [("centre", False), ("centre", True), ("wrap", False),
                                           ("origin", True)])
def test_stage_periodic_images(gpu, oracle, shift, centred):
    from asp_amd.stage import stage_particles
    rng = np.random.default_rng(9)
    L, n = 5.0, 30000
    pos = rng.uniform(-0.2 * L, 1.2 * L, (n, 3))
    h = rng.uniform(0.0, 0.08 * L, n)
    h[:50] = 0.0
    A = rng.uniform(0.5, 2.0, n)
    c = np.array([1.1, 3.3, 4.7])
    want = oracle.stage_particles(pos, h, [A], 2, L=L, centre=c, shift=shift, centred=centred,
                                  images=True)
    got = stage_particles(pos, h, A, projection_axis=2, box_width=L, centre=c, shift=shift,
                          origin_is_centre=centred, images=True)
    got = [got[0], got[1], got[2], got[3][0]]
    got = [t.cpu().numpy() for t in got]
    assert got[0].size == want[0].size > n
    for g, w in zip(got, want):  # originals, in order
        assert np.array_equal(g[:n].view(np.uint32), w[:n].view(np.uint32))
    assert np.array_equal(_as_set([g[n:] for g in got]), _as_set([w[n:] for w in want]))


def test_stage_chunked_host_path(gpu, oracle):
    """More particles than one host->device chunk (2^22): chunks on two streams, images
    claimed across chunks."""
    from asp_amd.stage import stage_particles
    rng = np.random.default_rng(12)
    n, L = 9_000_001, 1.0
    pos = rng.uniform(0.0, L, (n, 3))
    h = np.full(n, 2e-4)
    got = stage_particles(pos, h, projection_axis=1, box_width=L, shift="wrap", images=True)
    want = oracle.stage_particles(pos, h, [], 1, L=L, shift="wrap", images=True)
    got = [t.cpu().numpy() for t in got[:3]]
    for g, w in zip(got, want):
        assert np.array_equal(g[:n].view(np.uint32), w[:n].view(np.uint32))
    assert np.array_equal(_as_set([g[n:] for g in got]), _as_set([w[n:] for w in want]))


def test_periodic_map_matches_oracle_and_wraps(gpu, oracle):
    """create_periodic_image = the reference gather (oracle) over the restated staged set;
    a particle on a box face deposits on both sides."""
    from asp_amd.tools.projections import create_periodic_image
    rng = np.random.default_rng(3)
    L, n, G = 4.0, 6000, 96
    pos = rng.uniform(0.0, L, (n, 3))
    pos[0] = [0.01, 2.0, 2.0]          # hugs the x = 0 face
    h = rng.uniform(0.02, 0.12, n)
    h[0] = 0.1
    A = rng.uniform(0.5, 2.0, n)
    c = np.array([2.5, 1.0, 0.0])
    img = create_periodic_image(pos, h, A, (G, G), 16, 2, L, c)
    u, v, hh, a = oracle.stage_particles(pos, h, [A], 2, L=L, centre=c, shift="centre",
                                         images=True)
    st = np.stack([u, v, np.zeros_like(u)], axis=1).astype(np.float64)
    ref = oracle.create_image(st, hh.astype(np.float64), a.astype(np.float64), (G, G), 16, 2,
                              0.0, L, 0.0, L)
    assert_map_close(img, ref)
    one = create_periodic_image(pos[:1], h[:1], A[:1], (G, G), 16, 2, L)
    cols = np.nonzero(one.sum(axis=1))[0]
    assert cols.min() == 0 and cols.max() == G - 1  # both sides of the x faces


def test_periodic_map_translation_invariance(gpu):
    """Moving the centre by whole pixels rolls the periodic map (size-independent
    property; only fp32 rounding of the moved positions differs)."""
    from asp_amd.tools.projections import create_periodic_image
    rng = np.random.default_rng(5)
    L, n, G, k = 8.0, 40000, 128, 13
    pos = rng.uniform(0.0, L, (n, 3))
    h = rng.uniform(0.05, 0.3, n)
    A = rng.uniform(0.5, 2.0, n)
    c = np.array([4.0, 4.0, 4.0])
    m0 = create_periodic_image(pos, h, A, (G, G), 64, 2, L, c)
    m1 = create_periodic_image(pos, h, A, (G, G), 64, 2, L, c - np.array([k * L / G, 0.0, 0.0]))
    assert_map_close(np.roll(m0, k, axis=0), m1, abs_tol=1e-4, rel_tol=1e-3)


def test_stage_periodic_images_large_h(gpu, oracle):
    """Reach comparable to the box (2|h| up to 1.2 L): copies on both sides of an axis and
    several box widths over, as the oracle's restatement enumerates them; the periodic
    map then matches the oracle gather over that set.  Reach beyond 3 L is an error."""
    from asp_amd.stage import stage_particles
    from asp_amd.tools.projections import create_periodic_image
    rng = np.random.default_rng(19)
    L, n, G = 2.0, 3000, 48
    pos = rng.uniform(0.0, L, (n, 3))
    h = rng.uniform(0.01, 0.6 * L, n)
    A = rng.uniform(0.5, 2.0, n)
    want = oracle.stage_particles(pos, h, [A], 2, L=L, shift="wrap", images=True)
    got = stage_particles(pos, h, A, projection_axis=2, box_width=L, shift="wrap", images=True)
    got = [t.cpu().numpy() for t in (got[0], got[1], got[2], got[3][0])]
    assert got[0].size == want[0].size > 3 * n
    assert np.array_equal(_as_set([g[n:] for g in got]), _as_set([w[n:] for w in want]))
    img = create_periodic_image(pos, h, A, (G, G), 16, 2, L)
    st = np.stack([want[0], want[1], np.zeros_like(want[0])], axis=1).astype(np.float64)
    ref = oracle.create_image(st, want[2].astype(np.float64), want[3].astype(np.float64),
                              (G, G), 16, 2, 0.0, L, 0.0, L)
    assert_map_close(img, ref)
    h[0] = 2.0 * L  # 2|h| = 4 L
    with pytest.raises(NotImplementedError):
        stage_particles(pos, h, A, projection_axis=2, box_width=L, shift="wrap", images=True)


class _Unit:
    """Stand-in for a unyt Unit (unyt is not installed here): a name and a scale."""
    def __init__(self, name, scale):
        self.name, self.scale = name, scale

    def __pow__(self, k):
        return _Unit(f"{self.name}**{k}", self.scale ** k)

    def __eq__(self, other):
        return self.name == other.name


class _Q:
    """Stand-in for unyt_array: .value, .units, .to(units), ctor (values, units=...)."""
    def __init__(self, value, units):
        self.value, self.units = np.asarray(value, dtype=np.float64), units

    def to(self, units):
        return _Q(self.value * (self.units.scale / units.scale), units)


def test_periodic_helpers_unit_overloads(gpu, g8):
    """The reference's unyt overloads (_periodic_box_manipulations.py:49-51, :58-60,
    :70-72): operands converted to one unit (the positions' for calculate_periodic, the
    new origin's / centre's for the shifts), the NumPy body on the values, the result
    rewrapped in that unit.  Values must equal the plain call on the converted values."""
    from asp_amd.tools import (calculate_periodic, calculate_wrapped_distance, shift_centre,
                               shift_origin)
    kpc, Mpc = _Unit("kpc", 1.0), _Unit("Mpc", 1000.0)
    L, pos, c = float(g8["L"]), g8["pos"], g8["centre"]
    P = _Q(pos * 1000.0, kpc)           # positions in kpc
    C = _Q(c, Mpc)
    B = _Q(L, Mpc)
    r = calculate_periodic(P, B, False)
    assert isinstance(r, _Q) and r.units == kpc
    assert np.array_equal(bits(r.value), bits(calculate_periodic(P.value, L * 1000.0, False)))
    for f in (shift_origin, shift_centre):
        r = f(P, C, B, True)
        assert isinstance(r, _Q) and r.units == Mpc
        assert np.array_equal(bits(r.value), bits(f(P.to(Mpc).value, c, L, True)))
    d = calculate_wrapped_distance(_Q(c, Mpc), P, B, True)
    assert isinstance(d, _Q) and d.units == kpc ** 2
    assert np.array_equal(bits(d.value), bits(calculate_wrapped_distance(c * 1000.0, P.value,
                                                                         L * 1000.0, True)))
