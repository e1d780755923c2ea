"""Maps enqueued on two HIP streams (the library gives each stream its own workspace slot,
so map i + 1's binning overlaps map i's deposit): every map equals the one
a single stream produces -- int64 fixed-point maps bit-identical, neighbour counts exact --
for many alternating calls of different sizes (slot buffers grow independently), and the
slot workspaces are released by asp_release."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gate", ["0", "1"])
def test_two_stream_maps_equal_serial(gpu, oracle, gate, monkeypatch):
    # gate "1": each map's scatter waits for the previous map's deposit (ASP_SCATTER_GATE)
    monkeypatch.setenv("ASP_SCATTER_GATE", gate)
    import torch
    from asp_amd import _lib
    from asp_amd.device import project2d
    from asp_amd.plummer import plummer_torch
    dev = torch.device("cuda:0")
    G, ext = 512, (-4.0, 4.0, -4.0, 4.0)
    sets = []
    for n, seed, law in ((200_000, 1, "pixel"), (50_000, 2, "physical"), (400_000, 3, "pixel"),
                         (30_000, 4, "physical")):
        d = plummer_torch(n, seed=seed, h_law=law, extent=4.0, grid=G, device=dev)
        sets.append((d["x"], d["y"], d["h"], (d["m"] * d["T"]).contiguous(), d["m"]))
    kw = dict(image_size=(G, G), extent=ext, kernel="wendland_c2", deterministic=True)
    serial = [tuple(t.clone() for t in project2d(*s, **kw)) for s in sets]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    outs = [None] * 12
    for k in range(12):
        s = sets[k % len(sets)]
        with torch.cuda.stream(streams[k % 2]):
            outs[k] = project2d(*s, **kw)
    torch.cuda.synchronize()
    for k in range(12):
        want = serial[k % len(sets)]
        assert torch.equal(outs[k][0], want[0]) and torch.equal(outs[k][1], want[1]), k
    # counts on the second stream, exact against the oracle
    u, v, h, a0, a1 = sets[1]
    with torch.cuda.stream(streams[1]):
        cnt, _ = project2d(u, v, h, torch.ones_like(h), image_size=(G, G), extent=ext,
                           kernel="indicator")
    torch.cuda.synchronize()
    ref, _ = oracle.project_scatter(u.double().cpu().numpy(), v.double().cpu().numpy(),
                                    h.double().cpu().numpy(), np.ones(h.numel()), None, (G, G),
                                    64, *ext, kernel="indicator")
    assert np.array_equal(cnt.double().cpu().numpy(), ref)
    _lib.check(_lib.lib().asp_release(0))
    with torch.cuda.stream(streams[0]):
        again = project2d(*sets[0], **kw)
    torch.cuda.synchronize()
    assert torch.equal(again[0], serial[0][0])


def test_two_stream_cubes_equal_serial(gpu):
    """Cubes on two HIP streams (each its own workspace slot, round 5): every cube equals
    the one-stream cube -- voxel neighbour counts bit-exact, densities to fp32 rounding (fp64
    LDS atomics sum in any order) -- for alternating calls of different sizes."""
    import torch
    from asp_amd.device import project3d
    from asp_amd.plummer import plummer_torch
    dev = torch.device("cuda:0")
    C, ext = 128, (-4.0, 4.0) * 3
    sets = []
    for n, seed in ((200_000, 5), (60_000, 6), (300_000, 7)):
        d = plummer_torch(n, seed=seed, h_law="physical", extent=4.0, grid=C, device=dev)
        sets.append((d["x"], d["y"], d["z"], d["h"], d["m"]))
    kw = dict(cube_size=(C, C, C), extent=ext, kernel="wendland_c2")
    serial = [project3d(*s, **kw).clone() for s in sets]
    cnt = [project3d(*s[:4], torch.ones_like(s[3]), cube_size=(C, C, C), extent=ext,
                     kernel="indicator").clone() for s in sets]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    outs, couts = [None] * 6, [None] * 6
    for k in range(6):
        s = sets[k % len(sets)]
        with torch.cuda.stream(streams[k % 2]):
            outs[k] = project3d(*s, **kw)
            couts[k] = project3d(*s[:4], torch.ones_like(s[3]), cube_size=(C, C, C),
                                 extent=ext, kernel="indicator")
    torch.cuda.synchronize()
    for k in range(6):
        want = serial[k % len(sets)]
        assert torch.equal(couts[k], cnt[k % len(sets)]), k
        torch.testing.assert_close(outs[k], want, rtol=1e-6, atol=1e-6 * float(want.abs().max()))
