"""Lane-utilisation model of the cube deposit's lane-per-record path (CPU, numpy).

Samples the cfg-5 particle set (10^8 Plummer, physical h, 512^3 over [-4, 4]^3), forms the
(particle, brick) records the scatter makes, and for records of <= LANE_COLS columns
(the lane path) models a wave's time as the max over its 64 lanes of
sum_columns(setup + ceil(len / 2)) (the column set-up and the packed plane pairs), for
records in arrival order and with records split into size classes.
"""
import numpy as np

N_REAL, C, EXT, SAMPLE, LANE_COLS = 10**8, 512, 4.0, 200_000, 30
SETUP = 6.0  # cost of a column's set-up in units of one plane-pair iteration (estimate)
rng = np.random.default_rng(1)
u = rng.uniform(0.0, 0.999, SAMPLE)
ct = rng.uniform(-1, 1, SAMPLE)
ph = rng.uniform(0, 2 * np.pi, SAMPLE)
r = 1.0 / np.sqrt(u ** (-2 / 3) - 1.0)
st = np.sqrt(1 - ct * ct)
x, y, z = r * st * np.cos(ph), r * st * np.sin(ph), r * ct
rho = 3 / (4 * np.pi) * (1 + r * r) ** -2.5
h = 1.2 * np.cbrt((1.0 / N_REAL) / rho)
pitch = 2 * EXT / C
R = 2 * h / pitch                      # support radius in voxels
cx, cy, cz = (x + EXT) / pitch, (y + EXT) / pitch, (z + EXT) / pitch  # voxel-corner frame
lo = lambda c: np.maximum(np.ceil(c - R), 0).astype(int)
hi = lambda c: np.minimum(np.floor(c + R), C - 1).astype(int)
i0, i1, j0, j1, k0, k1 = lo(cx), hi(cx), lo(cy), hi(cy), lo(cz), hi(cz)
ok = (i0 <= i1) & (j0 <= j1) & (k0 <= k1)
recs = []  # (work, ncols) per (particle, brick) record of the lane path
wave_work = 0.0
for p in np.nonzero(ok)[0]:
    for bi in range(i0[p] // 16, i1[p] // 16 + 1):
        for bj in range(j0[p] // 16, j1[p] // 16 + 1):
            a0, a1 = max(i0[p], bi * 16), min(i1[p], bi * 16 + 15)
            b0, b1 = max(j0[p], bj * 16), min(j1[p], bj * 16 + 15)
            ii, jj = np.meshgrid(np.arange(a0, a1 + 1), np.arange(b0, b1 + 1), indexing="ij")
            s = (ii - cx[p]) ** 2 + (jj - cy[p]) ** 2
            rz = np.sqrt(np.maximum(R[p] ** 2 - s, 0.0))
            for bk in range(k0[p] // 32, k1[p] // 32 + 1):
                c0, c1 = max(k0[p], bk * 32), min(k1[p], bk * 32 + 31)
                la = np.maximum(np.ceil(cz[p] - rz), c0)
                lb = np.minimum(np.floor(cz[p] + rz), c1)
                ln = np.where((s < R[p] ** 2) & (la <= lb), lb - la + 1, 0)
                cols = ii.size
                work = (SETUP * (ln > 0) + np.ceil(ln / 2)).sum() + 1.0 * (ln == 0).sum()
                if cols <= LANE_COLS:
                    recs.append((work, cols * (c1 - c0 + 1)))
                else:
                    wave_work += work
w = np.array([a for a, _ in recs])
vol = np.array([b for _, b in recs])
perm = rng.permutation(w.size); w = w[perm]; vol = vol[perm]
def waves(ws):
    n = ws.size // 64 * 64
    return ws[:n].reshape(-1, 64).max(axis=1).sum()
base = waves(w)
print(f"lane-path records {w.size}, mean work {w.mean():.2f}, ideal {w.sum() / 64:.0f}, "
      f"random order {base:.0f} (utilisation {w.sum() / 64 / base:.2f})")
for edges in ([8, 27, 64], [4, 12, 36, 100], [6, 18, 48, 120], [12, 48]):
    cls = np.digitize(vol, edges)
    tot = sum(waves(w[cls == c]) for c in np.unique(cls))
    print(f"classes split at box volume {edges}: {tot:.0f} ({base / tot:.2f}x)")
print(f"wave-path work (lane-serial units) {wave_work:.0f} vs lane path {w.sum():.0f}")
