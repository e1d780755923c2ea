"""Wave-path model of the cube deposit (CPU, numpy): for the boxes of more than 40 columns,
wave time = sum over passes of the max lane cost, a lane's cost for a column (or a column
chunk) = set-up + packed plane pairs.  Compares the column-per-lane walk with columns split
into plane chunks of P planes (chunk-major or column-major item order)."""
import numpy as np

N_REAL, C, EXT, SAMPLE, LANE_COLS = 10**8, 512, 4.0, 60_000, 40
SETUP, MISS = 1.5, 1.0
rng = np.random.default_rng(2)
u = rng.uniform(0.0, 0.999, SAMPLE)
ct = rng.uniform(-1, 1, SAMPLE)
ph = rng.uniform(0, 2 * np.pi, SAMPLE)
r = 1.0 / np.sqrt(u ** (-2 / 3) - 1.0)
st = np.sqrt(1 - ct * ct)
x, y, z = r * st * np.cos(ph), r * st * np.sin(ph), r * ct
rho = 3 / (4 * np.pi) * (1 + r * r) ** -2.5
h = 1.2 * np.cbrt((1.0 / N_REAL) / rho)
pitch = 2 * EXT / C
R = 2 * h / pitch
cx, cy, cz = (x + EXT) / pitch, (y + EXT) / pitch, (z + EXT) / pitch
lo = lambda c: np.maximum(np.ceil(c - R), 0).astype(int)
hi = lambda c: np.minimum(np.floor(c + R), C - 1).astype(int)
i0, i1, j0, j1, k0, k1 = lo(cx), hi(cx), lo(cy), hi(cy), lo(cz), hi(cz)
ok = (i0 <= i1) & (j0 <= j1) & (k0 <= k1) & ((i1 - i0 + 1) * (j1 - j0 + 1) > LANE_COLS)
def passes(costs):
    n = -(-costs.size // 64) * 64
    c = np.zeros(n); c[:costs.size] = costs
    return c.reshape(-1, 64).max(axis=1).sum()
tot = {"columns": 0.0}
for P in (4, 8, 12):
    tot[f"P{P} chunk-major"] = 0.0
    tot[f"P{P} column-major"] = 0.0
for p in np.nonzero(ok)[0]:
    for bi in range(i0[p] // 16, i1[p] // 16 + 1):
        for bj in range(j0[p] // 16, j1[p] // 16 + 1):
            a0, a1 = max(i0[p], bi * 16), min(i1[p], bi * 16 + 15)
            b0, b1 = max(j0[p], bj * 16), min(j1[p], bj * 16 + 15)
            if (a1 - a0 + 1) * (b1 - b0 + 1) <= LANE_COLS:
                continue
            ii, jj = np.meshgrid(np.arange(a0, a1 + 1), np.arange(b0, b1 + 1), indexing="ij")
            s = ((ii - cx[p]) ** 2 + (jj - cy[p]) ** 2).ravel()
            rz = np.sqrt(np.maximum(R[p] ** 2 - s, 0.0))
            for bk in range(k0[p] // 32, k1[p] // 32 + 1):
                c0, c1 = max(k0[p], bk * 32), min(k1[p], bk * 32 + 31)
                la = np.maximum(np.ceil(cz[p] - rz), c0)
                lb = np.minimum(np.floor(cz[p] + rz), c1)
                hit = (s < R[p] ** 2) & (la <= lb)
                ln = np.where(hit, lb - la + 1, 0)
                tot["columns"] += passes(np.where(hit, SETUP + np.ceil(ln / 2), MISS))
                depth = c1 - c0 + 1
                for P in (4, 8, 12):
                    nch = -(-depth // P)
                    st_ = c0 + P * np.arange(nch)
                    ca = np.maximum(la[:, None], st_[None, :])
                    cb = np.minimum(lb[:, None], st_[None, :] + P - 1)
                    cl = np.where(hit[:, None] & (ca <= cb), cb - ca + 1, 0)
                    cost = np.where(cl > 0, SETUP + np.ceil(cl / 2), MISS)
                    tot[f"P{P} column-major"] += passes(cost.ravel())
                    tot[f"P{P} chunk-major"] += passes(cost.T.ravel())
base = tot["columns"]
for k, v in tot.items():
    print(f"{k:18s} {v:12.0f}  {base / v:5.2f}x")
