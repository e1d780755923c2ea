"""Lane utilisation of the cube wave path's plane walk: spheres of
radius r voxels clipped to a 16 x 16 x 32 brick, one lane per (i, j) column, 64 lanes per
pass; column order row-major (built), by distance from the axis, by length, and each lane
walking its columns back to back (the last three modelled only)."""
import numpy as np
rng = np.random.default_rng(1)
def columns(r):
    # sphere radius r voxels, center random in brick-ish coordinates; brick 16x16x32 at origin
    c = rng.uniform(-r, 16 + r, 2); cz = rng.uniform(-r, 32 + r)
    i0, i1 = max(0, int(np.ceil(c[0] - r))), min(15, int(np.floor(c[0] + r)))
    j0, j1 = max(0, int(np.ceil(c[1] - r))), min(15, int(np.floor(c[1] + r)))
    if i0 > i1 or j0 > j1: return None
    I, J = np.meshgrid(np.arange(i0, i1 + 1), np.arange(j0, j1 + 1), indexing="ij")
    rho2 = (I - c[0]) ** 2 + (J - c[1]) ** 2
    hz = np.sqrt(np.maximum(r * r - rho2, 0))
    a = np.maximum(np.ceil(cz - hz), 0); b = np.minimum(np.floor(cz + hz), 31)
    L = np.where((rho2 < r * r) & (b >= a), b - a + 1, 0)
    return L.ravel(), rho2.ravel()
def util(L, order):
    L = L[order]; steps = 0
    for p in range(0, len(L), 64):
        steps += np.ceil(L[p:p+64] / 2).max() if len(L[p:p+64]) else 0
    work = np.ceil(L / 2).sum()
    return work, steps * 64
for r in (4, 6, 8, 12):
    W = S1 = S2 = 0; S3 = 0
    for _ in range(3000):
        x = columns(r)
        if x is None: continue
        L, rho2 = x
        if len(L) <= 48: continue
        w, s1 = util(L, np.arange(len(L)))
        _, s2 = util(L, np.argsort(rho2, kind="stable"))
        _, s3 = util(L, np.argsort(-L, kind="stable"))
        W += w; S1 += s1; S2 += s2; S3 += s3
    print(f"r={r}: row-major util {W/S1:.2f}, by rho {W/S2:.2f}, by length {W/S3:.2f}")
print("flattened per-lane sums:")
for r in (4, 6, 8, 12):
    W = S = 0
    for _ in range(3000):
        x = columns(r)
        if x is None: continue
        L, rho2 = x
        if len(L) <= 48: continue
        P = np.ceil(L / 2)
        n = len(P); lanes = np.zeros(64)
        for t in range(n): lanes[t % 64] += P[t]
        W += P.sum(); S += lanes.max() * 64
    print(f"r={r}: util {W/S:.2f}")
