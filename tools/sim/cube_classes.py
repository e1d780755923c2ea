"""Lane-class model of the cube deposit's lane-per-record path (CPU, numpy; round 5).

Samples the cfg-5 particle set (10^8 Plummer, physical h, 512^3), forms every (particle,
brick) record of <= 48 columns with its per-column plane counts, and prices a wave of 64
records of one class as prep + sum over column steps (max over its lanes) of the column
set-up and the packed plane pairs.  Compares the box-volume classes (80 / 32 / 12) with
classes by column count; the deposit went 11.84 -> 11.07 ms on the GPU.
"""
import numpy as np, itertools
N_REAL, C, EXT, SAMPLE = 10**8, 512, 4.0, 150_000
rng = np.random.default_rng(1)
u = rng.uniform(0.0, 0.999, SAMPLE); ct = rng.uniform(-1, 1, SAMPLE); ph = rng.uniform(0, 2*np.pi, SAMPLE)
r = 1.0/np.sqrt(u**(-2/3)-1.0); st = np.sqrt(1-ct*ct)
x, y, z = r*st*np.cos(ph), r*st*np.sin(ph), r*ct
rho = 3/(4*np.pi)*(1+r*r)**-2.5
h = 1.2*np.cbrt((1.0/N_REAL)/rho)
pitch = 2*EXT/C; R = 2*h/pitch
cx, cy, cz = (x+EXT)/pitch, (y+EXT)/pitch, (z+EXT)/pitch
lo = lambda c: np.maximum(np.ceil(c-R), 0).astype(int)
hi = lambda c: np.minimum(np.floor(c+R), C-1).astype(int)
i0, i1, j0, j1, k0, k1 = lo(cx), hi(cx), lo(cy), hi(cy), lo(cz), hi(cz)
ok = (i0 <= i1) & (j0 <= j1) & (k0 <= k1)
recs = []
for p in np.nonzero(ok)[0]:
    for bi in range(i0[p]//16, i1[p]//16+1):
        for bj in range(j0[p]//16, j1[p]//16+1):
            a0, a1 = max(i0[p], bi*16), min(i1[p], bi*16+15)
            b0, b1 = max(j0[p], bj*16), min(j1[p], bj*16+15)
            ii, jj = np.meshgrid(np.arange(a0, a1+1), np.arange(b0, b1+1), indexing="ij")
            s = (ii-cx[p])**2 + (jj-cy[p])**2
            rz = np.sqrt(np.maximum(R[p]**2-s, 0.0))
            for bk in range(k0[p]//32, k1[p]//32+1):
                c0, c1 = max(k0[p], bk*32), min(k1[p], bk*32+31)
                la = np.maximum(np.ceil(cz[p]-rz), c0); lb = np.minimum(np.floor(cz[p]+rz), c1)
                ln = np.where((s < R[p]**2) & (la <= lb), lb-la+1, 0).ravel().astype(int)
                recs.append((ln, ii.size, c1-c0+1))
lane = [(g, nc, d) for g, nc, d in recs if nc <= 48]
print("lane records", len(lane), "wave records", len(recs)-len(lane))
PREP, SREJ, SACC, PAIR = 120, 12, 34, 15
def wave_cost(group):
    nc = max(len(g) for g in group); cost = PREP
    for c in range(nc):
        lens = [g[c] for g in group if c < len(g)]
        cost += SREJ + ((SACC-SREJ) if any(l > 0 for l in lens) else 0)
        cost += PAIR * max((l+1)//2 for l in lens)
    return cost
def total(keyfn):
    keys = np.array([keyfn(nc, d) for _, nc, d in lane])
    tot = 0
    for kv in np.unique(keys):
        idx = np.nonzero(keys == kv)[0]; rng.shuffle(idx)
        n = idx.size
        for w0 in range(0, n, 64):
            tot += wave_cost([lane[i][0] for i in idx[w0:w0+64]])
    return tot
vol = lambda nc, d: nc*d
base = total(lambda nc, d: np.digitize(nc*d, [12, 32, 80]))
print("current (vol 12/32/80)", base)
for name, fn in [("none", lambda nc, d: 0),
                 ("cols 8/16/30", lambda nc, d: np.digitize(nc, [8, 16, 30])),
                 ("cols 6/12/20/30/40", lambda nc, d: np.digitize(nc, [6, 12, 20, 30, 40])),
                 ("vol 8 classes", lambda nc, d: np.digitize(nc*d, [8, 16, 24, 32, 48, 80, 120])),
                 ("cols x depth", lambda nc, d: np.digitize(nc, [9, 20, 36])*4 + np.digitize(d, [3, 5, 8])),
                 ("cols 12 classes", lambda nc, d: np.digitize(nc, [4, 6, 9, 12, 16, 20, 25, 30, 36, 42, 48]))]:
    t = total(fn); print(f"{name:22s} {t} ({base/t:.3f}x)")
