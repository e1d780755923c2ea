"""CPU model of the k-NN shared cell pass (asp_knn.hip k_knn_wave, ASP_KNN_UNION): per
wave of 64 Morton-consecutive particles, the entries the shared pass streams against the
cell-scan distances the per-lane pass evaluates.  Plummer sphere, k = 32, W = 64.

    python tools/sim/knn_union.py [n] [uq ...]
"""
import sys

import numpy as np

sys.path.insert(0, "astro-sph-tools_amd")


def spread(v):
    v = v.astype(np.uint64) & np.uint64(0x1fffff)
    for sh, m in ((32, 0x1f00000000ffff), (16, 0x1f0000ff0000ff), (8, 0x100f00f00f00f00f),
                  (4, 0x10c30c30c30c30c3), (2, 0x1249249249249249)):
        v = (v | (v << np.uint64(sh))) & np.uint64(m)
    return v


def main():
    from asp_amd.plummer import plummer
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
    uqs = [int(a) for a in sys.argv[2:]] or [64, 56, 48, 32]
    k, W, fine = 32, 64, 1
    pos = plummer(n, seed=0, h_law="pixel", grid=64)["pos"]
    lo = pos.min(0)
    span = (pos.max(0) - lo).max()
    scale = 2.0 ** 21 / (span * (1 + 2.0 ** -20))
    q = np.clip(np.floor((pos - lo) * scale), 0, 2 ** 21 - 1).astype(np.int64)
    key = (spread(q[:, 0]) << np.uint64(2)) | (spread(q[:, 1]) << np.uint64(1)) | spread(q[:, 2])
    o = np.argsort(key, kind="stable")
    key, pos, q = key[o], pos[o], q[o]
    rng = np.random.default_rng(0)
    waves = rng.choice(n // 64, size=min(2000, n // 64), replace=False)
    res = {u: [] for u in uqs}
    lane_cells = []
    for wv in waves:
        b = wv * 64
        w0, w1 = max(0, b - W), min(n, b + 64 + W)
        P = pos[b:b + 64]
        d2 = ((P[:, None, :] - pos[None, w0:w1, :]) ** 2).sum(-1)
        mx = np.sort(d2, axis=1)[:, k - 1]
        R = np.sqrt(mx) * (1 + 2.0 ** -40)
        e = np.frexp(R * scale + 1.0)[1]
        sft = np.maximum(0, np.minimum(e, 21) - fine)
        klo = 0 if w0 == 0 else int(key[w0]) + 1
        khi = 2 ** 64 - 1 if w1 == n else int(key[w1 - 1])
        for u in uqs:
            need = (64 * u + 63) >> 6
            s = int(np.sort(sft)[need - 1])
            rg = sft <= s
            qa = np.maximum(0, np.floor((P[rg] - R[rg, None] - lo) * scale) - 1).astype(np.int64) >> s
            qb = np.minimum(2 ** 21 - 1, np.floor((P[rg] + R[rg, None] - lo) * scale) + 1).astype(np.int64) >> s
            A, B = qa.min(0), qb.max(0)
            g = [np.arange(A[a], B[a] + 1) for a in range(3)]
            C = np.stack(np.meshgrid(*g, indexing="ij"), -1).reshape(-1, 3)
            clo = lo + (C << s) / scale - 1 / scale
            chi = lo + ((C + 1) << s) / scale + 1 / scale
            gap = np.maximum(0, np.maximum(clo[None] - P[rg, None], P[rg, None] - chi[None]))
            md = (gap ** 2).sum(-1)
            need_c = (md * (1 - 2.0 ** -40) <= mx[rg, None]).any(0)
            C = C[need_c]
            k0 = ((spread(C[:, 0]) << np.uint64(2)) | (spread(C[:, 1]) << np.uint64(1)) | spread(C[:, 2])) << np.uint64(3 * s)
            k1 = k0 + np.uint64(1 << (3 * s))
            inside = (k0 >= np.uint64(klo)) & (k1 <= np.uint64(khi))
            j0 = np.searchsorted(key, k0[~inside])
            j1 = np.searchsorted(key, k1[~inside])
            res[u].append((len(C), int(inside.sum()), int((j1 - j0).sum()), int((~rg).sum()), int(np.prod(B - A + 1))))
    for u in uqs:
        a = np.array(res[u])
        print(f"uq {u}: cells listed {a[:, 0].mean() - a[:, 1].mean():.0f} (+{a[:, 1].mean():.0f} inside "
              f"the window), entries streamed per wave {a[:, 2].mean():.0f} (p90 {np.percentile(a[:, 2], 90):.0f},"
              f" max {a[:, 2].max()}), lanes left to their own pass {a[:, 3].mean():.1f}, box cells tested {np.median(a[:, 4]):.0f} (mean {a[:, 4].mean():.0f})")


if __name__ == "__main__":
    main()
