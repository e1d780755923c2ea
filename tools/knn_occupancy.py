"""Morton-cell occupancy of a Plummer set on the k-NN search's grid.

For each level L: the occupied cells and, for a typical PARTICLE, how many particles share
its level-L cell (the length of the binary search a lookup inside that cell costs).  The
grid is the search's: 2^21 quanta per axis over the bounding cube."""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "astro-sph-tools_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    a = ap.parse_args()
    from asp_amd.plummer import plummer_torch
    d = plummer_torch(a.n, seed=0, h_law="pixel", extent=4.0, grid=64, device="cpu")
    pos = np.stack([d[c].double().numpy() for c in "xyz"], 1)
    lo = pos.min(0)
    span = (pos.max(0) - lo).max()
    print(f"bounding cube edge {span:.2f}")
    q = np.floor((pos - lo) * (2 ** 21 / (span * (1 + 2 ** -20)))).astype(np.int64)
    for L in range(8, 13):
        c = q >> (21 - L)
        key = (c[:, 0] << (2 * L)) | (c[:, 1] << L) | c[:, 2]
        _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        per = cnt[inv]
        print(f"L={L}: occupied {cnt.size}, per-particle cell occupancy median {np.median(per):.0f} "
              f"mean {per.mean():.0f} p90 {np.percentile(per, 90):.0f} max {cnt.max()}")


if __name__ == "__main__":
    main()
