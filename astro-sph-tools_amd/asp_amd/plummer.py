"""Synthetic Plummer-sphere particle sets.

The reference ships no data generator; this is the build's synthetic workload.
Laws (a = 1, M = 1, seed-deterministic via numpy PCG64 ``default_rng``):

* radius        r = a (u^(-2/3) - 1)^(-1/2),  u ~ U(0, 0.999)
* direction     cos(theta) ~ U(-1, 1), phi ~ U(0, 2 pi)  (isotropic)
* density       rho = 3/(4 pi) (1 + r^2)^(-5/2)           (analytic)
* mass          m = 1/N
* temperature   T = 1e4 K (1 + r^2)^(-1/2)
* smoothing length, one of
    - ``"physical"``:  h = 1.2 (m / rho)^(1/3)      (~58 neighbours in 2h)
    - ``"pixel"``:     h = 0.75 * pixel pitch        (HBM-bound regime)
    - ``"knn32"``:     h = 1/2 distance to the 32nd nearest neighbour
                       (scipy cKDTree; the law BASELINE.md's container
                       timings used; small N only)

Everything is float64 here; callers round to float32 where the GPU path is fed.
"""
from __future__ import annotations

import numpy as np

__all__ = ["plummer", "plummer_torch"]


def plummer(n: int, seed: int = 0, h_law: str = "physical", *, extent: float = 4.0,
            grid: int | None = None):
    """Return a dict of float64 arrays: pos (n,3), h, m, rho, T, r."""
    rng = np.random.default_rng(seed)
    u = rng.uniform(0.0, 0.999, n)
    cos_t = rng.uniform(-1.0, 1.0, n)
    phi = rng.uniform(0.0, 2.0 * np.pi, n)
    r = 1.0 / np.sqrt(u ** (-2.0 / 3.0) - 1.0)
    sin_t = np.sqrt(np.maximum(0.0, 1.0 - cos_t * cos_t))
    pos = np.empty((n, 3), dtype=np.float64)
    pos[:, 0] = r * sin_t * np.cos(phi)
    pos[:, 1] = r * sin_t * np.sin(phi)
    pos[:, 2] = r * cos_t
    rho = (3.0 / (4.0 * np.pi)) * (1.0 + r * r) ** -2.5
    m = np.full(n, 1.0 / n)
    T = 1.0e4 / np.sqrt(1.0 + r * r)
    if h_law == "physical":
        h = 1.2 * np.cbrt(m / rho)
    elif h_law == "pixel":
        if grid is None:
            raise ValueError("h_law='pixel' needs grid=")
        h = np.full(n, 0.75 * (2.0 * extent) / grid)
    elif h_law == "knn32":
        from scipy.spatial import cKDTree
        d, _ = cKDTree(pos).query(pos, k=33)
        h = 0.5 * d[:, 32]
    else:
        raise ValueError(f"unknown h_law {h_law!r}")
    return {"pos": pos, "h": h, "m": m, "rho": rho, "T": T, "r": r}


def plummer_torch(n: int, seed: int = 0, h_law: str = "pixel", *, extent: float = 4.0,
                  grid: int = 4096, device="cuda", z_range=None):
    """Same laws as :func:`plummer`, generated directly in device memory (float32 SoA).

    Used by ``bench.py`` so that 10^8-particle inputs are resident in HBM without a
    host round trip.  Different random stream from :func:`plummer` (torch Philox),
    identical distribution.  Returns dict of 1-D float32 tensors x, y, z, h, m, T.
    ``z_range=(lo, hi)`` keeps only particles with lo <= z < hi (Z-slab sharding).
    """
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f64 = torch.float64
    u = torch.rand(n, generator=g, device=device, dtype=f64) * 0.999
    cos_t = torch.rand(n, generator=g, device=device, dtype=f64) * 2.0 - 1.0
    phi = torch.rand(n, generator=g, device=device, dtype=f64) * (2.0 * np.pi)
    r = 1.0 / torch.sqrt(u.clamp_min(1e-300) ** (-2.0 / 3.0) - 1.0)
    del u
    sin_t = torch.sqrt((1.0 - cos_t * cos_t).clamp_min(0.0))
    x = (r * sin_t * torch.cos(phi)).float()
    y = (r * sin_t * torch.sin(phi)).float()
    z = (r * cos_t).float()
    del sin_t, cos_t, phi
    m = torch.full((n,), 1.0 / n, device=device, dtype=torch.float32)
    T = (1.0e4 / torch.sqrt(1.0 + r * r)).float()
    if h_law == "physical":
        rho = (3.0 / (4.0 * np.pi)) * (1.0 + r * r) ** -2.5
        h = (1.2 * torch.pow((1.0 / n) / rho, 1.0 / 3.0)).float()
        del rho
    elif h_law == "pixel":
        h = torch.full((n,), 0.75 * (2.0 * extent) / grid, device=device, dtype=torch.float32)
    else:
        raise ValueError(f"unknown h_law {h_law!r}")
    del r
    out = {"x": x, "y": y, "z": z, "h": h, "m": m, "T": T}
    if z_range is not None:
        lo, hi = z_range
        keep = (z >= lo) & (z < hi)
        out = {k: v[keep].contiguous() for k, v in out.items()}
    return out
