"""The ``kernel_func`` plugin point for ARBITRARY Python kernels.

Reference: ``create_image(..., kernel_func)`` (_projector.py:26, 86) hands every pixel's
masked ``(r, h)`` to the callable and sums ``A * W`` (_pixel_calculations.pyx:30-34).  A
Python callable cannot run on the device, so the work splits:

* device -- the neighbour pairs: per-pixel counts (asp_project2d_f64 with the indicator
  kernel), then, tile range by tile range, every included (pixel, particle) pair with the
  reference's fp64 r^2 (asp_pairs_f64; the same exact decisions as the native kernels);
* host -- ``r = sqrt(r^2)`` (IEEE, as NumPy), ``W = kernel_func(r, h[pairs])`` on large
  batches, ``A * W`` and the per-pixel sums.

Differences from the reference, documented in DESIGN.md §6: the callable is called on
batches of many pixels' pairs at once (so it must be element-wise, as every SPH kernel
is), not once per pixel; the per-pixel sums run in pair order instead of NumPy's
pairwise order (~1e-16 relative).
"""
from __future__ import annotations

import numpy as np

from ... import _lib

TILE = 64
MAX_PAIRS = 1 << 25  # pairs per device call (12 B each on the host)


def project_callable(positions, smoothing_lengths, props, axes, image_size, chunk_size, extent,
                     kernel_func, device: int = 0, max_pairs=None):
    """Maps ``sum_pairs props[k][p] * kernel_func(r, h[p])`` for each of ``props``
    (float64 (nx, ny) arrays), ``axes`` = (pixel axis, cull axis)."""
    from ...device import project2d_f64
    if max_pairs is None:
        max_pairs = MAX_PAIRS
    nx, ny = int(image_size[0]), int(image_size[1])
    pos = np.ascontiguousarray(np.asarray(positions, dtype=np.float64))
    h = np.ascontiguousarray(np.asarray(smoothing_lengths, dtype=np.float64).reshape(-1))
    props = [np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1)) for a in props]
    outs = [np.zeros((nx, ny), dtype=np.float64) for _ in props]
    n = h.size
    if n == 0:
        return outs
    ext = tuple(float(np.asarray(e)) for e in extent)
    cnt, _ = project2d_f64(pos, h, np.ones(n), projection_axis=axes, image_size=(nx, ny),
                           extent=ext, chunk_size=chunk_size, kernel=_lib.ASP_KERNEL_INDICATOR,
                           device=device)
    cnt = cnt.astype(np.int64)  # exact: float32 sums of ones below 2^24
    ntx, nty = -(-nx // TILE), -(-ny // TILE)
    pad = np.zeros((ntx * TILE, nty * TILE), np.int64)
    pad[:nx, :ny] = cnt
    tiles = pad.reshape(ntx, TILE, nty, TILE).transpose(0, 2, 1, 3).reshape(ntx * nty, TILE * TILE)
    per_tile = tiles.sum(axis=1)
    axis_code = int(axes[0]) | (((int(axes[1]) + 1) << 4) if axes[1] != axes[0] else 0)
    L = _lib.lib()
    t0 = 0
    while t0 < ntx * nty:
        t1, tot = t0 + 1, int(per_tile[t0])
        while t1 < ntx * nty and tot + per_tile[t1] <= max_pairs:
            tot += int(per_tile[t1])
            t1 += 1
        counts = tiles[t0:t1].reshape(-1)
        offsets = np.zeros(counts.size + 1, np.int64)
        np.cumsum(counts, out=offsets[1:])
        if tot:
            part = np.empty(tot, np.int32)
            r2 = np.empty(tot, np.float64)
            _lib.check(L.asp_pairs_f64(
                _lib.ptr(pos, _lib._d), _lib.ptr(h, _lib._d), n, axis_code, *ext, nx, ny,
                int(chunk_size), t0, t1, _lib.ptr(offsets, _lib._i64), _lib.ptr(part, _lib._i32),
                _lib.ptr(r2, _lib._d), 0, device, None))
            W = np.asarray(kernel_func(np.sqrt(r2), h[part]), dtype=np.float64)
            if W.shape != r2.shape:
                raise ValueError(f"kernel_func returned shape {W.shape} for {r2.shape} pairs")
            nz = counts > 0
            starts = offsets[:-1][nz]
            for A, out in zip(props, outs):
                vals = np.zeros(counts.size)
                vals[nz] = np.add.reduceat(A[part] * W, starts)
                vals = vals.reshape(t1 - t0, TILE, TILE)
                for i, t in enumerate(range(t0, t1)):
                    tx, ty = divmod(t, nty)
                    x0, y0 = tx * TILE, ty * TILE
                    out[x0:x0 + TILE, y0:y0 + TILE] = vals[i, :min(TILE, nx - x0), :min(TILE, ny - y0)]
        t0 = t1
    return outs
