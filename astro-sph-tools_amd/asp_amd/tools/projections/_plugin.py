"""The ``kernel_func`` plugin point for ARBITRARY Python kernels.

Reference: ``create_image(..., kernel_func)`` (_projector.py:26, 86) hands every pixel's
masked ``(r, h)`` to the callable and sums ``A * W`` (_pixel_calculations.pyx:30-34).  A
Python callable cannot run on the device, so the work splits:

* device -- the neighbour pairs, in one session per map (``asp_pairs_begin``: the
  particles are staged and binned ONCE, each GPU tile's pairs counted; ``asp_pairs_emit``:
  every included (pixel, particle) pair of a tile range with the reference's fp64 r^2, the
  same exact decisions as the native kernels, from the records the session keeps
  resident);
* host -- ``r = sqrt(r^2)`` (IEEE, as NumPy), ``W = kernel_func(r, h[pairs])``, ``A * W``
  and the per-pixel sums.

Two calling modes:

* ``"batch"`` (default): the callable is called on the pairs of many pixels at once (so it
  must be element-wise, as every SPH kernel is), per-pixel sums by ``np.add.reduceat``;
* ``"per_pixel"``: the reference's own contract (S15) -- one call per pixel, in the
  reference's chunk-by-chunk pixel order, on that pixel's arrays in particle order (empty
  arrays for pixels without neighbours), summed by ``np.sum`` as .pyx:34 does: the map is
  the reference's bit for bit on the same pairs, for any callable (stateful, non-element-
  wise); one Python call per pixel, all pairs held on the host.

Differences from the reference in batch mode: the per-pixel sums run in
pair order instead of NumPy's pairwise order (~1e-16 relative); with ``deterministic`` the
pairs of every pixel are put in particle order first, so the map is reproducible.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ... import _lib

TILE = 64
MAX_PAIRS = 1 << 25  # pairs per emit (12 B each on the host)


class _Session:
    """asp_pairs_begin / asp_pairs_emit / asp_pairs_end on host arrays."""

    def __init__(self, pos, h, axes, extent, image_size, chunk_size, device):
        self.nx, self.ny = int(image_size[0]), int(image_size[1])
        self.ntx, self.nty = -(-self.nx // TILE), -(-self.ny // TILE)
        self.tile_pairs = np.zeros(self.ntx * self.nty, np.int64)
        self._keep = (pos, h)
        axis_code = int(axes[0]) | (((int(axes[1]) + 1) << 4) if axes[1] != axes[0] else 0)
        self._h = C.c_void_p()
        L = _lib.lib()
        _lib.check(L.asp_pairs_begin(
            _lib.ptr(pos, _lib._d), _lib.ptr(h, _lib._d), h.size, axis_code, *extent, self.nx,
            self.ny, int(chunk_size), 0, device, None, _lib.ptr(self.tile_pairs, _lib._i64),
            C.byref(self._h)))

    def emit(self, t0, t1):
        """(offsets, particle, r2) of tiles [t0, t1)."""
        tot = int(self.tile_pairs[t0:t1].sum())
        offsets = np.empty((t1 - t0) * TILE * TILE + 1, np.int64)
        part = np.empty(max(tot, 1), np.int32)
        r2 = np.empty(max(tot, 1), np.float64)
        _lib.check(_lib.lib().asp_pairs_emit(self._h, t0, t1, _lib.ptr(offsets, _lib._i64),
                                             _lib.ptr(part, _lib._i32), _lib.ptr(r2, _lib._d)))
        return offsets, part[:tot], r2[:tot]

    def close(self):
        if self._h:
            _lib.lib().asp_pairs_end(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _ranges(tile_pairs, max_pairs):
    """Consecutive tile ranges of at most max_pairs pairs (a single heavier tile alone)."""
    t0, nt = 0, tile_pairs.size
    while t0 < nt:
        t1, tot = t0 + 1, int(tile_pairs[t0])
        while t1 < nt and tot + int(tile_pairs[t1]) <= max_pairs:
            tot += int(tile_pairs[t1])
            t1 += 1
        yield t0, t1
        t0 = t1


def project_callable(positions, smoothing_lengths, props, axes, image_size, chunk_size, extent,
                     kernel_func, device: int = 0, max_pairs=None, mode: str = "batch",
                     deterministic: bool = False):
    """Maps ``sum_pairs props[k][p] * kernel_func(r, h[p])`` for each of ``props``
    (float64 (nx, ny) arrays), ``axes`` = (pixel axis, cull axis)."""
    if mode not in ("batch", "per_pixel"):
        raise ValueError(f"unknown kernel_func mode {mode!r}")
    if max_pairs is None:
        max_pairs = MAX_PAIRS
    nx, ny = int(image_size[0]), int(image_size[1])
    pos = np.ascontiguousarray(np.asarray(positions, dtype=np.float64))
    h = np.ascontiguousarray(np.asarray(smoothing_lengths, dtype=np.float64).reshape(-1))
    props = [np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1)) for a in props]
    # the session reads h.size rows of positions: every array must describe the same particles
    # (the native path's checks, device._f64_arg)
    if pos.ndim != 2 or pos.shape != (h.size, 3):
        raise ValueError(f"positions must be (N, 3) with N = len(smoothing_lengths) = {h.size}, "
                         f"got {pos.shape}")
    for a in props:
        if a.size != h.size:
            raise ValueError(f"property of {a.size} values for {h.size} particles")
    ext = tuple(float(np.asarray(e)) for e in extent)
    with _Session(pos, h, axes, ext, (nx, ny), chunk_size, device) as S:
        if mode == "per_pixel":
            return _per_pixel(S, h, props, nx, ny, int(chunk_size), kernel_func)
        outs = [np.zeros((nx, ny), dtype=np.float64) for _ in props]
        for t0, t1 in _ranges(S.tile_pairs, max_pairs):
            if not S.tile_pairs[t0:t1].any():
                continue
            offsets, part, r2 = S.emit(t0, t1)
            counts = np.diff(offsets)
            if deterministic:  # particle order inside every pixel: a reproducible sum
                pix = np.repeat(np.arange(counts.size), counts)
                order = np.lexsort((part, pix))
                part, r2 = part[order], r2[order]
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
                    tx, ty = divmod(t, S.nty)
                    x0, y0 = tx * TILE, ty * TILE
                    out[x0:x0 + TILE, y0:y0 + TILE] = vals[i, :min(TILE, nx - x0), :min(TILE, ny - y0)]
        return outs


def _per_pixel(S, h, props, nx, ny, cs, kernel_func):
    """The reference's loop (_projector.py:53-71 inside :89-111): chunks, then pixels;
    one kernel_func call per pixel on its pairs in particle order."""
    offsets, part, r2 = S.emit(0, S.ntx * S.nty)
    counts = np.diff(offsets)
    pix = np.repeat(np.arange(counts.size), counts)
    order = np.lexsort((part, pix))
    part, r2 = part[order], r2[order]
    # tile-layout slot q -> image pixel (xi, yi)
    q = np.arange(counts.size)
    t, k = np.divmod(q, TILE * TILE)
    tx, ty = np.divmod(t, S.nty)
    xi, yi = tx * TILE + k // TILE, ty * TILE + k % TILE
    inside = (xi < nx) & (yi < ny)
    start = np.zeros((nx, ny), np.int64)
    cnt = np.zeros((nx, ny), np.int64)
    start[xi[inside], yi[inside]] = offsets[:-1][inside]
    cnt[xi[inside], yi[inside]] = counts[inside]
    outs = [np.zeros((nx, ny), dtype=np.float64) for _ in props]
    for A, out in zip(props, outs):  # one reference call per property map
        for xc in range(0, nx, cs):
            for yc in range(0, ny, cs):
                for x in range(xc, min(xc + cs, nx)):
                    for y in range(yc, min(yc + cs, ny)):
                        a, b = start[x, y], start[x, y] + cnt[x, y]
                        sel = part[a:b]
                        W = kernel_func(np.sqrt(r2[a:b]), h[sel])
                        out[x, y] = np.sum(A[sel] * W)
    return outs
