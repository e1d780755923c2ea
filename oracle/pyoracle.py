"""ctypes binding of the CPU oracle (oracle/asp_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` as the checker.  The product path never imports it.

Inputs are the reference's own: positions (N, 3) float64, smoothing lengths, properties,
``CoordinateAxes`` value (0/1/2) -> (u, v) columns exactly as
``_projector.py:38-46`` / ``_pixel_calculations.pyx:20-28`` select them.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ASP_ORACLE_LIB: another build of the same source (tests/test_oracle_sanitized.py loads the
# AddressSanitizer / UBSan build oracle/_san/liboracle_san.so through it)
LIB_PATH = os.environ.get("ASP_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

KERNELS = {"cubic": 0, "quartic_spline_kernel": 0, "wendland_c2": 1, "indicator": 2}
AXIS_COLS = {0: (1, 2), 1: (0, 2), 2: (0, 1)}

_lib = None

_d = C.POINTER(C.c_double)
_i64 = C.POINTER(C.c_int64)
_i32 = C.POINTER(C.c_int32)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_kernel_eval.argtypes = [C.c_int, _d, _d, _d, C.c_int64]
        L.oracle_create_image.argtypes = [_d, _d, _d, _d, _d, _d, C.c_int64, C.c_int, C.c_int, C.c_int,
                                          C.c_double, C.c_double, C.c_double, C.c_double, C.c_int,
                                          _i64, C.c_int64, C.c_int, _d]
        L.oracle_chunk_members.argtypes = [_d, _d, _d, C.c_int64, C.c_int, C.c_int, C.c_int,
                                           C.c_double, C.c_double, C.c_double, C.c_double,
                                           _i64, _i32, C.c_int64]
        L.oracle_chunk_members.restype = C.c_int64
        L.oracle_pixel_neighbours.argtypes = [_d, _d, _d, C.c_int64, C.c_int, C.c_int, C.c_int,
                                              C.c_double, C.c_double, C.c_double, C.c_double,
                                              _i64, C.c_int64, _i64, _i32, C.c_int64]
        L.oracle_pixel_neighbours.restype = C.c_int64
        L.oracle_project_scatter.argtypes = [_d, _d, _d, _d, _d, _d, _d, C.c_int64, C.c_int, C.c_int,
                                             C.c_int, C.c_double, C.c_double, C.c_double,
                                             C.c_double, C.c_int, C.c_int, _d, _d]
        L.oracle_chunk_ranges.argtypes = [_d, _d, _d, C.c_int64, C.c_int, C.c_int, C.c_int,
                                          C.c_double, C.c_double, C.c_double, C.c_double,
                                          _i32, _i32, _i32, _i32]
        L.oracle_project3d.argtypes = [_d, _d, _d, _d, _d, C.c_int64, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int] + [C.c_double] * 6 + [C.c_int, C.c_int,
                                                                                _d]
        L.oracle_voxel_neighbours.argtypes = [_d, _d, _d, _d, C.c_int64, C.c_int, C.c_int,
                                              C.c_int] + [C.c_double] * 6 + [_i64, C.c_int64,
                                                                            _i64, _i32, C.c_int64]
        L.oracle_voxel_neighbours.restype = C.c_int64
        _lib = L
    return _lib


def _p(a, t=_d):
    return a.ctypes.data_as(t) if a is not None else None


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _uv(positions, axis):
    positions = np.asarray(positions, dtype=np.float64).reshape(-1, 3)
    a, b = AXIS_COLS[int(getattr(axis, "value", axis))]
    return _f64(positions[:, a]), _f64(positions[:, b])


def _axes(positions, projection_axis):
    """(u, v, cu, cv): pixel-test columns and cull columns.  ``projection_axis`` is an
    axis (0/1/2 or enum: both the same) or a (pixel axis, cull axis) pair -- the
    reference derives the two separately (_projector.py:38-46 vs .pyx:20-28)."""
    if isinstance(projection_axis, tuple):
        pa, ca = (int(a) for a in projection_axis)
    else:
        pa = ca = int(getattr(projection_axis, "value", projection_axis))
    u, v = _uv(positions, pa)
    if ca == pa:
        return u, v, None, None
    cu, cv = _uv(positions, ca)
    return u, v, cu, cv


def kernel_eval(kernel, r, h):
    r, h = _f64(r), _f64(h)
    w = np.empty_like(r)
    lib().oracle_kernel_eval(KERNELS[kernel], _p(r), _p(h), _p(w), r.size)
    return w


def create_image(positions, smoothing_lengths, particle_properties, image_size, chunk_size,
                 projection_axis, x_min, x_max, y_min, y_max, kernel="cubic", nthreads=0,
                 chunk_ids=None, out=None):
    """Reference-exact restatement of ``create_image`` (gather, fp64).  ``out``: a
    C-contiguous float64 (nx, ny) array written in place (with ``chunk_ids`` only those
    chunks' pixels are touched, so concurrent calls on disjoint chunks may share it)."""
    u, v, cu, cv = _axes(positions, projection_axis)
    h, A = _f64(smoothing_lengths), _f64(particle_properties)
    nx, ny = int(image_size[0]), int(image_size[1])
    if out is None:
        img = np.zeros((nx, ny), dtype=np.float64)
    else:
        img = out
        if img.shape != (nx, ny) or img.dtype != np.float64 or not img.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous float64 (nx, ny) array")
    ids = None if chunk_ids is None else np.ascontiguousarray(chunk_ids, dtype=np.int64)
    rc = lib().oracle_create_image(_p(u), _p(v), _p(cu), _p(cv), _p(h), _p(A), u.size, nx, ny, int(chunk_size),
                                   float(x_min), float(x_max), float(y_min), float(y_max),
                                   KERNELS[kernel], _p(ids, _i64), 0 if ids is None else ids.size,
                                   int(nthreads), _p(img))
    if rc != 0:
        raise RuntimeError(f"oracle_create_image failed ({rc})")
    return img


def create_image_cols(u, v, h, A, image_size, chunk_size, x_min, x_max, y_min, y_max,
                      kernel="cubic", nthreads=0, chunk_ids=None, out=None):
    """``create_image`` on prepared C-contiguous float64 columns (u, v = the projected
    axes, cull on the same columns), no per-call column copies: the CPU baseline's
    per-chunk timing calls this from a thread pool on a shared ``out``."""
    nx, ny = int(image_size[0]), int(image_size[1])
    img = np.zeros((nx, ny), dtype=np.float64) if out is None else out
    ids = None if chunk_ids is None else np.ascontiguousarray(chunk_ids, dtype=np.int64)
    rc = lib().oracle_create_image(_p(u), _p(v), None, None, _p(h), _p(A), u.size, nx, ny,
                                   int(chunk_size), float(x_min), float(x_max), float(y_min),
                                   float(y_max), KERNELS[kernel], _p(ids, _i64),
                                   0 if ids is None else ids.size, int(nthreads), _p(img))
    if rc != 0:
        raise RuntimeError(f"oracle_create_image failed ({rc})")
    return img


def project_scatter(u, v, h, a0, a1, image_size, chunk_size, x_min, x_max, y_min, y_max,
                    kernel="cubic", nthreads=0, cu=None, cv=None):
    """O(pairs) restatement; returns (out0, out1-or-None), float64 (nx, ny).  cu, cv:
    the cull's columns when they differ from (u, v) (the reference's mixed axes)."""
    u, v, h, a0 = _f64(u), _f64(v), _f64(h), _f64(a0)
    cu = None if cu is None else _f64(cu)
    cv = None if cv is None else _f64(cv)
    a1 = None if a1 is None else _f64(a1)
    nx, ny = int(image_size[0]), int(image_size[1])
    o0 = np.empty((nx, ny), np.float64)
    o1 = None if a1 is None else np.empty((nx, ny), np.float64)
    rc = lib().oracle_project_scatter(_p(u), _p(v), _p(cu), _p(cv), _p(h), _p(a0), _p(a1), u.size, nx, ny,
                                      int(chunk_size), float(x_min), float(x_max), float(y_min),
                                      float(y_max), KERNELS[kernel], int(nthreads), _p(o0), _p(o1))
    if rc != 0:
        raise RuntimeError(f"oracle_project_scatter failed ({rc})")
    return o0, o1


def chunk_members(positions, smoothing_lengths, image_size, chunk_size, projection_axis,
                  x_min, x_max, y_min, y_max):
    u, v = _uv(positions, projection_axis)
    h = _f64(smoothing_lengths)
    nx, ny, cs = int(image_size[0]), int(image_size[1]), int(chunk_size)
    nch = ((nx + cs - 1) // cs) * ((ny + cs - 1) // cs)
    offs = np.zeros(nch + 1, np.int64)
    cap = max(1, u.size * 4)
    while True:
        idx = np.empty(cap, np.int32)
        t = lib().oracle_chunk_members(_p(u), _p(v), _p(h), u.size, nx, ny, cs, float(x_min),
                                       float(x_max), float(y_min), float(y_max), _p(offs, _i64),
                                       _p(idx, _i32), cap)
        if t >= 0:
            return offs, idx[:t]
        cap = -t


def pixel_neighbours(positions, smoothing_lengths, image_size, chunk_size, projection_axis,
                     x_min, x_max, y_min, y_max, pixels):
    u, v = _uv(positions, projection_axis)
    h = _f64(smoothing_lengths)
    pix = np.ascontiguousarray(pixels, dtype=np.int64)
    offs = np.zeros(pix.size + 1, np.int64)
    cap = max(1, u.size)
    while True:
        idx = np.empty(cap, np.int32)
        t = lib().oracle_pixel_neighbours(_p(u), _p(v), _p(h), u.size, int(image_size[0]),
                                          int(image_size[1]), int(chunk_size), float(x_min),
                                          float(x_max), float(y_min), float(y_max), _p(pix, _i64),
                                          pix.size, _p(offs, _i64), _p(idx, _i32), cap)
        if t >= 0:
            return offs, idx[:t]
        cap = -t


def chunk_ranges(u, v, h, image_size, chunk_size, x_min, x_max, y_min, y_max):
    u, v, h = _f64(u), _f64(v), _f64(h)
    out = [np.empty(u.size, np.int32) for _ in range(4)]
    lib().oracle_chunk_ranges(_p(u), _p(v), _p(h), u.size, int(image_size[0]), int(image_size[1]),
                              int(chunk_size), float(x_min), float(x_max), float(y_min),
                              float(y_max), *[_p(o, _i32) for o in out])
    return tuple(out)


def project3d(x, y, z, h, a, cube_size, extent, kernel="cubic", planes=None, nthreads=0):
    """Cube restatement (scatter, fp64): (nx, ny, k_hi - k_lo) float64.
    ``extent = (x_min, x_max, y_min, y_max, z_min, z_max)``."""
    x, y, z, h, a = (_f64(t) for t in (x, y, z, h, a))
    nx, ny, nz = (int(c) for c in cube_size)
    k_lo, k_hi = (0, nz) if planes is None else (int(planes[0]), int(planes[1]))
    out = np.empty((nx, ny, k_hi - k_lo), np.float64)
    rc = lib().oracle_project3d(_p(x), _p(y), _p(z), _p(h), _p(a), x.size, nx, ny, nz, k_lo,
                                k_hi, *[float(e) for e in extent], KERNELS[kernel],
                                int(nthreads), _p(out))
    if rc != 0:
        raise RuntimeError(f"oracle_project3d failed ({rc})")
    return out


def voxel_neighbours(x, y, z, h, cube_size, extent, voxels):
    x, y, z, h = (_f64(t) for t in (x, y, z, h))
    vox = np.ascontiguousarray(voxels, dtype=np.int64)
    offs = np.zeros(vox.size + 1, np.int64)
    cap = max(1, x.size)
    while True:
        idx = np.empty(cap, np.int32)
        t = lib().oracle_voxel_neighbours(_p(x), _p(y), _p(z), _p(h), x.size,
                                          *[int(c) for c in cube_size],
                                          *[float(e) for e in extent], _p(vox, _i64), vox.size,
                                          _p(offs, _i64), _p(idx, _i32), cap)
        if t >= 0:
            return offs, idx[:t]
        cap = -t


# ---------------------------------------------------------------------------------------
# Periodic box: NumPy restatement of the reference's helpers,
# tools/_periodic_box_manipulations.py:10-72 (pinned by tests/golden/g8_periodic.npz, made
# by running the reference's own function bodies), and of the periodic images the staging
# pass appends (asp_stage_particles; build-defined, include/asp.h).
# ---------------------------------------------------------------------------------------
def pb_wrap(x, L, centred=False):
    """make_periodic (:36-43): one wrap by L of the coordinates outside the box."""
    x = np.array(x, dtype=np.float64)
    lo = -(L / 2) if centred else 0.0
    out = (x < lo) | (x >= lo + L)
    s = np.sign(x + (L / 2) if centred else x)
    return np.where(out, -s * L + x, x)


def pb_shift(x, c, L, kind, centred=False):
    """shift_origin (:54-57) / shift_centre (:63-69)."""
    x = np.asarray(x, dtype=np.float64)
    if kind == "origin" or centred:
        return pb_wrap(x - c, L, centred)
    return pb_wrap(x + ((L / 2) - c), L, False)


def pb_displacement(frm, to, L):
    """calculate_wrapped_displacement (:10-20)."""
    d = np.asarray(to, np.float64) - np.asarray(frm, np.float64)
    return np.where(np.abs(d) > L / 2, d - np.sign(d) * L, d)


def pb_distance(frm, to, L, squared=False):
    """calculate_wrapped_distance (:22-34)."""
    d = pb_displacement(frm, to, L)
    s = (d ** 2).sum(axis=1 if d.ndim > 1 else 0)
    return s if squared else np.sqrt(s)


def stage_particles(positions, h, props, axis, L=None, centre=None, shift=None,
                    centred=False, images=False):
    """What asp_stage_particles produces: (u, v, h, props) float32, the originals in input
    order followed by the periodic images (the device appends those in an unspecified
    order; compare them as a set)."""
    pos = np.asarray(positions, np.float64).reshape(-1, 3)
    a, b = AXIS_COLS[int(getattr(axis, "value", axis))]
    x, y = pos[:, a], pos[:, b]
    if shift == "wrap":
        x, y = pb_wrap(x, L, centred), pb_wrap(y, L, centred)
    elif shift in ("origin", "centre"):
        c = np.asarray(centre, np.float64)
        x, y = pb_shift(x, c[a], L, shift, centred), pb_shift(y, c[b], L, shift, centred)
    hh = None if h is None else np.asarray(h, np.float64)
    pp = [np.asarray(p, np.float64) for p in props]
    cols = [x, y] + ([hh] if hh is not None else []) + pp
    out = [c.astype(np.float32) for c in cols]
    if not images:
        return out
    lo = -(L / 2) if centred else 0.0
    R = 2.0 * np.abs(hh) * (1.0 + 2.0 ** -20) + 2.0 ** -20 * L
    inside = (x >= lo) & (x < lo + L) & (y >= lo) & (y < lo + L)
    ok = inside & (R > 0) & (R <= 3 * L)
    # copies at x + k L whose reach [x + kL - R, x + kL + R] meets [lo, lo + L)
    with np.errstate(invalid="ignore"):
        kx0 = np.where(ok, np.floor((lo - x - R) / L) + 1, 0).astype(np.int64)
        kx1 = np.where(ok, np.ceil((lo + L - x + R) / L) - 1, 0).astype(np.int64)
        ky0 = np.where(ok, np.floor((lo - y - R) / L) + 1, 0).astype(np.int64)
        ky1 = np.where(ok, np.ceil((lo + L - y + R) / L) - 1, 0).astype(np.int64)
    extra = [[] for _ in cols]
    for kx in range(-3, 4):
        for ky in range(-3, 4):
            if kx == 0 and ky == 0:
                continue
            sel = (kx0 <= kx) & (kx <= kx1) & (ky0 <= ky) & (ky <= ky1)
            shifted = [x[sel] + kx * L, y[sel] + ky * L] + [c[sel] for c in cols[2:]]
            for k, c in enumerate(shifted):
                extra[k].append(c)
    return [np.concatenate([o] + [e.astype(np.float32) for e in ex]) for o, ex in zip(out, extra)]


def table_interp3(table, grids, points, fill=-np.inf):
    """Linear interpolation of a 3-D table (IonisationTableBase.__call__,
    data_structures/_IonisationTable.py:44-52 -> scipy 1.15 RegularGridInterpolator with
    bounds_error=False, fill_value=-inf), restated in NumPy with scipy's operation order
    (_rgi.py: find_indices, _evaluate_linear, then fill, then NaN):
      i_d = largest i with g_d[i] <= x_d, clamped to [0, n_d - 2];
      y_d = (x_d - g_d[i_d]) / (g_d[i_d + 1] - g_d[i_d]);
      v = 0; for the 8 corners (last axis fastest): v = v + t[corner] * ((w0 * w1) * w2)."""
    t = np.asarray(table, np.float64)
    P = np.asarray(points, np.float64).reshape(-1, 3)
    idx, y = [], []
    for d in range(3):
        g = np.asarray(grids[d], np.float64)
        x = P[:, d]
        i = np.clip(np.searchsorted(g, x, side="right") - 1, 0, g.size - 2)
        with np.errstate(invalid="ignore"):
            y.append((x - g[i]) / (g[i + 1] - g[i]))
        idx.append(i)
    v = np.zeros(P.shape[0])
    for a in (0, 1):
        for b in (0, 1):
            for e in (0, 1):
                w0 = y[0] if a else 1 - y[0]
                w1 = y[1] if b else 1 - y[1]
                w2 = y[2] if e else 1 - y[2]
                with np.errstate(invalid="ignore"):
                    v = v + t[idx[0] + a, idx[1] + b, idx[2] + e] * ((w0 * w1) * w2)
    oob = np.zeros(P.shape[0], bool)
    for d in range(3):
        g = np.asarray(grids[d], np.float64)
        oob |= (P[:, d] < g[0]) | (P[:, d] > g[-1])
    v[oob] = fill
    v[np.isnan(P).any(axis=1)] = np.nan
    return v


def table_at_redshift(table, grids, points2, z, zaxis=2, fill=-np.inf):
    """IonisationTableBase.evaluate_at_redshift (_IonisationTable.py:54-58): the constant z
    inserted as column `zaxis`, then table_interp3."""
    P2 = np.asarray(points2, np.float64)
    P = np.empty((P2.shape[0], 3))
    P[:, np.arange(3) != zaxis] = P2
    P[:, zaxis] = z
    return table_interp3(table, grids, P, fill)
