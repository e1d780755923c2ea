"""``create_image`` -- drop-in for the reference's map renderer, running on MI355X.

Reference: /root/reference/src/astro_sph_tools/tools/projections/_projector.py:75-120
(with process_chunk :13-73 and calculate_pixel_value, _pixel_calculations.pyx:9-36).

Same signature, argument meaning and result: a fresh ``np.float64`` array of shape
``(Nx, Ny)`` indexed ``img[x_index, y_index]``; pixel (xi, yi) samples the lower-left
corner ``(x_min + xi*dx, y_min + yi*dy)`` with ``dy = (y_max - y_min)/Nx`` (reference
quirk S2); the value is the sum of ``A_p W(r_p, h_p)`` over particles passing the
reference's cull of the ``chunk_size`` tile holding the pixel and ``r_p^2 < (2h_p)^2``.

Differences, all documented in DESIGN.md §6: values are sums of float32 terms on the GPU
(upcast on return); neighbour sets are decided with the reference's fp64 arithmetic on
the caller's own fp64 values and are identical; an arbitrary ``kernel_func`` is evaluated
on the host over device-produced neighbour pairs, in batches (it must be element-wise);
``x_max > x_min`` and ``y_max > y_min`` are required (ValueError); non-finite particle
inputs are excluded.
"""
from __future__ import annotations

import numbers

import numpy as np

from ... import _lib
from ..._axes import reference_axes
from ._kernels import kernel_id_of, native_kernel_id, quartic_spline_kernel


def _lengths(positions, smoothing_lengths, *fields):
    pos = np.asarray(positions)
    if pos.ndim != 2 or pos.shape[1] != 3:
        raise ValueError(f"positions must have shape (N, 3), got {pos.shape}")
    n = pos.shape[0]
    lens = [np.asarray(f).reshape(-1).shape[0] for f in (smoothing_lengths,) + fields]
    if any(k != n for k in lens):
        raise ValueError(f"positions ({n}), smoothing_lengths ({lens[0]}) and "
                         f"particle_properties ({lens[1]}) differ in length")


def _check_chunk_size(chunk_size):
    # the reference feeds chunk_size to range(0, N, chunk_size)
    if not isinstance(chunk_size, numbers.Integral):
        raise TypeError(f"'{type(chunk_size).__name__}' object cannot be interpreted as an integer")
    if chunk_size == 0:
        raise ValueError("range() arg 3 must not be zero")
    return int(chunk_size)


def _run(positions, smoothing_lengths, props, projection_axis, image_size, chunk_size,
         extent, kernel_id, ratio, deterministic, device):
    """The reader's fp64 arrays straight to asp_project2d_f64 (staging in HBM -- the
    host-side step of _projector.py:38-51 -- and the projection with the reference's
    fp64 decisions on the original values).  Returns the float32 host map(s)."""
    nx, ny = int(image_size[0]), int(image_size[1])
    out0 = np.zeros((nx, ny), dtype=np.float32)
    out1 = None if len(props) < 2 else np.zeros_like(out0)
    if nx <= 0 or ny <= 0 or chunk_size < 0:
        # empty image, or range(0, N, negative) -> no tiles -> all zeros (reference)
        return out0, out1
    _lib.require_gpu(device)
    from ...device import project2d_f64
    pos = np.asarray(positions)
    if pos.ndim != 2 or pos.shape[1] != 3:
        raise ValueError(f"positions must have shape (N, 3), got {pos.shape}")
    return project2d_f64(pos, smoothing_lengths, props[0], props[1] if len(props) > 1 else None,
                         projection_axis=reference_axes(projection_axis), image_size=(nx, ny),
                         extent=tuple(float(np.asarray(e)) for e in extent),
                         chunk_size=chunk_size, kernel=kernel_id, ratio=ratio,
                         deterministic=deterministic, device=device, out0=out0, out1=out1)


def _run_callable(positions, smoothing_lengths, props, projection_axis, image_size, chunk_size,
                  extent, kernel_func, device, mode, deterministic):
    nx, ny = int(image_size[0]), int(image_size[1])
    if nx <= 0 or ny <= 0 or chunk_size < 0:
        return [np.zeros((max(nx, 0), max(ny, 0))) for _ in props]
    _lib.require_gpu(device)
    from ._plugin import project_callable
    pos = np.asarray(positions)
    if pos.ndim != 2 or pos.shape[1] != 3:
        raise ValueError(f"positions must have shape (N, 3), got {pos.shape}")
    return project_callable(pos, smoothing_lengths, props, reference_axes(projection_axis),
                            (nx, ny), chunk_size, extent, kernel_func, device=device, mode=mode,
                            deterministic=deterministic)


def create_image(positions: np.ndarray, smoothing_lengths: np.ndarray,
                 particle_properties: np.ndarray, image_size: tuple, chunk_size: int,
                 projection_axis, x_min: float, x_max: float, y_min: float, y_max: float,
                 kernel_func=quartic_spline_kernel, *, device: int = 0,
                 dtype=np.float64, deterministic: bool = False,
                 kernel_func_mode: str = "batch") -> np.ndarray:
    """Project particle property A onto an (Nx, Ny) pixel grid (reference semantics).

    ``device`` selects the GPU; ``dtype=np.float32`` skips the host upcast (opt-in);
    ``deterministic=True`` selects int64 fixed-point accumulation (bitwise reproducible,
    input-order independent; see ASP_F_DETERMINISTIC in include/asp.h) -- for an arbitrary
    ``kernel_func``, per-pixel sums in particle order.  ``kernel_func_mode`` (arbitrary
    callables only, _plugin.py): ``"batch"`` calls it on many pixels' pairs at once (it
    must be element-wise), ``"per_pixel"`` once per pixel exactly as the reference does.
    """
    cs = _check_chunk_size(chunk_size)
    kid = kernel_id_of(kernel_func)
    _lengths(positions, smoothing_lengths, particle_properties)
    if kid is None:  # an arbitrary Python kernel: the plugin path (_plugin.py)
        img, = _run_callable(positions, smoothing_lengths, [particle_properties],
                             projection_axis, image_size, cs, (x_min, x_max, y_min, y_max),
                             kernel_func, device, kernel_func_mode, deterministic)
        return img.astype(dtype, copy=False)
    img, _ = _run(positions, smoothing_lengths, [particle_properties], projection_axis,
                  image_size, cs, (x_min, x_max, y_min, y_max), kid, False, deterministic,
                  device)
    return img.astype(dtype, copy=False)


def create_weighted_image(positions, smoothing_lengths, weights, values, image_size,
                          chunk_size, projection_axis, x_min, x_max, y_min, y_max,
                          kernel_func=quartic_spline_kernel, *, device: int = 0,
                          return_components: bool = False, dtype=np.float64,
                          deterministic: bool = False, kernel_func_mode: str = "batch"):
    """Weighted-average map, e.g. mass-weighted temperature.

    ``sum(w v W) / sum(w W)`` per pixel over the same neighbour sets as
    :func:`create_image`, 0 where the denominator is 0.  Equals
    ``create_image(.., w*v, ..) / create_image(.., w, ..)`` (two reference calls), computed
    in one pass with both maps accumulated together.  With ``return_components`` the two
    sums are returned as well: ``(ratio, sum_wvW, sum_wW)``.
    """
    cs = _check_chunk_size(chunk_size)
    kid = kernel_id_of(kernel_func)
    if deterministic and kid is not None:
        # the native deterministic mode is an int64 fixed point per tile: a ratio of two
        # such maps is imprecise where only kernel tails reach; the plug-in
        # path's deterministic mode (fp64 sums in particle order) has no such limit
        raise ValueError("deterministic=True cannot form a weighted (ratio) map with a native "
                         "kernel: use deterministic=False, or pass the kernel as a plain "
                         "Python callable (the kernel_func plug-in sums in fp64, in order)")
    _lengths(positions, smoothing_lengths, weights)
    w = np.asarray(weights, dtype=np.float64).reshape(-1)
    vals = np.asarray(values, dtype=np.float64).reshape(-1)
    if vals.shape[0] != w.shape[0]:
        raise ValueError("values and positions differ in length")
    ext = (x_min, x_max, y_min, y_max)
    if kid is None:  # an arbitrary Python kernel: the plugin path (_plugin.py)
        s0, s1 = _run_callable(positions, smoothing_lengths, [w * vals, w], projection_axis,
                               image_size, cs, ext, kernel_func, device, kernel_func_mode,
                               deterministic)
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = np.where(s1 != 0, s0 / s1, 0.0)
        if return_components:
            return ratio.astype(dtype, copy=False), s0.astype(dtype), s1.astype(dtype)
        return ratio.astype(dtype, copy=False)
    if return_components:
        s0, s1 = _run(positions, smoothing_lengths, [w * vals, w], projection_axis, image_size,
                      cs, ext, kid, False, deterministic, device)
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = np.where(s1 != 0, s0.astype(np.float64) / s1, 0.0)
        return ratio.astype(dtype, copy=False), s0.astype(dtype), s1.astype(dtype)
    r, _ = _run(positions, smoothing_lengths, [w * vals, w], projection_axis, image_size, cs,
                ext, kid, True, deterministic, device)
    return r.astype(dtype, copy=False)


def create_images(positions, smoothing_lengths, particle_properties, image_size, chunk_size,
                  projection_axis, x_min, x_max, y_min, y_max,
                  kernel_func=quartic_spline_kernel, *, device: int = 0, dtype=np.float64):
    """One :func:`create_image` map per array of ``particle_properties`` (a sequence of 1..6
    property arrays, e.g. mass, mass * temperature, ion masses) from ONE binning of the
    particles: the callers that render several maps of one snapshot
    (io/data_structures/_SnapshotBase.py:618-906) pay the counting and scattering once
    (asp_project2d_props_f64).  Same semantics as ``create_image`` per map (the
    reference's fp64 decisions on the reader's values); native kernels only."""
    import torch
    cs = _check_chunk_size(chunk_size)
    kid = native_kernel_id(kernel_func)
    props = [np.asarray(a, dtype=np.float64).reshape(-1) for a in particle_properties]
    if not 1 <= len(props) <= 6:
        raise ValueError("particle_properties: 1 .. 6 arrays")
    for a in props:
        _lengths(positions, smoothing_lengths, a)
    nx, ny = int(image_size[0]), int(image_size[1])
    if nx <= 0 or ny <= 0 or cs < 0:
        return [np.zeros((max(nx, 0), max(ny, 0)), dtype=dtype) for _ in props]
    _lib.require_gpu(device)
    from ...device import project2d_props_f64
    maps = project2d_props_f64(np.asarray(positions), smoothing_lengths, props,
                               projection_axis=reference_axes(projection_axis),
                               image_size=(nx, ny),
                               extent=tuple(float(np.asarray(e)) for e in (x_min, x_max, y_min, y_max)),
                               chunk_size=cs, kernel=kid, device=device)
    torch.cuda.synchronize(maps[0].device)
    return [m.cpu().numpy().astype(dtype, copy=False) for m in maps]


def create_periodic_image(positions, smoothing_lengths, particle_properties, image_size,
                          chunk_size, projection_axis, box_width, centre=None,
                          kernel_func=quartic_spline_kernel, *, origin_is_centre: bool = False,
                          device: int = 0, dtype=np.float64, deterministic: bool = False):
    """Map of a whole periodic box, footprints wrapping across its faces (SURVEY.md §8(f)
    rank 2: the reference ships the box helpers, tools/_periodic_box_manipulations.py, but
    its projector ignores periodicity).

    Positions are moved with the reference's ``shift_centre(positions, centre, box_width,
    origin_is_centre)`` when ``centre`` is given, else wrapped with ``calculate_periodic``
    (fp64, on the device).  The image spans the box ``[lo, lo + L)`` on both projected axes
    (``lo = 0``, or ``-L/2`` with ``origin_is_centre``) and each pixel is ``create_image``'s
    sum over every periodic image of every particle (the staged copies of
    ``asp_stage_particles``; same neighbour decisions, same kernels).
    """
    import torch

    from ...device import project2d
    from ...stage import stage_particles
    cs = _check_chunk_size(chunk_size)
    kid = native_kernel_id(kernel_func)
    L = float(box_width)
    nx, ny = int(image_size[0]), int(image_size[1])
    if nx <= 0 or ny <= 0 or cs < 0:
        return np.zeros((max(nx, 0), max(ny, 0)), dtype=dtype)
    u, v, h, props = stage_particles(positions, smoothing_lengths, particle_properties,
                                     projection_axis=projection_axis, box_width=L,
                                     centre=centre, shift="wrap" if centre is None else "centre",
                                     origin_is_centre=origin_is_centre, images=True,
                                     device=device)
    lo = -(L / 2) if origin_is_centre else 0.0
    out, _ = project2d(u, v, h, props[0], image_size=(nx, ny), extent=(lo, lo + L, lo, lo + L),
                       chunk_size=cs, kernel=kid, deterministic=deterministic)
    torch.cuda.synchronize(u.device)
    return out.cpu().numpy().astype(dtype, copy=False)
