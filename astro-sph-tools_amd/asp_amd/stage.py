"""Snapshot arrays -> the projector's device-resident float32 SoA.

The reader side of the path (io/data_structures/_SnapshotBase.py:599-725) hands the
projector positions (N, 3) float64 in row-major order plus float64 per-particle fields;
``create_image`` (_projector.py:38-51) selects the two projected columns and the
projector wants float32.  :func:`stage_particles` does that selection and conversion on
the device (``asp_stage_particles``: host arrays are streamed through HBM in chunks, the
copy of one chunk overlapping the conversion of the previous), so a snapshot field goes
from the reader to HBM without a host-side float32 copy.

The periodic options apply the reference's box helpers (tools/_periodic_box_manipulations.py)
on the way -- ``shift="centre"`` (shift_centre), ``"origin"`` (shift_origin), ``"wrap"``
(calculate_periodic), all fp64 and bit-identical to the reference -- and
``images=True`` appends a copy one box width over for every particle whose footprint
crosses a box face, so a projection of the staged set over the box is the periodic map
(``create_periodic_image``).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._axes import axis_index

_SHIFT = {None: 0, "wrap": _lib.ASP_PB_WRAP, "origin": _lib.ASP_PB_SHIFT_ORIGIN,
          "centre": _lib.ASP_PB_SHIFT_CENTRE, "center": _lib.ASP_PB_SHIFT_CENTRE}


def _is_device(a):
    return hasattr(a, "is_cuda") and a.is_cuda


def _host_f64(a, name, shape=None):
    x = np.ascontiguousarray(np.asarray(a), dtype=np.float64)
    if shape is not None and x.shape != shape:
        raise ValueError(f"{name} must have shape {shape}, got {x.shape}")
    return x


def _dev_f64(t, name, dev, n):
    import torch
    if t.dtype != torch.float64 or t.device != dev:
        raise ValueError(f"{name} must be a float64 tensor on {dev}")
    t = t.contiguous()
    if t.shape[0] != n:
        raise ValueError(f"{name} has {t.shape[0]} rows, expected {n}")
    return t


def stage_particles(positions, smoothing_lengths=None, *properties, projection_axis=2,
                    box_width=None, centre=None, shift=None, origin_is_centre: bool = False,
                    images: bool = False, device: int = 0, stream=None):
    """Stage particles for projection; returns ``(u, v, h, props)`` float32 device tensors.

    ``positions`` (N, 3) and the 1-D fields are NumPy (or unyt) host arrays, or float64
    torch tensors already on the device.  ``properties``: at most two fields (a0, a1).
    ``h`` is None when ``smoothing_lengths`` is None.  With images the tensors are longer
    than N: the periodic copies follow the N originals.
    """
    import torch
    if len(properties) > 2:
        raise ValueError("at most two properties per call")
    if shift not in _SHIFT:
        raise ValueError(f"shift must be one of {sorted(k for k in _SHIFT if k)} or None")
    pb = _SHIFT[shift]
    if origin_is_centre:
        pb |= _lib.ASP_PB_ORIGIN_IS_CENTRE
    if images:
        pb |= _lib.ASP_PB_IMAGES
    if (pb & ~_lib.ASP_PB_ORIGIN_IS_CENTRE) and box_width is None:
        raise ValueError("the periodic options need box_width")
    if shift in ("origin", "centre", "center") and centre is None:
        raise ValueError(f"shift={shift!r} needs centre")
    if images and smoothing_lengths is None:
        raise ValueError("periodic images need smoothing lengths")
    axis = axis_index(projection_axis)
    on_dev = _is_device(positions)
    if on_dev:
        dev = positions.device
        pos = positions.contiguous()
        if pos.dtype != torch.float64 or pos.dim() != 2 or pos.shape[1] != 3:
            raise ValueError("positions must be an (N, 3) float64 tensor")
        n = pos.shape[0]
        h = None if smoothing_lengths is None else _dev_f64(smoothing_lengths, "smoothing_lengths", dev, n)
        props = [_dev_f64(p, f"property {i}", dev, n) for i, p in enumerate(properties)]
        flags = _lib.ASP_F_DEVICE_PTRS
        device = dev.index or 0
    else:
        pos = np.asarray(positions)
        if pos.ndim != 2 or pos.shape[1] != 3:
            raise ValueError(f"positions must have shape (N, 3), got {pos.shape}")
        pos = _host_f64(pos, "positions")
        n = pos.shape[0]
        h = None if smoothing_lengths is None else _host_f64(np.asarray(smoothing_lengths).reshape(-1),
                                                             "smoothing_lengths", (n,))
        props = [_host_f64(np.asarray(p).reshape(-1), f"property {i}", (n,))
                 for i, p in enumerate(properties)]
        flags = 0
        _lib.require_gpu(device)
        dev = torch.device("cuda", device)
    c = None if centre is None else _host_f64(np.asarray(centre, dtype=np.float64).reshape(-1),
                                              "centre", (3,))
    L = float(box_width) if box_width is not None else 0.0
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    P, Pd = _lib.ptr, (lambda a: _lib.ptr(a, _lib._d))
    cap = n if not images else n + max(1024, n // 4)
    while True:
        outs = [torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
                for _ in range(2 + (h is not None) + len(props))]
        u, v = outs[0], outs[1]
        hf = outs[2] if h is not None else None
        pf = outs[2 + (h is not None):]
        n_out = _lib.C.c_int64(0)
        rc = _lib.lib().asp_stage_particles(
            Pd(pos), Pd(h), Pd(props[0] if props else None), Pd(props[1] if len(props) > 1 else None),
            n, axis, Pd(c), L, pb, P(u), P(v), P(hf), P(pf[0] if pf else None),
            P(pf[1] if len(pf) > 1 else None), cap, _lib.C.byref(n_out), flags, device, stream)
        if rc == _lib.ASP_ERR_INVALID and n_out.value > cap:
            cap = n_out.value  # more periodic images than guessed: once more, sized
            continue
        _lib.check(rc)
        m = n_out.value
        return u[:m], v[:m], (hf[:m] if hf is not None else None), [p[:m] for p in pf]
