"""Periodic-box helpers on the GPU, mirroring the reference module
/root/reference/src/astro_sph_tools/tools/_periodic_box_manipulations.py (:10-72).

Same names, arguments and results; the arithmetic is the reference's fp64 NumPy
operation sequence, done by ``asp_periodic`` / ``asp_wrapped_distance`` (asp_stage.hip),
bit-identical to it (tests/test_gpu_stage.py against the golden vectors G8, produced by
running the reference's own function bodies).  NumPy inputs give NumPy results; float64
torch tensors on the GPU stay there.  There is no CPU fallback: without a GPU these raise.

unyt arrays: the reference registers unyt overloads of ``calculate_periodic``,
``shift_origin`` and ``shift_centre`` (:49-51, :58-60, :70-72) that convert every operand
to one unit, run the NumPy body on the values and rewrap the result in that unit; the
wrapped displacement / distance work on unyt arrays through NumPy's unit propagation
(result in the units of ``to_positions``, squared for a squared distance).  The same is
done here for any unit-carrying array (``.value``, ``.units``, ``.to(units)`` -- unyt's
interface; unyt itself is not installed in this image, so the tests drive it with a
stand-in class: parity with unyt is unpinned beyond that interface).
"""
from __future__ import annotations

import numpy as np

from .. import _lib


def _has_units(x) -> bool:
    return hasattr(x, "units") and hasattr(x, "value") and hasattr(x, "to")


def _in(x, units):
    """The numerical values of ``x`` in ``units`` (plain arrays pass through)."""
    return x.to(units).value if _has_units(x) else x


def _wrap(like, values, units):
    """``values`` as an array of ``like``'s unit-carrying type, in ``units``."""
    return type(like)(values, units=units)


def _prep(x):
    """(device float64 tensor, was_numpy)."""
    import torch
    if hasattr(x, "is_cuda") and x.is_cuda:
        if x.dtype != torch.float64:
            raise ValueError("device tensors must be float64")
        return x.contiguous(), False
    a = np.ascontiguousarray(np.asarray(x), dtype=np.float64)
    _lib.require_gpu(0)
    return torch.from_numpy(a).to("cuda"), True


def _period(t, shape):
    """Elements after which a broadcast operand repeats in C order, or None."""
    full = int(np.prod(shape)) if len(shape) else 1
    if tuple(t.shape) == tuple(shape):
        return t, full
    if t.dim() <= len(shape) and tuple(t.shape) == tuple(shape[len(shape) - t.dim():]):
        return t, max(1, t.numel())
    return t.broadcast_to(shape).contiguous(), full  # other broadcasts: expanded on device


def _run(op, a, b, box_width, origin_is_centre=False):
    import torch
    ta, na = _prep(a)
    tb, nb = _prep(b) if b is not None else (None, True)
    shape = torch.broadcast_shapes(ta.shape, tb.shape) if tb is not None else ta.shape
    ta, pa = _period(ta, shape)
    pb = 1
    if tb is not None:
        tb, pb = _period(tb, shape)
    out = torch.empty(shape, dtype=torch.float64, device=ta.device)
    P = lambda t: _lib.ptr(t, _lib._d)  # noqa: E731
    _lib.check(_lib.lib().asp_periodic(
        op, P(ta), pa, P(tb), pb, out.numel(), float(box_width), int(bool(origin_is_centre)),
        P(out), ta.device.index or 0, torch.cuda.current_stream(ta.device).cuda_stream))
    return out.cpu().numpy() if (na and nb) else out


def calculate_wrapped_displacement(from_positions, to_positions, box_width):
    """``to - from`` with every component farther than half a box brought back by one box
    width (reference :10-20)."""
    if _has_units(to_positions):
        u = to_positions.units
        return _wrap(to_positions, _run(_lib.ASP_PB_DISPLACEMENT, _in(from_positions, u),
                                        to_positions.value, _in(box_width, u)), u)
    return _run(_lib.ASP_PB_DISPLACEMENT, from_positions, to_positions, box_width)


def calculate_wrapped_distance(from_position, to_positions, box_width,
                               do_squared_distance=False):
    """Length of the wrapped displacement (reference :22-34): rows of 3 for (N, 3)
    inputs, a scalar for two (3,) vectors."""
    import torch
    if _has_units(to_positions):
        u = to_positions.units
        d = calculate_wrapped_distance(_in(from_position, u), to_positions.value,
                                       _in(box_width, u), do_squared_distance)
        return _wrap(to_positions, d, u ** 2 if do_squared_distance else u)
    tf, nf = _prep(from_position)
    tt, nt = _prep(to_positions)
    shape = torch.broadcast_shapes(tf.shape, tt.shape)
    if len(shape) not in (1, 2) or shape[-1] != 3:
        raise ValueError(f"positions must be (3,) or (N, 3), got {tuple(shape)}")
    tf, pf = _period(tf, shape)
    tt, pt = _period(tt, shape)
    rows = 1 if len(shape) == 1 else shape[0]
    out = torch.empty(rows, dtype=torch.float64, device=tf.device)
    P = lambda t: _lib.ptr(t, _lib._d)  # noqa: E731
    _lib.check(_lib.lib().asp_wrapped_distance(
        P(tf), pf, P(tt), pt, rows, float(box_width), int(bool(do_squared_distance)), P(out),
        tf.device.index or 0, torch.cuda.current_stream(tf.device).cuda_stream))
    if len(shape) == 1:
        return np.float64(out.item()) if (nf and nt) else out[0]
    return out.cpu().numpy() if (nf and nt) else out


def make_periodic(positions, box_width, origin_is_centre: bool = False):
    """Wrap every coordinate outside the box back by one box width, IN PLACE
    (reference :36-43)."""
    if _has_units(positions):  # the reference's body on a unyt array: values, same unit
        vals = positions.value
        make_periodic(vals, _in(box_width, positions.units), origin_is_centre)
        return
    res = _run(_lib.ASP_PB_WRAP, positions, None, box_width, origin_is_centre)
    if isinstance(res, np.ndarray):
        positions[...] = res
    else:
        positions.copy_(res)


def calculate_periodic(start_positions, box_width, origin_is_centre: bool = False):
    """A wrapped copy (reference :45-48; unyt overload :49-51: in the positions' unit)."""
    if _has_units(start_positions):
        u = start_positions.units
        return _wrap(start_positions, calculate_periodic(start_positions.value,
                                                         _in(box_width, u), origin_is_centre), u)
    return _run(_lib.ASP_PB_WRAP, start_positions, None, box_width, origin_is_centre)


def shift_origin(start_positions, new_origin, box_width, origin_is_centre: bool = False):
    """Positions relative to ``new_origin``, wrapped (reference :54-57; unyt overload
    :58-60: everything in the new origin's unit)."""
    if _has_units(start_positions):
        u = new_origin.units
        return _wrap(start_positions, shift_origin(start_positions.to(u).value, new_origin.value,
                                                   _in(box_width, u), origin_is_centre), u)
    return _run(_lib.ASP_PB_SHIFT_ORIGIN, start_positions, new_origin, box_width,
                origin_is_centre)


def shift_centre(start_positions, new_centre, box_width, origin_is_centre: bool = False):
    """Positions moved so that ``new_centre`` is the box centre, wrapped (reference
    :63-69; unyt overload :70-72: everything in the new centre's unit)."""
    if _has_units(start_positions):
        u = new_centre.units
        return _wrap(start_positions, shift_centre(start_positions.to(u).value, new_centre.value,
                                                   _in(box_width, u), origin_is_centre), u)
    return _run(_lib.ASP_PB_SHIFT_CENTRE, start_positions, new_centre, box_width,
                origin_is_centre)
