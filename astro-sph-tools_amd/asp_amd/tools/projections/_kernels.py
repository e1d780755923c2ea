"""SPH kernels, the ``kernel_func`` plugin point of ``create_image``.

Mirrors ``quartic_spline_kernel`` (/root/reference/src/astro_sph_tools/tools/projections/
_kernels.pyx:9-20): ``W(r, h)`` over two 1-D float64 arrays, returning a new float64
array, evaluated ON THE GPU (asp_kernel_eval).  Despite its name the reference kernel is
the M4 cubic spline with support 2h and 3-D normalisation 1/(pi h^3); that is kept.

The kernel objects also carry the C-ABI kernel id, which is how ``create_image``
recognises them and runs the whole projection natively.  Any other callable (the
reference's own compiled kernel included) goes through the plugin path: neighbour pairs
from the device, the callable evaluated on the host (_plugin.py).
"""
from __future__ import annotations

import numpy as np

from ... import _lib


class SPHKernel:
    """A device-evaluable SPH kernel: callable like the reference's kernel_func."""

    def __init__(self, name: str, kernel_id: int, doc: str):
        self.__name__ = name
        self.kernel_id = kernel_id
        self.__doc__ = doc

    def __repr__(self):
        return f"<asp_amd SPH kernel {self.__name__} (id {self.kernel_id})>"

    def __call__(self, r, h, *, device: int = 0):
        r = np.asarray(r)
        h = np.asarray(h)
        # The reference's typed memoryview signature (double[:] r, double[:] h) raises
        # ValueError for any other buffer dtype or dimensionality.
        for a in (r, h):
            if a.dtype != np.float64:
                raise ValueError(f"Buffer dtype mismatch, expected 'double' but got '{a.dtype}'")
            if a.ndim != 1:
                raise ValueError(f"Buffer has wrong number of dimensions (expected 1, got {a.ndim})")
        if h.shape[0] < r.shape[0]:
            raise ValueError("h is shorter than r")
        r = np.ascontiguousarray(r)
        h = np.ascontiguousarray(h[: r.shape[0]])
        w = np.zeros(r.shape[0], dtype=np.float64)
        if r.shape[0] == 0:
            return w
        _lib.require_gpu(device)
        _lib.check(_lib.lib().asp_kernel_eval(self.kernel_id, _lib.ptr(r, _lib._d),
                                              _lib.ptr(h, _lib._d), _lib.ptr(w, _lib._d),
                                              r.shape[0], 0, device, None))
        return w


quartic_spline_kernel = SPHKernel(
    "quartic_spline_kernel", _lib.ASP_KERNEL_CUBIC_SPLINE,
    "M4 cubic spline, support 2h: W = (1 - 1.5q^2 + 0.75q^3)/(pi h^3) for q < 1, "
    "0.25 (2-q)^3/(pi h^3) for 1 <= q < 2, else 0 (q = r/h).  _kernels.pyx:9-20.")

cubic_spline_kernel = quartic_spline_kernel

wendland_c2_kernel = SPHKernel(
    "wendland_c2_kernel", _lib.ASP_KERNEL_WENDLAND_C2,
    "Wendland C2, support 2h, 3-D normalisation: W = 21/(16 pi h^3) (1-q/2)^4 (1+2q), "
    "q = r/h < 2.  Build-defined (SURVEY.md §8(a)).")

indicator_kernel = SPHKernel(
    "indicator_kernel", _lib.ASP_KERNEL_INDICATOR,
    "W = 1 for every pair inside 2h: create_image with this kernel and A = 1 counts the "
    "neighbours of every pixel (neighbour-set verification).")

KERNELS = {k.kernel_id: k for k in (quartic_spline_kernel, wendland_c2_kernel, indicator_kernel)}


def kernel_id_of(kernel_func):
    """The C-ABI kernel id of one of this package's kernels, or None for any other
    callable (it then runs through the plugin path, _plugin.project_callable)."""
    kid = getattr(kernel_func, "kernel_id", None)
    if isinstance(kernel_func, SPHKernel) and kid in KERNELS:
        return kid
    if not callable(kernel_func):
        raise TypeError(f"kernel_func {kernel_func!r} is not callable")
    return None


def native_kernel_id(kernel_func) -> int:
    """kernel_id_of for the paths with no plugin (device arrays, cubes, periodic maps)."""
    kid = kernel_id_of(kernel_func)
    if kid is None:
        raise TypeError(f"kernel_func {kernel_func!r} cannot run on the GPU here; use "
                        "quartic_spline_kernel, wendland_c2_kernel or indicator_kernel "
                        "(create_image accepts any callable)")
    return kid
