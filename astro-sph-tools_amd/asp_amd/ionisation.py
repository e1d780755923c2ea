"""Ionisation tables on the GPU.

Mirrors the reference's ``IonisationTableBase`` (/root/reference/src/astro_sph_tools/
data_structures/_IonisationTable.py:30-69): a table over N input axes interpolated
linearly (scipy's RegularGridInterpolator with ``bounds_error=False``,
``fill_value=-inf``), ``__call__(gas_state)`` and ``evaluate_at_redshift(gas_state, z)``.
The HM01 tables (io/ionisation_tables/_HM01.py:61-92) are 3-D over
(log10 n_H, log10 T, redshift) with the redshift axis at index 2 and take the specialised
``asp_table_interp3`` (LDS slab of the two redshift layers); any other number of axes
(1 .. 6) takes ``asp_table_interp``.  Both are bit-identical to scipy 1.15's linear
evaluation, including its choice of arithmetic order (the Cython 2-D fast path for a
writeable native-float64 2-D table, ``_evaluate_linear`` otherwise).  Reading the HDF5
files stays with the caller (h5py is the reference's reader); pass the arrays.

:func:`ion_masses` forms what an ion column map projects: ``m * X_element * f_ion``
per particle, on the device.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def _dev(a):
    import torch
    if hasattr(a, "is_cuda") and a.is_cuda:
        return a.to(torch.float64).contiguous(), False
    _lib.require_gpu(0)
    a = np.ascontiguousarray(np.asarray(a), dtype=np.float64)
    if not a.flags.writeable:  # torch.from_numpy wants a writeable buffer
        a = a.copy()
    return torch.from_numpy(a).cuda(), True


class IonisationTable:
    """``IonisationTable(table, axis0, axis1, axis2, redshift_input_index=2)``."""

    def __init__(self, table, *table_positions, redshift_input_index: int = -1):
        n = len(table_positions)
        if n == 0:
            raise IndexError("No input dimensions were specified for table interpolation construction.")
        t = np.asarray(table, dtype=np.float64)
        if t.ndim != n:
            raise IndexError(f"Interpolation table has {t.ndim} dimensions but {n} arrays were "
                             "used to specify the table positions.")
        if n > 6:
            raise NotImplementedError("the device interpolator handles 1 .. 6 table axes")
        for k, g in enumerate(table_positions):
            g = np.asarray(g, dtype=np.float64)
            if g.ndim != 1 or g.size != t.shape[k] or g.size < 2 or not np.all(np.diff(g) > 0):
                raise ValueError(f"table axis {k} must be strictly ascending with "
                                 f"{t.shape[k]} >= 2 points")
        self._n = n
        # scipy 1.15 takes its Cython 2-D path (value * w0 * w1) for a writeable
        # native-float64 2-D table; every other table goes through _evaluate_linear
        raw = table if hasattr(table, "dtype") else np.asarray(table)
        if not np.issubdtype(raw.dtype, np.inexact):
            raw = raw.astype(float)  # RegularGridInterpolator._check_values: a fresh array
        self._order = int(n == 2 and raw.dtype == np.float64 and raw.dtype.isnative
                          and bool(raw.flags.writeable))
        # the reference's index arithmetic for a negative redshift index, kept as is
        self._z = redshift_input_index if redshift_input_index >= 0 else n - redshift_input_index
        self._table, _ = _dev(t)
        self._axes = [_dev(g)[0] for g in table_positions]
        self._table_host = t

    def _run(self, pts, ncol, z, mode=0, a0=None, a1=None):
        import torch
        P, host = _dev(pts)
        if P.dim() != 2 or P.shape[1] != ncol:
            raise ValueError(f"gas_state must have shape (N, {ncol})")
        if ncol == self._n - 1 and not 0 <= self._z < self._n:
            # the reference's column assignment fails the same way (:56-57)
            raise IndexError(f"redshift input index {self._z} is out of bounds for "
                             f"{self._n} table dimensions")
        out = torch.empty(P.shape[0], dtype=torch.float64, device=P.device)
        d = lambda t: _lib.ptr(t, _lib._d)  # noqa: E731
        st = torch.cuda.current_stream(P.device).cuda_stream
        dev = P.device.index or 0
        if self._n == 3:
            _lib.check(_lib.lib().asp_table_interp3(
                d(self._table), *self._table.shape, *(d(g) for g in self._axes), d(P), ncol,
                self._z if ncol == 2 else 0, float(z), P.shape[0], -np.inf, mode,
                d(a0), d(a1), d(out), dev, st))
        else:
            import ctypes as C
            shape = (C.c_int32 * self._n)(*self._table.shape)
            axes = (C.c_void_p * self._n)(*(g.data_ptr() for g in self._axes))
            _lib.check(_lib.lib().asp_table_interp(
                d(self._table), self._n, shape, axes, d(P), ncol,
                self._z if ncol == self._n - 1 else 0, float(z), P.shape[0], -np.inf, mode,
                self._order, d(a0), d(a1), d(out), dev, st))
        return out.cpu().numpy() if host else out

    def __call__(self, gas_state):
        return self._run(gas_state, self._n, 0.0)

    def evaluate_at_redshift(self, gas_state, redshift: float):
        return self._run(gas_state, self._n - 1, redshift)

    @property
    def number_of_input_dimensions(self) -> int:
        return self._n

    @property
    def ionisation_fraction_table(self) -> np.ndarray:
        return self._table_host.copy()

    def get_table_dimension(self, dimension: int) -> np.ndarray:
        return self._axes[dimension].cpu().numpy()


def ion_masses(table: IonisationTable, masses, element_mass_fractions, log10_nH, log10_T,
               redshift: float, *, table_is_log10: bool):
    """Per-particle ion mass ``m * X * f_ion(log10 n_H, log10 T, z)`` on the device
    (``f_ion = 10^value`` when the table holds log10 fractions).  The result is the
    ``particle_properties`` of an ion column map."""
    import torch
    m, host = _dev(masses)
    X, _ = _dev(element_mass_fractions)
    state = torch.stack([_dev(log10_nH)[0], _dev(log10_T)[0]], dim=1).contiguous()
    out = table._run(state, 2, redshift, 2 if table_is_log10 else 1, m, X)
    return out.cpu().numpy() if (host and hasattr(out, "is_cuda")) else out
