"""``create_cube`` -- the 512^3 volumetric deposit (BASELINE configs[4]).

The reference has no volumetric renderer; this is the build's natural extension of
``create_image`` (/root/reference/src/astro_sph_tools/tools/projections/_projector.py:75-120,
_pixel_calculations.pyx:9-36) to voxels, with the same argument conventions:

* voxel (i, j, k) samples the corner ``(x_min + i*dx, y_min + j*dy, z_min + k*dz)``,
  ``dx = (x_max - x_min)/Nx``, ``dy = (y_max - y_min)/Ny``, ``dz = (z_max - z_min)/Nz``
  (each axis its own pitch: the 2-D y-pitch quirk S2 is not carried over);
* neighbours are the particles with ``r^2 < (2h)^2``, r the 3-D distance, decided in
  fp64 (bit-exact sets vs the CPU restatement ``oracle/asp_oracle.c:oracle_project3d``);
* the value is ``sum_p A_p W(r_p, h_p)`` with the same kernel plugins; with ``A = m``
  the cube is the SPH density field.

Returns a fresh ``(Nx, Ny, Nz)`` array (``float64`` by default, computed in fp32 terms
with fp64 accumulation on the GPU).  ``planes=(k_lo, k_hi)`` returns only those z planes.
"""
from __future__ import annotations

import numpy as np

from ... import _lib
from ._kernels import native_kernel_id, quartic_spline_kernel


def create_cube(positions: np.ndarray, smoothing_lengths: np.ndarray,
                particle_properties: np.ndarray, cube_size: tuple, x_min: float, x_max: float,
                y_min: float, y_max: float, z_min: float, z_max: float,
                kernel_func=quartic_spline_kernel, *, planes=None, device: int = 0,
                dtype=np.float64) -> np.ndarray:
    """Deposit particle property A onto an (Nx, Ny, Nz) voxel grid."""
    pos = np.asarray(positions)
    if pos.ndim != 2 or pos.shape[1] != 3:
        raise ValueError(f"positions must have shape (N, 3), got {pos.shape}")
    n = pos.shape[0]
    h = np.asarray(smoothing_lengths).reshape(-1)
    A = np.asarray(particle_properties).reshape(-1)
    if h.shape[0] != n or A.shape[0] != n:
        raise ValueError(f"positions ({n}), smoothing_lengths ({h.shape[0]}) and "
                         f"particle_properties ({A.shape[0]}) differ in length")
    kid = native_kernel_id(kernel_func)
    nx, ny, nz = (int(c) for c in cube_size)
    k_lo, k_hi = (0, nz) if planes is None else (int(planes[0]), int(planes[1]))
    if min(nx, ny, nz) <= 0 or k_hi <= k_lo:
        return np.zeros((max(nx, 0), max(ny, 0), max(k_hi - k_lo, 0)), dtype=dtype)
    _lib.require_gpu(device)
    f32 = np.float32
    cols = [np.ascontiguousarray(pos[:, c], dtype=f32) for c in range(3)]
    h32, A32 = np.ascontiguousarray(h, dtype=f32), np.ascontiguousarray(A, dtype=f32)
    out = np.zeros((nx, ny, k_hi - k_lo), dtype=np.float32)
    P = _lib.ptr
    ext = [float(np.asarray(e)) for e in (x_min, x_max, y_min, y_max, z_min, z_max)]
    _lib.check(_lib.lib().asp_project3d(P(cols[0]), P(cols[1]), P(cols[2]), P(h32), P(A32), n,
                                        *ext, nx, ny, nz, k_lo, k_hi, kid, 0, P(out), device,
                                        None))
    return out.astype(dtype, copy=False)
