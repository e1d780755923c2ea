"""Device-resident entry point: project float32 SoA torch tensors already in HBM.

This is the path ``bench.py`` and the multi-GPU driver use (no host round trip).  torch
only provides the device memory and the stream; all compute is libasp_hip.so.
"""
from __future__ import annotations

from . import _lib

_KERNEL_NAMES = {"cubic": _lib.ASP_KERNEL_CUBIC_SPLINE, "quartic_spline_kernel": 0,
                 "cubic_spline": 0, "wendland_c2": _lib.ASP_KERNEL_WENDLAND_C2,
                 "indicator": _lib.ASP_KERNEL_INDICATOR}


def kernel_id(kernel) -> int:
    if isinstance(kernel, int):
        return kernel
    if isinstance(kernel, str):
        return _KERNEL_NAMES[kernel]
    from .tools.projections._kernels import kernel_id_of
    return kernel_id_of(kernel)


def _check(t, name, n=None, device=None):
    import torch
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor")
    if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.dim() != 1:
        raise ValueError(f"{name} must be a contiguous 1-D float32 device tensor")
    if n is not None and t.shape[0] != n:
        raise ValueError(f"{name} has {t.shape[0]} elements, expected {n}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")


def project2d(u, v, h, a0, a1=None, *, image_size, extent, chunk_size: int = 64,
              kernel="cubic", ratio: bool = False, accumulate: bool = False, out0=None,
              out1=None, stream=None, deterministic: bool = False):
    """Project device-resident particles; returns ``(out0, out1)`` (out1 None for one map).

    ``extent = (u_min, u_max, v_min, v_max)``; images are (nx, ny) float32 tensors on the
    particles' device.  ``ratio`` turns (sum a0 W, sum a1 W) into their ratio in out0.
    """
    import torch
    dev = u.device
    n = u.shape[0]
    for t, name in ((u, "u"), (v, "v"), (h, "h"), (a0, "a0")):
        _check(t, name, n, dev)
    if a1 is not None:
        _check(a1, "a1", n, dev)
    nx, ny = int(image_size[0]), int(image_size[1])
    if out0 is None:
        out0 = torch.empty((nx, ny), dtype=torch.float32, device=dev)
    if a1 is not None and out1 is None:
        out1 = torch.empty((nx, ny), dtype=torch.float32, device=dev)
    for t in (out0, out1):
        if t is not None and (t.dtype != torch.float32 or t.device != dev or not t.is_contiguous()
                              or t.numel() != nx * ny):
            raise ValueError("outputs must be contiguous float32 (nx, ny) tensors on the device")
    flags = _lib.ASP_F_DEVICE_PTRS
    if ratio:
        flags |= _lib.ASP_F_RATIO
    if accumulate:
        flags |= _lib.ASP_F_ACCUMULATE
    if deterministic:
        flags |= _lib.ASP_F_DETERMINISTIC
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    P = _lib.ptr
    x_min, x_max, y_min, y_max = (float(e) for e in extent)
    _lib.check(_lib.lib().asp_project2d(
        P(u), P(v), P(h), P(a0), P(a1), n, x_min, x_max, y_min, y_max, nx, ny, int(chunk_size),
        kernel_id(kernel), flags, P(out0), P(out1), dev.index or 0, stream))
    return out0, (out1 if a1 is not None else None)


def project3d(x, y, z, h, a, *, cube_size, extent, kernel="cubic", planes=None,
              accumulate: bool = False, out=None, stream=None):
    """Deposit device-resident particles into a voxel cube (asp_project3d).

    ``extent = (x_min, x_max, y_min, y_max, z_min, z_max)``; ``planes = (k_lo, k_hi)``
    restricts the output to those z planes (default: all).  Returns the
    (nx, ny, k_hi - k_lo) float32 tensor on the particles' device.
    """
    import torch
    dev = x.device
    n = x.shape[0]
    for t, name in ((x, "x"), (y, "y"), (z, "z"), (h, "h"), (a, "a")):
        _check(t, name, n, dev)
    nx, ny, nz = (int(c) for c in cube_size)
    k_lo, k_hi = (0, nz) if planes is None else (int(planes[0]), int(planes[1]))
    shape = (nx, ny, max(0, k_hi - k_lo))
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=dev)
    if (out.dtype != torch.float32 or out.device != dev or not out.is_contiguous()
            or out.numel() != shape[0] * shape[1] * shape[2]):
        raise ValueError("out must be a contiguous float32 (nx, ny, k_hi - k_lo) tensor on the device")
    flags = _lib.ASP_F_DEVICE_PTRS | (_lib.ASP_F_ACCUMULATE if accumulate else 0)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    P = _lib.ptr
    e = [float(v) for v in extent]
    _lib.check(_lib.lib().asp_project3d(P(x), P(y), P(z), P(h), P(a), n, *e, nx, ny, nz, k_lo,
                                        k_hi, kernel_id(kernel), flags, P(out), dev.index or 0,
                                        stream))
    return out


def stats(device: int = 0):
    """Counters of the last projection on ``device`` (records, work items, wide, ...)."""
    return _lib.last_stats(device)
