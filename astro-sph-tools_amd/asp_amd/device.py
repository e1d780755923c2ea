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
    from .tools.projections._kernels import native_kernel_id
    return native_kernel_id(kernel)


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
              out1=None, stream=None, deterministic: bool = False, rows=None):
    """Project device-resident particles; returns ``(out0, out1)`` (out1 None for one map).

    ``extent = (u_min, u_max, v_min, v_max)``; images are (nx, ny) float32 tensors on the
    particles' device.  ``ratio`` turns (sum a0 W, sum a1 W) into their ratio in out0.
    ``rows = (row_lo, row_hi)``: only those image rows (asp_project2d_rows, the row-slab
    decomposition): outputs are (row_hi - row_lo, ny), each pixel the whole image's.
    """
    import torch
    dev = u.device
    n = u.shape[0]
    for t, name in ((u, "u"), (v, "v"), (h, "h"), (a0, "a0")):
        _check(t, name, n, dev)
    if a1 is not None:
        _check(a1, "a1", n, dev)
    nx, ny = int(image_size[0]), int(image_size[1])
    r0, r1 = (0, nx) if rows is None else (int(rows[0]), int(rows[1]))
    if not 0 <= r0 < r1 <= nx:
        raise ValueError(f"rows must satisfy 0 <= row_lo < row_hi <= nx, got {(r0, r1)}")
    mx = r1 - r0  # rows written
    if out0 is None:
        out0 = torch.empty((mx, ny), dtype=torch.float32, device=dev)
    if a1 is not None and out1 is None:
        out1 = torch.empty((mx, ny), dtype=torch.float32, device=dev)
    for t in (out0, out1):
        if t is not None and (t.dtype != torch.float32 or t.device != dev or not t.is_contiguous()
                              or t.numel() != mx * ny):
            raise ValueError("outputs must be contiguous float32 (rows, ny) tensors on the device")
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
    if rows is None:
        _lib.check(_lib.lib().asp_project2d(
            P(u), P(v), P(h), P(a0), P(a1), n, x_min, x_max, y_min, y_max, nx, ny,
            int(chunk_size), kernel_id(kernel), flags, P(out0), P(out1), dev.index or 0, stream))
    else:
        _lib.check(_lib.lib().asp_project2d_rows(
            P(u), P(v), P(h), P(a0), P(a1), n, x_min, x_max, y_min, y_max, nx, ny,
            int(chunk_size), r0, r1, kernel_id(kernel), flags, P(out0), P(out1), dev.index or 0,
            stream))
    return out0, (out1 if a1 is not None else None)


def project2d_props(u, v, h, props, *, image_size, extent, chunk_size: int = 64,
                    kernel="cubic", accumulate: bool = False, outs=None, stream=None,
                    mass=None, density=None, ratio: bool = False):
    """asp_project2d_props: one map per property of ``props`` (1..6 device float32 arrays)
    from ONE binning of the particles -- the same neighbour sets, the counting and
    scattering done once.  Returns the list of (nx, ny) float32 maps.

    ``mass`` (and ``density``): the SPH-weighted maps of asp_project2d_sph,
    sum_j (m_j / rho_j) A_j W (``density`` None: sum_j m_j A_j W); ``ratio`` (two
    properties): out0 = the weighted mean of props[0] over props[1]'s weights."""
    import torch
    dev = u.device
    n = u.shape[0]
    k = len(props)
    if not 1 <= k <= 6:
        raise ValueError("props: 1 .. 6 arrays")
    for t, name in ((u, "u"), (v, "v"), (h, "h")):
        _check(t, name, n, dev)
    for j, a in enumerate(props):
        _check(a, f"props[{j}]", n, dev)
    if density is not None and mass is None:
        raise ValueError("density needs mass (the weights are m / rho)")
    for t, name in ((mass, "mass"), (density, "density")):
        if t is not None:
            _check(t, name, n, dev)
    if ratio and k != 2:
        raise ValueError("ratio needs exactly two properties")
    nx, ny = int(image_size[0]), int(image_size[1])
    if outs is None:
        outs = [torch.empty((nx, ny), dtype=torch.float32, device=dev) for _ in range(k)]
    if len(outs) != k:
        raise ValueError("one output per property")
    for t in outs:
        if t.dtype != torch.float32 or t.device != dev or not t.is_contiguous() or \
                t.numel() != nx * ny:
            raise ValueError("outputs must be contiguous float32 (nx, ny) tensors on the device")
    flags = _lib.ASP_F_DEVICE_PTRS | (_lib.ASP_F_ACCUMULATE if accumulate else 0) | \
        (_lib.ASP_F_RATIO if ratio else 0)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    P = _lib.ptr
    pa = (_lib._f * k)(*[P(a) for a in props])
    po = (_lib._f * k)(*[P(o) for o in outs])
    x_min, x_max, y_min, y_max = (float(e) for e in extent)
    tail = (n, x_min, x_max, y_min, y_max, nx, ny, int(chunk_size), kernel_id(kernel), flags, po,
            dev.index or 0, stream)
    if mass is not None:
        _lib.check(_lib.lib().asp_project2d_sph(
            P(u), P(v), P(h), P(mass), P(density) if density is not None else None, pa, k,
            *tail))
    else:
        _lib.check(_lib.lib().asp_project2d_props(P(u), P(v), P(h), pa, k, *tail))
    return outs


def project2d_props_f64(positions, h, props, *, projection_axis=2, image_size, extent,
                        chunk_size: int = 64, kernel="cubic", device: int = 0, mass=None,
                        density=None, ratio: bool = False):
    """asp_project2d_props_f64 on the reader's float64 arrays (host NumPy arrays or float64
    device tensors; host arrays are copied to the device): the maps of every property from
    one binning, every decision the reference's fp64 test.  Returns float32 device maps.
    ``mass`` / ``density`` / ``ratio``: as :func:`project2d_props` (asp_project2d_sph_f64;
    the weights m / rho are formed in fp64 from the reader's values)."""
    import numpy as np
    import torch
    from ._axes import axis_index
    if isinstance(projection_axis, tuple):  # (pixel axis, cull axis): reference_axes()
        axis = int(projection_axis[0])
        if int(projection_axis[1]) != axis:
            axis |= (int(projection_axis[1]) + 1) << 4  # ASP_AXIS_CULL
    else:
        axis = axis_index(projection_axis)
    k = len(props)
    if not 1 <= k <= 6:
        raise ValueError("props: 1 .. 6 arrays")
    dev = positions.device if hasattr(positions, "is_cuda") and positions.is_cuda \
        else torch.device("cuda", device)

    def on_dev(a, shape):
        t = a if hasattr(a, "is_cuda") and a.is_cuda else torch.from_numpy(
            np.ascontiguousarray(np.asarray(a), dtype=np.float64))
        t = t.to(device=dev, dtype=torch.float64).contiguous()
        if tuple(t.shape) != shape:
            raise ValueError(f"array of shape {tuple(t.shape)}, expected {shape}")
        return t

    n = int(positions.shape[0])
    pos = on_dev(positions, (n, 3))
    hh = on_dev(np.asarray(h).reshape(-1) if not hasattr(h, "is_cuda") else h.reshape(-1), (n,))
    pr = [on_dev(np.asarray(a).reshape(-1) if not hasattr(a, "is_cuda") else a.reshape(-1), (n,))
          for a in props]
    if density is not None and mass is None:
        raise ValueError("density needs mass (the weights are m / rho)")
    if ratio and k != 2:
        raise ValueError("ratio needs exactly two properties")
    flat = lambda a: np.asarray(a).reshape(-1) if not hasattr(a, "is_cuda") else a.reshape(-1)  # noqa: E731
    wm = None if mass is None else on_dev(flat(mass), (n,))
    wr = None if density is None else on_dev(flat(density), (n,))
    nx, ny = int(image_size[0]), int(image_size[1])
    outs = [torch.empty((nx, ny), dtype=torch.float32, device=dev) for _ in range(k)]
    P = _lib.ptr
    pa = (_lib._d * k)(*[P(a, _lib._d) for a in pr])
    po = (_lib._f * k)(*[P(o) for o in outs])
    x_min, x_max, y_min, y_max = (float(e) for e in extent)
    flags = _lib.ASP_F_DEVICE_PTRS | (_lib.ASP_F_RATIO if ratio else 0)
    tail = (n, axis, x_min, x_max, y_min, y_max, nx, ny, int(chunk_size), kernel_id(kernel), flags,
            po, dev.index or 0, torch.cuda.current_stream(dev).cuda_stream)
    if wm is not None:
        _lib.check(_lib.lib().asp_project2d_sph_f64(
            P(pos, _lib._d), P(hh, _lib._d), P(wm, _lib._d),
            P(wr, _lib._d) if wr is not None else None, pa, k, *tail))
    else:
        _lib.check(_lib.lib().asp_project2d_props_f64(P(pos, _lib._d), P(hh, _lib._d), pa, k, *tail))
    return outs


def _f64_arg(a, name, n, shape_tail=()):
    """A float64 input of create_image: a contiguous host array (NumPy / unyt) or a
    float64 device tensor; returns (object keeping it alive, ctypes pointer, on_device)."""
    import numpy as np
    if hasattr(a, "is_cuda") and a.is_cuda:
        import torch
        if a.dtype != torch.float64:
            raise ValueError(f"{name} must be float64")
        a = a.contiguous()
        if tuple(a.shape) != (n,) + shape_tail:
            raise ValueError(f"{name} has shape {tuple(a.shape)}, expected {(n,) + shape_tail}")
        return a, _lib.ptr(a, _lib._d), True
    x = np.ascontiguousarray(np.asarray(a), dtype=np.float64)
    if shape_tail == () and x.ndim != 1:
        x = x.reshape(-1)
    if x.shape != (n,) + shape_tail:
        raise ValueError(f"{name} has shape {x.shape}, expected {(n,) + shape_tail}")
    return x, _lib.ptr(x, _lib._d), False


def project2d_f64(positions, h, a0, a1=None, *, projection_axis=2, image_size, extent,
                  chunk_size: int = 64, kernel="cubic", ratio: bool = False,
                  accumulate: bool = False, out0=None, out1=None, device: int = 0,
                  stream=None, deterministic: bool = False, device_out: bool = False):
    """asp_project2d_f64: the reader's float64 arrays (positions (N, 3), h, a0[, a1]) --
    host NumPy arrays or float64 device tensors -- projected with the reference's fp64
    decisions on those values.  ``projection_axis``: an axis (int 0/1/2, enum, "x") or a
    (pixel axis, cull axis) pair (asp_amd._axes.reference_axes).  Returns float32 maps:
    device tensors for device inputs or ``device_out`` (host inputs staged through pinned
    buffers, maps left on ``device`` -- e.g. for an RCCL sum), else NumPy arrays."""
    import numpy as np
    import torch
    from ._axes import axis_index
    if isinstance(projection_axis, tuple):  # (pixel axis, cull axis): reference_axes()
        axis = int(projection_axis[0])
        if int(projection_axis[1]) != axis:
            axis |= (int(projection_axis[1]) + 1) << 4  # ASP_AXIS_CULL
    else:
        axis = axis_index(projection_axis)
    n = int(positions.shape[0])
    keep = []
    pos, ppos, on_dev = _f64_arg(positions, "positions", n, (3,))
    keep.append(pos)
    ptrs = [ppos]
    for arr, name in ((h, "smoothing_lengths"), (a0, "a0"), (a1, "a1")):
        if arr is None:
            ptrs.append(None)
            continue
        x, px, d = _f64_arg(arr, name, n)
        if d != on_dev:
            raise ValueError("positions and fields must all be host arrays or all device tensors")
        keep.append(x)
        ptrs.append(px)
    nx, ny = int(image_size[0]), int(image_size[1])
    nout = 1 if a1 is None else 2
    flags = (_lib.ASP_F_RATIO if ratio else 0) | (_lib.ASP_F_ACCUMULATE if accumulate else 0) | \
        (_lib.ASP_F_DETERMINISTIC if deterministic else 0)
    if on_dev:
        dev = pos.device
        device = dev.index or 0
        flags |= _lib.ASP_F_DEVICE_PTRS
        if out0 is None:
            out0 = torch.empty((nx, ny), dtype=torch.float32, device=dev)
        if nout == 2 and out1 is None:
            out1 = torch.empty((nx, ny), dtype=torch.float32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
    elif device_out:
        _lib.require_gpu(device)
        flags |= _lib.ASP_F_DEVICE_OUTPUTS
        dev = torch.device("cuda", device)
        if out0 is None:
            out0 = (torch.zeros if accumulate else torch.empty)((nx, ny), dtype=torch.float32, device=dev)
        if nout == 2 and out1 is None:
            out1 = (torch.zeros if accumulate else torch.empty)((nx, ny), dtype=torch.float32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
    else:
        _lib.require_gpu(device)
        if out0 is None:
            out0 = np.zeros((nx, ny), dtype=np.float32)
        if nout == 2 and out1 is None:
            out1 = np.zeros((nx, ny), dtype=np.float32)
    for t in (out0, out1):
        if t is not None and (t.dtype not in (np.float32, torch.float32) or int(np.prod(t.shape)) != nx * ny):
            raise ValueError("outputs must be float32 (nx, ny) arrays")
    x_min, x_max, y_min, y_max = (float(np.asarray(e)) for e in extent)
    _lib.check(_lib.lib().asp_project2d_f64(
        ptrs[0], ptrs[1], ptrs[2], ptrs[3], n, axis, x_min, x_max, y_min, y_max, nx, ny,
        int(chunk_size), kernel_id(kernel), flags, _lib.ptr(out0), _lib.ptr(out1),
        int(device), stream))
    return out0, (out1 if nout == 2 else None)


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
