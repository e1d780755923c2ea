"""Smoothing lengths from the k-th nearest neighbour, on the GPU.

Replaces the scipy KDTree query of the reference's SWIFT reader
(/root/reference/src/astro_sph_tools/io/SWIFT/_SnapshotSWIFT.py:62-83), which gives dark
matter particles ``h = tree.query(positions, k=32)[0][:, 31]``: the distance to the 32nd
nearest particle, the particle itself counted.  Same distance arithmetic (fp64
Euclidean), so the values are bit-identical (asp_knn_smoothing_lengths, csrc/asp_knn.hip).
"""
from __future__ import annotations

import numpy as np

from . import _lib


def knn_smoothing_lengths(positions, k: int = 32, *, device: int = 0, stream=None):
    """Distance from every particle to its k-th nearest neighbour (itself included).

    ``positions``: (N, 3) float64 -- a NumPy (or unyt) host array, returning a NumPy
    array, or a float64 torch tensor on the GPU, returning a tensor there.  ``inf`` where
    fewer than k particles exist (as scipy reports a missing neighbour).
    """
    import torch
    k = int(k)
    if hasattr(positions, "is_cuda") and positions.is_cuda:
        pos = positions.contiguous()
        if pos.dtype != torch.float64 or pos.dim() != 2 or pos.shape[1] != 3:
            raise ValueError("positions must be an (N, 3) float64 tensor")
        h = torch.empty(pos.shape[0], dtype=torch.float64, device=pos.device)
        if stream is None:
            stream = torch.cuda.current_stream(pos.device).cuda_stream
        _lib.check(_lib.lib().asp_knn_smoothing_lengths(
            _lib.ptr(pos, _lib._d), pos.shape[0], k, _lib.ptr(h, _lib._d), _lib.ASP_F_DEVICE_PTRS,
            pos.device.index or 0, stream))
        return h
    pos = np.ascontiguousarray(np.asarray(positions), dtype=np.float64)
    if pos.ndim != 2 or pos.shape[1] != 3:
        raise ValueError(f"positions must have shape (N, 3), got {pos.shape}")
    _lib.require_gpu(device)
    h = np.empty(pos.shape[0], dtype=np.float64)
    _lib.check(_lib.lib().asp_knn_smoothing_lengths(_lib.ptr(pos, _lib._d), pos.shape[0], k,
                                                    _lib.ptr(h, _lib._d), 0, device, None))
    return h
