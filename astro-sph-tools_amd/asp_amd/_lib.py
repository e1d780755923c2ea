"""ctypes binding of libasp_hip.so (the C-ABI in include/asp.h).

The product path has no CPU fallback: if the HIP library is missing this module raises
at import-use time, and if no GPU is visible every projection call raises RuntimeError.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)  # astro-sph-tools_amd/
LIB_PATH = os.environ.get("ASP_LIB", os.path.join(ROOT, "lib", "libasp_hip.so"))

ASP_KERNEL_CUBIC_SPLINE = 0
ASP_KERNEL_WENDLAND_C2 = 1
ASP_KERNEL_INDICATOR = 2

ASP_F_DEVICE_PTRS = 0x1
ASP_F_RATIO = 0x2
ASP_F_ACCUMULATE = 0x4
ASP_F_DETERMINISTIC = 0x8
ASP_F_DEVICE_OUTPUTS = 0x10

ASP_PB_WRAP = 0x1
ASP_PB_SHIFT_ORIGIN = 0x2
ASP_PB_SHIFT_CENTRE = 0x4
ASP_PB_ORIGIN_IS_CENTRE = 0x8
ASP_PB_IMAGES = 0x10
ASP_PB_DISPLACEMENT = 0x20

ASP_OK = 0
ASP_ERR_INVALID = -1
ASP_ERR_HIP = -2
ASP_ERR_NOMEM = -3
ASP_ERR_UNSUPPORTED = -4

# Every symbol include/asp.h declares (tests check the library exports all of them).
EXPORTS = ("asp_version", "asp_last_error", "asp_device_count", "asp_project2d",
           "asp_project2d_rows", "asp_project2d_props", "asp_project2d_props_f64",
           "asp_project2d_sph", "asp_project2d_sph_f64",
           "asp_project2d_f64", "asp_pairs_begin", "asp_pairs_emit", "asp_pairs_end",
           "asp_project3d", "asp_kernel_eval", "asp_chunk_ranges", "asp_pixel_neighbours", "asp_ratio",
           "asp_profile", "asp_profile_stages", "asp_profile_read", "asp_last_stats",
           "asp_release", "asp_stage_particles", "asp_periodic", "asp_wrapped_distance",
           "asp_knn_smoothing_lengths", "asp_table_interp3", "asp_table_interp")

STAGES = ("memset", "count", "colscan", "tilescan", "scatter", "scale", "deposit", "merge",
          "wide", "ratio", "cube_count", "cube_colscan", "cube_tilescan", "cube_scatter",
          "cube_deposit", "cube_merge", "gather", "knn_prep", "knn_search")

_lib = None

_f = C.POINTER(C.c_float)
_d = C.POINTER(C.c_double)
_i32 = C.POINTER(C.c_int32)
_i64 = C.POINTER(C.c_int64)


class ASPError(RuntimeError):
    pass


def build():
    """Compile libasp_hip.so in-tree (hipcc --offload-arch=gfx950)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", ROOT], check=True)


def lib():
    """Load libasp_hip.so (torch first when present, so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP extension not built: {LIB_PATH} missing "
                          f"(run `make -C {ROOT}` or __graft_entry__.build())")
    if "torch" not in sys.modules:
        try:  # torch ships its own libamdhip64; load it first so there is one runtime
            import torch  # noqa: F401
        except Exception:
            pass
    L = C.CDLL(LIB_PATH)
    L.asp_version.restype = C.c_int
    L.asp_last_error.restype = C.c_char_p
    L.asp_device_count.restype = C.c_int
    L.asp_project2d.argtypes = [_f, _f, _f, _f, _f, C.c_int64, C.c_double, C.c_double,
                                C.c_double, C.c_double, C.c_int32, C.c_int32, C.c_int32,
                                C.c_int32, C.c_int32, _f, _f, C.c_int32, C.c_void_p]
    if hasattr(L, "asp_project2d_rows"):  # (absent from an older A/B build, ASP_LIB)
      L.asp_project2d_rows.argtypes = [_f, _f, _f, _f, _f, C.c_int64, C.c_double, C.c_double,
                                       C.c_double, C.c_double, C.c_int32, C.c_int32,
                                       C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                       _f, _f, C.c_int32, C.c_void_p]
    if hasattr(L, "asp_project2d_props"):  # (absent from an older A/B build, ASP_LIB)
        L.asp_project2d_props.argtypes = [_f, _f, _f, C.POINTER(_f), C.c_int32, C.c_int64,
                                          C.c_double, C.c_double, C.c_double, C.c_double,
                                          C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                          C.POINTER(_f), C.c_int32, C.c_void_p]
        L.asp_project2d_props_f64.argtypes = [_d, _d, C.POINTER(_d), C.c_int32, C.c_int64,
                                              C.c_int32, C.c_double, C.c_double, C.c_double,
                                              C.c_double, C.c_int32, C.c_int32, C.c_int32,
                                              C.c_int32, C.c_int32, C.POINTER(_f), C.c_int32,
                                              C.c_void_p]
    if hasattr(L, "asp_project2d_sph"):
        L.asp_project2d_sph.argtypes = [_f, _f, _f, _f, _f, C.POINTER(_f), C.c_int32, C.c_int64,
                                        C.c_double, C.c_double, C.c_double, C.c_double,
                                        C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                        C.POINTER(_f), C.c_int32, C.c_void_p]
        L.asp_project2d_sph_f64.argtypes = [_d, _d, _d, _d, C.POINTER(_d), C.c_int32, C.c_int64,
                                            C.c_int32, C.c_double, C.c_double, C.c_double,
                                            C.c_double, C.c_int32, C.c_int32, C.c_int32,
                                            C.c_int32, C.c_int32, C.POINTER(_f), C.c_int32,
                                            C.c_void_p]
    L.asp_project2d_f64.argtypes = [_d, _d, _d, _d, C.c_int64, C.c_int32, C.c_double,
                                    C.c_double, C.c_double, C.c_double, C.c_int32, C.c_int32,
                                    C.c_int32, C.c_int32, C.c_int32, _f, _f, C.c_int32,
                                    C.c_void_p]
    L.asp_pairs_begin.argtypes = [_d, _d, C.c_int64, C.c_int32, C.c_double, C.c_double,
                                  C.c_double, C.c_double, C.c_int32, C.c_int32, C.c_int32,
                                  C.c_int32, C.c_int32, C.c_void_p, _i64, C.POINTER(C.c_void_p)]
    L.asp_pairs_emit.argtypes = [C.c_void_p, C.c_int32, C.c_int32, _i64, _i32, _d]
    L.asp_pairs_end.argtypes = [C.c_void_p]
    L.asp_project3d.argtypes = ([_f] * 5 + [C.c_int64] + [C.c_double] * 6 + [C.c_int32] * 7
                                + [_f, C.c_int32, C.c_void_p])
    L.asp_kernel_eval.argtypes = [C.c_int32, _d, _d, _d, C.c_int64, C.c_int32, C.c_int32,
                                  C.c_void_p]
    L.asp_chunk_ranges.argtypes = [_f, _f, _f, C.c_int64, C.c_double, C.c_double, C.c_double,
                                   C.c_double, C.c_int32, C.c_int32, C.c_int32, _i32, _i32,
                                   _i32, _i32, C.c_int32, C.c_int32, C.c_void_p]
    L.asp_pixel_neighbours.argtypes = [_f, _f, _f, C.c_int64, C.c_double, C.c_double,
                                       C.c_double, C.c_double, C.c_int32, C.c_int32, C.c_int32,
                                       _i64, C.c_int64, _i64, _i32, C.c_int64, _i64, C.c_int32]
    L.asp_ratio.argtypes = [_f, _f, C.c_int64, C.c_int32, C.c_void_p]
    L.asp_profile.argtypes = [C.c_int32, C.c_int32]
    L.asp_profile_stages.argtypes = [C.c_int32, C.c_uint32]
    L.asp_profile_read.argtypes = [C.c_int32, _d, _i64, C.c_int32]
    L.asp_last_stats.argtypes = [C.c_int32, _i64, C.c_int32]
    L.asp_release.argtypes = [C.c_int32]
    L.asp_stage_particles.argtypes = [_d, _d, _d, _d, C.c_int64, C.c_int32, _d, C.c_double,
                                      C.c_int32, _f, _f, _f, _f, _f, C.c_int64, _i64, C.c_int32,
                                      C.c_int32, C.c_void_p]
    L.asp_periodic.argtypes = [C.c_int32, _d, C.c_int64, _d, C.c_int64, C.c_int64, C.c_double,
                               C.c_int32, _d, C.c_int32, C.c_void_p]
    L.asp_wrapped_distance.argtypes = [_d, C.c_int64, _d, C.c_int64, C.c_int64, C.c_double,
                                       C.c_int32, _d, C.c_int32, C.c_void_p]
    L.asp_knn_smoothing_lengths.argtypes = [_d, C.c_int64, C.c_int32, _d, C.c_int32, C.c_int32,
                                            C.c_void_p]
    L.asp_table_interp3.argtypes = ([_d, C.c_int32, C.c_int32, C.c_int32, _d, _d, _d, _d,
                                     C.c_int32, C.c_int32, C.c_double, C.c_int64, C.c_double,
                                     C.c_int32, _d, _d, _d, C.c_int32, C.c_void_p])
    L.asp_table_interp.argtypes = ([_d, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_void_p),
                                    _d, C.c_int32, C.c_int32, C.c_double, C.c_int64, C.c_double,
                                    C.c_int32, C.c_int32, _d, _d, _d, C.c_int32, C.c_void_p])
    for name in ("asp_project2d", "asp_project2d_f64", "asp_pairs_begin", "asp_pairs_emit",
                 "asp_pairs_end", "asp_project3d", "asp_kernel_eval", "asp_chunk_ranges",
                 "asp_pixel_neighbours", "asp_ratio", "asp_profile", "asp_profile_stages",
                 "asp_profile_read", "asp_last_stats", "asp_release", "asp_stage_particles",
                 "asp_periodic", "asp_wrapped_distance", "asp_knn_smoothing_lengths",
                 "asp_table_interp3", "asp_table_interp"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


def check(rc: int):
    if rc == ASP_OK:
        return
    msg = lib().asp_last_error().decode(errors="replace")
    if rc == ASP_ERR_INVALID:
        raise ValueError(msg)
    if rc == ASP_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == ASP_ERR_NOMEM:
        raise MemoryError(msg)
    raise ASPError(f"HIP error: {msg}")


def require_gpu(device: int = 0):
    n = lib().asp_device_count()
    if n <= 0:
        raise RuntimeError("no HIP device visible: the projector runs on MI355X only "
                           "(there is no CPU fallback)")
    if not 0 <= device < n:
        raise ValueError(f"device {device} out of range (have {n})")


def ptr(a, t=_f):
    """ctypes pointer of a numpy array, or of a torch tensor's device memory, or NULL."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return C.cast(C.c_void_p(a.data_ptr()), t)
    return a.ctypes.data_as(t)


def last_stats(device: int = 0):
    s = (C.c_int64 * 15)()
    check(lib().asp_last_stats(device, s, 15))
    return {"records": s[0], "items": s[1], "wide": s[2], "tile": s[3], "tiles": s[4],
            "records_per_item": s[5], "merges": s[6], "slabs": s[7], "large": s[8],
            "evals": s[9], "evals_small": s[10], "evals_gather": s[11], "evals_wide": s[12],
            "scatter_path": s[13], "placement_runs": s[14]}


def profile(device: int = 0, enable: bool = True, stages=None):
    """Start (and reset) / stop per-stage HIP-event timing inside the library; ``stages``
    (names of STAGES) limits the events to those stages."""
    if stages is None or not enable:
        check(lib().asp_profile(device, 1 if enable else 0))
    else:
        mask = 0
        for s in stages:
            mask |= 1 << STAGES.index(s)
        check(lib().asp_profile_stages(device, mask))


def profile_read(device: int = 0):
    """{stage: (total_ms, launches)} since the last reset."""
    ms = (C.c_double * len(STAGES))()
    n = (C.c_int64 * len(STAGES))()
    check(lib().asp_profile_read(device, ms, n, len(STAGES)))
    return {s: (ms[i], n[i]) for i, s in enumerate(STAGES)}
