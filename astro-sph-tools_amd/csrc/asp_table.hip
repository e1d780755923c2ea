// asp_table.hip -- ionisation-table interpolation on the device.
//
// The reference's ion tables (data_structures/_IonisationTable.py:30-58, read by
// io/ionisation_tables/_HM01.py:61-92) interpolate a 3-D table of ion fractions over
// (log10 n_H, log10 T, redshift) with scipy's RegularGridInterpolator (linear,
// bounds_error=False, fill_value=-inf).  Ion column maps weight each particle by
// m * X_element * f_ion before projecting.  This file restates scipy 1.15's
// linear evaluation (scipy/interpolate/_rgi.py:_evaluate_linear, find_indices) in fp64 with
// the same operation order, so values are bit-identical to the reference's
// (tests/test_gpu_table.py):
//   per axis d: i_d = the largest i with g_d[i] <= x_d, clamped to [0, n_d - 2];
//               y_d = (x_d - g_d[i_d]) / (g_d[i_d + 1] - g_d[i_d]);
//   value = 0, then for the 8 corners in itertools.product order (last axis fastest),
//           value = value + t[corner] * ((w_0 * w_1) * w_2), w_d = 1 - y_d or y_d;
//   outside [g_d[0], g_d[-1]] on any axis: fill; NaN on any axis: NaN.
// Element-wise gather work (the table is small and stays in L2): one lane per point.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../../include/asp.h"
#include "asp_host.hpp"

namespace asp {

constexpr int kTabBlock = 256;
constexpr int kTabPerThread = 4;      // points per thread (amortises the LDS axis copy)
constexpr int kTabLdsAxis = 2048;     // axes up to this many nodes in total go through LDS

struct TabAxes {
    const double* g[3];
    int n[3];
};

// largest i with g[i] <= x, clamped to [0, n - 2] (find_indices' interval search).  A guess
// from the mean node spacing, corrected against the nodes: O(1) for the (near-)uniform
// axes of the HM01 tables, exact for any strictly ascending axis (binary search when the
// guess is off by more than one node).
__device__ __forceinline__ int interval(const double* __restrict__ g, int n, double inv, double x) {
    if (!(x >= g[1])) return 0;
    if (x >= g[n - 2]) return n - 2;
    // here g[1] <= x < g[n - 2]: the answer lies in [1, n - 3]
    int i = (int)((x - g[0]) * inv);
    i = min(max(i, 1), n - 3);
    if (g[i] <= x) {
        if (x < g[i + 1]) return i;
        if (x < g[i + 2]) return i + 1;
    } else if (g[i - 1] <= x) {
        return i - 1;
    }
    int lo = 1, hi = n - 2;  // invariant: g[lo] <= x < g[hi]
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (g[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

// one axis of find_indices: interval i, normalised distance y, and the NaN / out-of-bounds
// flags _prepare_xi / _find_out_of_bounds derive from the same coordinate
__device__ __forceinline__ void locate(const double* __restrict__ g, int n, double inv, double x,
                                       int& i, double& y, bool& nan, bool& oob) {
    nan |= x != x;
    oob |= x < g[0] || x > g[n - 1];
    i = interval(g, n, inv, x);
    y = (x - g[i]) / (g[i + 1] - g[i]);
}

typedef double pair_t __attribute__((ext_vector_type(2), aligned(8)));

// _evaluate_linear: v = 0; v = v + t[corner] * ((w0 * w1) * w2) over the corners in
// itertools.product order (last axis fastest).  The two corners along the last axis are
// adjacent in the table and come in with one load.
__device__ __forceinline__ double interp3(const double* __restrict__ t, const int n[3],
                                          const int i[3], const double y[3]) {
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < 8; c += 2) {
        const int a = (c >> 2) & 1, b = (c >> 1) & 1;
        const double w0 = a ? y[0] : 1 - y[0], w1 = b ? y[1] : 1 - y[1];
        const long long o = ((long long)(i[0] + a) * n[1] + (i[1] + b)) * n[2] + i[2];
        const pair_t p = *reinterpret_cast<const pair_t*>(t + o);
        v = v + p.x * ((w0 * w1) * (1 - y[2]));
        v = v + p.y * ((w0 * w1) * y[2]);
    }
    return v;
}

// pts: (n, 3) rows, or (n, 2) rows with the constant zc inserted at axis zaxis
// (IonisationTableBase.evaluate_at_redshift, _IonisationTable.py:54-58).  mode 1: out =
// a0 * a1 * value (ion masses m * X * f); mode 2: out = a0 * a1 * 10^value (exp10).  Each thread
// takes kTabPerThread points strided by the block size (coalesced loads).
template <int NCOL, bool LDS>
__global__ __launch_bounds__(kTabBlock) void k_table(const double* __restrict__ t, TabAxes A,
                                                     const double* __restrict__ pts, int zaxis,
                                                     double zc, long long n, double fill,
                                                     int mode, const double* __restrict__ a0,
                                                     const double* __restrict__ a1,
                                                     double* __restrict__ out) {
    __shared__ double s_g[LDS ? kTabLdsAxis : 1];
    const double* g[3];
    int nn[3];
    double inv[3];
    if constexpr (LDS) {
        int off = 0;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            for (int k = threadIdx.x; k < A.n[d]; k += kTabBlock) s_g[off + k] = A.g[d][k];
            g[d] = s_g + off;
            off += A.n[d];
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int d = 0; d < 3; ++d) g[d] = A.g[d];
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        nn[d] = A.n[d];
        inv[d] = (double)(A.n[d] - 1) / (g[d][A.n[d] - 1] - g[d][0]);
    }
    // evaluate_at_redshift: the fixed axis is located once per thread (same values)
    int fi = 0;
    double fy = 0.0;
    bool fnan = false, foob = false;
    if constexpr (NCOL == 2) locate(g[zaxis], nn[zaxis], inv[zaxis], zc, fi, fy, fnan, foob);
    const long long base = (long long)blockIdx.x * (kTabBlock * kTabPerThread) + threadIdx.x;
#pragma unroll
    for (int r = 0; r < kTabPerThread; ++r) {
        const long long p = base + (long long)r * kTabBlock;
        if (p >= n) return;
        int i[3];
        double y[3];
        bool nan = false, oob = false;
        if constexpr (NCOL == 3) {
#pragma unroll
            for (int d = 0; d < 3; ++d) locate(g[d], nn[d], inv[d], pts[3 * p + d], i[d], y[d], nan, oob);
        } else {
            nan = fnan;
            oob = foob;
            const double x0 = pts[2 * p], x1 = pts[2 * p + 1];
#pragma unroll
            for (int d = 0, c = 0; d < 3; ++d) {
                if (d == zaxis) {
                    i[d] = fi;
                    y[d] = fy;
                } else {
                    locate(g[d], nn[d], inv[d], c == 0 ? x0 : x1, i[d], y[d], nan, oob);
                    ++c;
                }
            }
        }
        double v = nan ? (double)NAN : (oob ? fill : interp3(t, nn, i, y));
        if (mode == 1) v = (a0[p] * a1[p]) * v;
        else if (mode == 2) v = (a0[p] * a1[p]) * exp10(v);
        out[p] = v;
    }
}

// evaluate_at_redshift with the redshift as the last table axis (HM01): every point reads
// the same two z layers, t[:, :, iz] and t[:, :, iz + 1], which go to LDS as adjacent
// pairs (41 x 141 x 2 fp64 = 92.5 KB for HM01) together with the two free axes.  The
// corner gathers then hit LDS instead of pulling a whole L2 line per lane (the global
// kernel above is L2-bandwidth bound on random gas states: 2.0 ms vs 0.8 ms on sorted ones
// at 1e8).  One 1024-thread workgroup per CU, persistent over batches of 4 points/thread.
constexpr int kSlabBlock = 1024;
constexpr int kSlabPerThread = 4;
constexpr int kSlabMax = 16384;   // doubles: n0 * n1 * 2 <= 16384 (128 KiB)

__global__ __launch_bounds__(kSlabBlock) void k_table_slab(const double* __restrict__ t, TabAxes A,
                                                           const double* __restrict__ pts,
                                                           double zc, long long n, double fill,
                                                           int mode, const double* __restrict__ a0,
                                                           const double* __restrict__ a1,
                                                           double* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) double s_slab[kSlabMax];
    __shared__ double s_g[kTabLdsAxis];
    const int n0 = A.n[0], n1 = A.n[1], n2 = A.n[2];
    for (int k = threadIdx.x; k < n0; k += kSlabBlock) s_g[k] = A.g[0][k];
    for (int k = threadIdx.x; k < n1; k += kSlabBlock) s_g[n0 + k] = A.g[1][k];
    const double* g0 = s_g;
    const double* g1 = s_g + n0;
    // the fixed axis is located from global memory by every thread (same values)
    int fi;
    double fy;
    bool fnan = false, foob = false;
    const double inv2 = (double)(n2 - 1) / (A.g[2][n2 - 1] - A.g[2][0]);
    locate(A.g[2], n2, inv2, zc, fi, fy, fnan, foob);
    for (int k = threadIdx.x; k < n0 * n1 * 2; k += kSlabBlock)
        s_slab[k] = t[(long long)(k >> 1) * n2 + fi + (k & 1)];
    __syncthreads();
    const double inv0 = (double)(n0 - 1) / (g0[n0 - 1] - g0[0]);
    const double inv1 = (double)(n1 - 1) / (g1[n1 - 1] - g1[0]);
    const double wz0 = 1 - fy, wz1 = fy;
    const long long step = (long long)gridDim.x * (kSlabBlock * kSlabPerThread);
    for (long long base = (long long)blockIdx.x * (kSlabBlock * kSlabPerThread) + threadIdx.x;
         base < n; base += step) {
        double x0[kSlabPerThread], x1[kSlabPerThread], w[kSlabPerThread];
#pragma unroll
        for (int r = 0; r < kSlabPerThread; ++r) {
            const long long p = base + (long long)r * kSlabBlock;
            const bool ok = p < n;
            x0[r] = ok ? pts[2 * p] : 0.0;
            x1[r] = ok ? pts[2 * p + 1] : 0.0;
            w[r] = (ok && mode) ? a0[p] * a1[p] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < kSlabPerThread; ++r) {
            const long long p = base + (long long)r * kSlabBlock;
            if (p >= n) break;
            int i0, i1;
            double y0, y1;
            bool nan = fnan, oob = foob;
            locate(g0, n0, inv0, x0[r], i0, y0, nan, oob);
            locate(g1, n1, inv1, x1[r], i1, y1, nan, oob);
            double v;
            if (nan) {
                v = NAN;
            } else if (oob) {
                v = fill;
            } else {
                v = 0.0;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int a = c >> 1, b = c & 1;
                    const double w0 = a ? y0 : 1 - y0, w1 = b ? y1 : 1 - y1;
                    const double2 q = *reinterpret_cast<const double2*>(
                        s_slab + 2 * ((i0 + a) * n1 + (i1 + b)));
                    v = v + q.x * ((w0 * w1) * wz0);
                    v = v + q.y * ((w0 * w1) * wz1);
                }
            }
            if (mode == 1) v = w[r] * v;
            else if (mode == 2) v = w[r] * exp10(v);
            out[p] = v;
        }
    }
}

// ----------------------------------------------------------------------------------
// Any number of table axes (IonisationTableBase accepts N input dimensions,
// _IonisationTable.py:31-49).  scipy 1.15 evaluates N != 2 with _evaluate_linear:
//   weight = 1; weight = weight * w_d over the axes in order; value = value + t * weight,
// and a writeable native-fp64 2-D table with the Cython evaluate_linear_2d:
//   value = value + t[corner] * w_0 * w_1   (left to right: the table value first).
// Both over the corners in itertools.product order (last axis fastest).  `vfirst` selects
// the 2-D form.  One lane per point; the axes are read from global memory (L1/L2).
// ----------------------------------------------------------------------------------
constexpr int kTabMaxDims = 6;
struct TabND {
    const double* g[kTabMaxDims];
    int n[kTabMaxDims];
    long long stride[kTabMaxDims];
};

template <int D>
__global__ __launch_bounds__(kTabBlock) void k_table_nd(const double* __restrict__ t, TabND A,
                                                        const double* __restrict__ pts, int ncol,
                                                        int zaxis, double zc, long long n,
                                                        double fill, int mode, int vfirst,
                                                        const double* __restrict__ a0,
                                                        const double* __restrict__ a1,
                                                        double* __restrict__ out) {
    const long long p = (long long)blockIdx.x * kTabBlock + threadIdx.x;
    if (p >= n) return;
    int i[D];
    double y[D];
    bool nan = false, oob = false;
#pragma unroll
    for (int d = 0, c = 0; d < D; ++d) {
        double x;
        if (ncol == D) {
            x = pts[(long long)D * p + d];
        } else if (d == zaxis) {
            x = zc;
        } else {
            x = pts[(long long)ncol * p + c];
            ++c;
        }
        const double inv = (double)(A.n[d] - 1) / (A.g[d][A.n[d] - 1] - A.g[d][0]);
        locate(A.g[d], A.n[d], inv, x, i[d], y[d], nan, oob);
    }
    double v;
    if (nan) {
        v = NAN;
    } else if (oob) {
        v = fill;
    } else {
        v = 0.0;
#pragma unroll
        for (int c = 0; c < (1 << D); ++c) {
            long long o = 0;
#pragma unroll
            for (int d = 0; d < D; ++d) o += (long long)(i[d] + ((c >> (D - 1 - d)) & 1)) * A.stride[d];
            double term;
            if (vfirst) {
                term = t[o];
#pragma unroll
                for (int d = 0; d < D; ++d) term = term * (((c >> (D - 1 - d)) & 1) ? y[d] : 1 - y[d]);
            } else {
                double w = 1.0;
#pragma unroll
                for (int d = 0; d < D; ++d) w = w * (((c >> (D - 1 - d)) & 1) ? y[d] : 1 - y[d]);
                term = t[o] * w;
            }
            v = v + term;
        }
    }
    if (mode == 1) v = (a0[p] * a1[p]) * v;
    else if (mode == 2) v = (a0[p] * a1[p]) * exp10(v);
    out[p] = v;
}

}  // namespace asp

using namespace asp;

extern "C" int asp_table_interp3(const double* table, int32_t n0, int32_t n1, int32_t n2,
                                 const double* g0, const double* g1, const double* g2,
                                 const double* points, int32_t ncol, int32_t zaxis, double zvalue,
                                 int64_t n, double fill, int32_t mode, const double* a0,
                                 const double* a1, double* out, int32_t device, void* stream) {
    t_err.clear();
    if (n0 < 2 || n1 < 2 || n2 < 2) return fail(ASP_ERR_INVALID, "every table axis needs >= 2 points");
    if (ncol != 3 && ncol != 2) return fail(ASP_ERR_INVALID, "points must have 3 (or 2 + zvalue) columns");
    if (ncol == 2 && (zaxis < 0 || zaxis > 2)) return fail(ASP_ERR_INVALID, "bad fixed axis");
    if (mode < 0 || mode > 2) return fail(ASP_ERR_INVALID, "bad mode");
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (n == 0) return ASP_OK;
    if (!table || !g0 || !g1 || !g2 || !points || !out || (mode && (!a0 || !a1)))
        return fail(ASP_ERR_INVALID, "NULL array");
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    TabAxes A{{g0, g1, g2}, {n0, n1, n2}};
    const bool lds = (long long)n0 + n1 + n2 <= kTabLdsAxis;
    const dim3 grid((unsigned)((n + kTabBlock * kTabPerThread - 1) / (kTabBlock * kTabPerThread)));
    hipStream_t st = (hipStream_t)stream;
    if (ncol == 3) {
        if (lds) hipLaunchKernelGGL((k_table<3, true>), grid, dim3(kTabBlock), 0, st, table, A, points, 0, 0.0, (long long)n, fill, (int)mode, a0, a1, out);
        else hipLaunchKernelGGL((k_table<3, false>), grid, dim3(kTabBlock), 0, st, table, A, points, 0, 0.0, (long long)n, fill, (int)mode, a0, a1, out);
    } else if (zaxis == 2 && (long long)n0 * n1 * 2 <= kSlabMax && (long long)n0 + n1 <= kTabLdsAxis) {
        int dev_cus = 0;
        ASP_HIP(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, device));
        const long long need = (n + kSlabBlock * kSlabPerThread - 1) / (kSlabBlock * kSlabPerThread);
        const unsigned blocks = (unsigned)std::min<long long>(need, (long long)dev_cus * 2);
        hipLaunchKernelGGL(k_table_slab, dim3(blocks), dim3(kSlabBlock), 0, st, table, A, points, zvalue, (long long)n, fill, (int)mode, a0, a1, out);
    } else {
        if (lds) hipLaunchKernelGGL((k_table<2, true>), grid, dim3(kTabBlock), 0, st, table, A, points, (int)zaxis, zvalue, (long long)n, fill, (int)mode, a0, a1, out);
        else hipLaunchKernelGGL((k_table<2, false>), grid, dim3(kTabBlock), 0, st, table, A, points, (int)zaxis, zvalue, (long long)n, fill, (int)mode, a0, a1, out);
    }
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}

extern "C" int asp_table_interp(const double* table, int32_t ndim, const int32_t* shape,
                                const double* const* axes, const double* points, int32_t ncol,
                                int32_t zaxis, double zvalue, int64_t n, double fill,
                                int32_t mode, int32_t order, const double* a0, const double* a1,
                                double* out, int32_t device, void* stream) {
    t_err.clear();
    if (ndim < 1 || ndim > kTabMaxDims) return fail(ASP_ERR_UNSUPPORTED, "1 .. 6 table axes");
    if (!shape || !axes) return fail(ASP_ERR_INVALID, "NULL shape / axes");
    for (int d = 0; d < ndim; ++d)
        if (shape[d] < 2 || !axes[d]) return fail(ASP_ERR_INVALID, "every table axis needs >= 2 points");
    if (ncol != ndim && !(ncol == ndim - 1 && zaxis >= 0 && zaxis < ndim))
        return fail(ASP_ERR_INVALID, "points must have ndim (or ndim - 1 + zvalue) columns");
    if (mode < 0 || mode > 2 || order < 0 || order > 1) return fail(ASP_ERR_INVALID, "bad mode / order");
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (n == 0) return ASP_OK;
    if (!table || !points || !out || (mode && (!a0 || !a1))) return fail(ASP_ERR_INVALID, "NULL array");
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    TabND A{};
    long long st = 1;
    for (int d = ndim - 1; d >= 0; --d) {
        A.g[d] = axes[d];
        A.n[d] = shape[d];
        A.stride[d] = st;
        st *= shape[d];
    }
    const dim3 grid((unsigned)((n + kTabBlock - 1) / kTabBlock));
    hipStream_t s = (hipStream_t)stream;
    const int vfirst = order == 1 && ndim == 2;
#define ASP_TAB_ND(D)                                                                          \
    case D:                                                                                    \
        hipLaunchKernelGGL((k_table_nd<D>), grid, dim3(kTabBlock), 0, s, table, A, points,     \
                           (int)ncol, (int)zaxis, zvalue, (long long)n, fill, (int)mode,       \
                           vfirst, a0, a1, out);                                               \
        break;
    switch (ndim) {
        ASP_TAB_ND(1)
        ASP_TAB_ND(2)
        ASP_TAB_ND(3)
        ASP_TAB_ND(4)
        ASP_TAB_ND(5)
        ASP_TAB_ND(6)
    }
#undef ASP_TAB_ND
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}
