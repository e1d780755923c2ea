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

struct TabAxes {
    const double* g[3];
    int n[3];
};

// largest i with g[i] <= x, clamped to [0, n - 2] (find_indices' interval search)
__device__ __forceinline__ int interval(const double* __restrict__ g, int n, double x) {
    int lo = 0, hi = n - 1;  // invariant: answer in [lo, hi)
    if (!(x >= g[1])) return 0;
    if (x >= g[n - 2]) return n - 2;
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (g[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ double interp3(const double* __restrict__ t, const TabAxes& A, double x0,
                                          double x1, double x2, double fill) {
    const double xs[3] = {x0, x1, x2};
    int i[3];
    double y[3];
    bool nan = false, oob = false;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double* g = A.g[d];
        const double x = xs[d];
        nan |= x != x;
        oob |= x < g[0] || x > g[A.n[d] - 1];
        i[d] = interval(g, A.n[d], x);
        y[d] = (x - g[i[d]]) / (g[i[d] + 1] - g[i[d]]);
    }
    if (nan) return NAN;
    if (oob) return fill;
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int a = (c >> 2) & 1, b = (c >> 1) & 1, e = c & 1;
        const double w0 = a ? y[0] : 1 - y[0], w1 = b ? y[1] : 1 - y[1], w2 = e ? y[2] : 1 - y[2];
        const long long o = ((long long)(i[0] + a) * A.n[1] + (i[1] + b)) * A.n[2] + (i[2] + e);
        v = v + t[o] * ((w0 * w1) * w2);
    }
    return v;
}

// pts: (n, 3) rows, or (n, 2) rows with the constant zc inserted at axis zaxis
// (IonisationTableBase.evaluate_at_redshift, _IonisationTable.py:54-58).  mode 1: out =
// a0 * a1 * value (ion masses m * X * f); mode 2: out = a0 * a1 * 10^value.
__global__ __launch_bounds__(kTabBlock) void k_table(const double* __restrict__ t, TabAxes A,
                                                     const double* __restrict__ pts, int ncol,
                                                     int zaxis, double zc, long long n, double fill,
                                                     int mode, const double* __restrict__ a0,
                                                     const double* __restrict__ a1,
                                                     double* __restrict__ out) {
    long long i = (long long)blockIdx.x * kTabBlock + threadIdx.x;
    if (i >= n) return;
    double x[3];
    if (ncol == 3) {
        x[0] = pts[3 * i];
        x[1] = pts[3 * i + 1];
        x[2] = pts[3 * i + 2];
    } else {
        int c = 0;
#pragma unroll
        for (int d = 0; d < 3; ++d) x[d] = d == zaxis ? zc : pts[2 * i + (c++)];
    }
    double v = interp3(t, A, x[0], x[1], x[2], fill);
    if (mode == 1) v = (a0[i] * a1[i]) * v;
    else if (mode == 2) v = (a0[i] * a1[i]) * pow(10.0, v);
    out[i] = v;
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
    hipLaunchKernelGGL(k_table, dim3((unsigned)((n + kTabBlock - 1) / kTabBlock)), dim3(kTabBlock),
                       0, (hipStream_t)stream, table, A, points, (int)ncol, (int)zaxis, zvalue,
                       (long long)n, fill, (int)mode, a0, a1, out);
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}
