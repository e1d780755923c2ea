// asp_knn.hip -- smoothing lengths from the k-th nearest neighbour.
//
// Replaces the scipy KDTree query of io/SWIFT/_SnapshotSWIFT.py:62-83: particles without
// SPH smoothing lengths (dark matter) get h = the distance to their k-th nearest
// neighbour, the particle itself counted (k = 32 there).  The distance is scipy's
// Euclidean one in fp64, d2 = ((x_i - x_j)^2 + (y_i - y_j)^2) + (z_i - z_j)^2 and
// h = sqrt(d2_(k)), so results are bit-identical to the reference (tests/test_gpu_knn.py);
// +inf when n < k (scipy's value for a missing neighbour).
//
// MI355X layout: particles sorted along a 63-bit Morton curve (21 bits per axis over the
// bounding cube; rocPRIM radix sort), positions gathered into sorted fp64 SoA so that the
// particles a thread scans are contiguous and shared with its neighbours in the wave
// (L1/L2 hits).  Per particle (one thread):
//   1. an upper bound R on the k-th distance from the finest Morton cell around it that
//      holds k + 1 particles (any k points bound the k-th nearest distance from above);
//   2. every cell of the Morton level whose cell edge is >= R that the ball of radius R
//      (plus one quantum of slack) touches -- at most 3 per axis, each a contiguous
//      key range found by binary search -- own cell first, cells whose box lies beyond
//      the current k-th distance skipped;
//   3. a register top-k (the k smallest d2 seen; replace-the-maximum), exact in fp64.
// The k-th smallest d2 over a superset of the ball is the exact answer.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/asp.h"
#include "asp_host.hpp"

namespace asp {

constexpr int kKnnBlock = 256;
constexpr int kQBits = 21;                       // quantisation bits per axis
constexpr long long kQMax = (1LL << kQBits) - 1;
constexpr int kRedBlocks = 1024;                 // bounding-box partial reductions

__device__ __forceinline__ unsigned long long spread21(unsigned long long v) {
    v &= 0x1fffffULL;
    v = (v | v << 32) & 0x1f00000000ffffULL;
    v = (v | v << 16) & 0x1f0000ff0000ffULL;
    v = (v | v << 8) & 0x100f00f00f00f00fULL;
    v = (v | v << 4) & 0x10c30c30c30c30c3ULL;
    v = (v | v << 2) & 0x1249249249249249ULL;
    return v;
}

__device__ __forceinline__ unsigned long long morton3(long long a, long long b, long long c) {
    return (spread21(a) << 2) | (spread21(b) << 1) | spread21(c);
}

// Per-block min / max of each coordinate (NaN ignored) -> part[block][6].
__global__ __launch_bounds__(kKnnBlock) void k_bbox(const double* __restrict__ pos, long long n,
                                                    double* __restrict__ part) {
    __shared__ double s[6][kKnnBlock];
    double m[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x; i < n;
         i += (long long)gridDim.x * kKnnBlock) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double x = pos[3 * i + a];
            m[a] = fmin(m[a], x);
            m[3 + a] = fmax(m[3 + a], x);
        }
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) s[a][threadIdx.x] = m[a];
    __syncthreads();
    for (int o = kKnnBlock / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                s[a][threadIdx.x] = fmin(s[a][threadIdx.x], s[a][threadIdx.x + o]);
                s[3 + a][threadIdx.x] = fmax(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + o]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[(long long)blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

// Quantisation: q = floor((x - lo_a) * scale) on a cube of edge span over the largest
// axis extent, clamped to [0, 2^21 - 1]; the grid struct every kernel shares.
struct KGrid {
    double lo[3];
    double scale;   // quanta per unit length
    double quantum; // 1 / scale
};

__global__ __launch_bounds__(kKnnBlock) void k_bbox_final(const double* __restrict__ part, int nb,
                                                          KGrid* __restrict__ g) {
    __shared__ double s[6][kKnnBlock];
    double m[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int b = threadIdx.x; b < nb; b += kKnnBlock)
        for (int a = 0; a < 3; ++a) {
            m[a] = fmin(m[a], part[6 * b + a]);
            m[3 + a] = fmax(m[3 + a], part[6 * b + 3 + a]);
        }
    for (int a = 0; a < 6; ++a) s[a][threadIdx.x] = m[a];
    __syncthreads();
    for (int o = kKnnBlock / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o)
            for (int a = 0; a < 3; ++a) {
                s[a][threadIdx.x] = fmin(s[a][threadIdx.x], s[a][threadIdx.x + o]);
                s[3 + a][threadIdx.x] = fmax(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + o]);
            }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    double span = 0.0;
    for (int a = 0; a < 3; ++a) {
        g->lo[a] = __builtin_isfinite(s[a][0]) ? s[a][0] : 0.0;
        double e = s[3 + a][0] - s[a][0];
        if (__builtin_isfinite(e)) span = fmax(span, e);
    }
    if (!(span > 0.0)) span = 1.0;
    // 2^21 quanta over span * (1 + 2^-20): the largest coordinate stays below 2^21
    g->scale = (double)(1LL << kQBits) / (span * (1.0 + 0x1p-20));
    g->quantum = 1.0 / g->scale;
}

__device__ __forceinline__ long long quant(double x, double lo, double scale) {
    double q = floor((x - lo) * scale);
    if (!(q >= 0.0)) return 0;  // also NaN
    return q > (double)kQMax ? kQMax : (long long)q;
}

__global__ __launch_bounds__(kKnnBlock) void k_keys(const double* __restrict__ pos, long long n,
                                                    const KGrid* __restrict__ g,
                                                    unsigned long long* __restrict__ keys,
                                                    int* __restrict__ idx) {
    long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (i >= n) return;
    const KGrid G = *g;
    keys[i] = morton3(quant(pos[3 * i], G.lo[0], G.scale), quant(pos[3 * i + 1], G.lo[1], G.scale),
                      quant(pos[3 * i + 2], G.lo[2], G.scale));
    idx[i] = (int)i;
}

__global__ __launch_bounds__(kKnnBlock) void k_gather(const double* __restrict__ pos, long long n,
                                                      const int* __restrict__ idx,
                                                      double* __restrict__ xs, double* __restrict__ ys,
                                                      double* __restrict__ zs) {
    long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (i >= n) return;
    long long p = idx[i];
    xs[i] = pos[3 * p];
    ys[i] = pos[3 * p + 1];
    zs[i] = pos[3 * p + 2];
}

// The k smallest d2 seen, in registers (static indexing only): replace the maximum.
template <int K>
struct TopK {
    double v[K];
    double mx;  // the k-th smallest so far (+inf until k values are in)
    int mi;
    __device__ __forceinline__ void init(int k) {
#pragma unroll
        for (int q = 0; q < K; ++q) v[q] = q < k ? INFINITY : -INFINITY;  // -inf: unused slot
        mx = INFINITY;
        mi = 0;
    }
    __device__ __forceinline__ void insert(double d) {
        if (!(d < mx)) return;
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (q == mi) v[q] = d;
        mx = v[0];
        mi = 0;
#pragma unroll
        for (int q = 1; q < K; ++q)
            if (v[q] > mx) {
                mx = v[q];
                mi = q;
            }
    }
};

// scipy's squared Euclidean distance (query point first), fp64, no contraction
__device__ __forceinline__ double dist2(double x, double y, double z, double a, double b, double c) {
    double dx = x - a, dy = y - b, dz = z - c;
    return (dx * dx + dy * dy) + dz * dz;
}

__device__ __forceinline__ long long lower_bound(const unsigned long long* __restrict__ keys,
                                                 long long n, unsigned long long key) {
    long long lo = 0, len = n;
    while (len > 0) {
        long long half = len >> 1;
        if (keys[lo + half] < key) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return lo;
}

template <int K>
__global__ __launch_bounds__(kKnnBlock) void k_knn(const double* __restrict__ xs,
                                                   const double* __restrict__ ys,
                                                   const double* __restrict__ zs,
                                                   const unsigned long long* __restrict__ keys,
                                                   const int* __restrict__ idx, long long n, int k,
                                                   const KGrid* __restrict__ g,
                                                   double* __restrict__ h) {
    long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (i >= n) return;
    const KGrid G = *g;
    const double x = xs[i], y = ys[i], z = zs[i];
    TopK<K> T;
    T.init(k);
    // 1. the finest Morton cell around i holding >= k + 1 particles (its key range grown
    //    level by level by galloping out from i); its k-th distance bounds the answer
    //    from above (any k points do) and its particles go in first
    long long w0 = i, w1 = i + 1;
    if (n >= k + 1) {
        const unsigned long long key = keys[i];
        for (int sh = 0; sh <= 3 * kQBits; sh += 3) {
            const unsigned long long pre = sh >= 63 ? 0ULL : key >> sh;
            auto same = [&](long long j) { return sh >= 63 || (keys[j] >> sh) == pre; };
            // grow w0 down: gallop, then bisect
            long long step = 1;
            while (w0 - step >= 0 && same(w0 - step)) { w0 -= step; step <<= 1; }
            for (step >>= 1; step > 0; step >>= 1)
                if (w0 - step >= 0 && same(w0 - step)) w0 -= step;
            step = 1;
            while (w1 - 1 + step < n && same(w1 - 1 + step)) { w1 += step; step <<= 1; }
            for (step >>= 1; step > 0; step >>= 1)
                if (w1 - 1 + step < n && same(w1 - 1 + step)) w1 += step;
            if (w1 - w0 >= k + 1) break;
        }
    } else {
        w0 = 0;
        w1 = n;
    }
    for (long long j = w0; j < w1; ++j) T.insert(dist2(x, y, z, xs[j], ys[j], zs[j]));
    if (T.mx < INFINITY) {
        // 2. the cells of the level whose edge (2^shift quanta) is >= R
        const double R = sqrt(T.mx) * (1.0 + 0x1p-40);
        // cell edge 2^shift >= R + 1 quantum (in quanta), so the slackened ball spans at
        // most 3 cells per axis
        int e;
        frexp(R * G.scale + 1.0, &e);  // < 2^e
        const int shift = std::min(e, kQBits);
        const double c[3] = {x, y, z};
        long long ca[3], cb[3], co[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            long long qa = std::max<long long>(0, quant(c[a] - R, G.lo[a], G.scale) - 1);
            long long qb = std::min<long long>(kQMax, quant(c[a] + R, G.lo[a], G.scale) + 1);
            ca[a] = qa >> shift;
            cb[a] = qb >> shift;
            co[a] = quant(c[a], G.lo[a], G.scale) >> shift;
        }
        const int sh3 = 3 * shift;
        // own cell first (the k-th distance shrinks fastest there), then the others
        for (int pass = 0; pass < 2; ++pass) {
            for (long long cx = ca[0]; cx <= cb[0]; ++cx)
                for (long long cy = ca[1]; cy <= cb[1]; ++cy)
                    for (long long cz = ca[2]; cz <= cb[2]; ++cz) {
                        bool own = cx == co[0] && cy == co[1] && cz == co[2];
                        if (own != (pass == 0)) continue;
                        // skip cells whose box (one quantum of slack) lies beyond the k-th d2
                        const long long cc[3] = {cx, cy, cz};
                        double md = 0.0;
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            double lo = G.lo[a] + (double)(cc[a] << shift) * G.quantum - G.quantum;
                            double hi = G.lo[a] + (double)((cc[a] + 1) << shift) * G.quantum + G.quantum;
                            double d = c[a] < lo ? lo - c[a] : (c[a] > hi ? c[a] - hi : 0.0);
                            md += d * d;
                        }
                        if (md * (1.0 - 0x1p-40) > T.mx) continue;
                        unsigned long long p = morton3(cx, cy, cz);
                        unsigned long long k0 = sh3 >= 63 ? 0ULL : p << sh3;
                        unsigned long long k1 = sh3 >= 63 ? ~0ULL : (p + 1) << sh3;
                        long long j0 = lower_bound(keys, n, k0);
                        long long j1 = sh3 >= 63 ? n : lower_bound(keys + j0, n - j0, k1) + j0;
                        // [w0, w1) is in already
                        for (long long j = j0; j < std::min(j1, w0); ++j)
                            T.insert(dist2(x, y, z, xs[j], ys[j], zs[j]));
                        for (long long j = std::max(j0, w1); j < j1; ++j)
                            T.insert(dist2(x, y, z, xs[j], ys[j], zs[j]));
                    }
        }
    }
    h[idx[i]] = sqrt(T.mx);
}

static int knn(const double* pos, long long n, int k, double* h, int flags, int device,
               hipStream_t st) {
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (k < 1 || k > 64) return fail(ASP_ERR_INVALID, "k must be in [1, 64]");
    if (n > 0 && (!pos || !h)) return fail(ASP_ERR_INVALID, "NULL array");
    if (n > 0x7fffffffLL) return fail(ASP_ERR_UNSUPPORTED, "n >= 2^31 particles per call");
    if (n == 0) return ASP_OK;
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    const bool dev = flags & ASP_F_DEVICE_PTRS;
    const double* dpos = pos;
    double* dh = h;
    if (!dev) {
        ASP_TRY(ensure(ws.knn[0], (size_t)n * 3 * sizeof(double)));
        ASP_TRY(ensure(ws.knn[1], (size_t)n * sizeof(double)));
        ASP_HIP(hipMemcpyAsync(ws.knn[0].p, pos, (size_t)n * 3 * sizeof(double),
                               hipMemcpyHostToDevice, st));
        dpos = (const double*)ws.knn[0].p;
        dh = (double*)ws.knn[1].p;
    }
    ASP_TRY(ensure(ws.knn[2], (size_t)kRedBlocks * 6 * sizeof(double) + 256));
    ASP_TRY(ensure(ws.knn[3], (size_t)n * 2 * sizeof(unsigned long long)));  // keys in / out
    ASP_TRY(ensure(ws.knn[4], (size_t)n * 2 * sizeof(int)));                 // index in / out
    ASP_TRY(ensure(ws.knn[5], (size_t)n * 3 * sizeof(double)));              // sorted SoA
    double* part = (double*)ws.knn[2].p;
    KGrid* dg = (KGrid*)(part + kRedBlocks * 6);
    unsigned long long* kin = (unsigned long long*)ws.knn[3].p;
    unsigned long long* kout = kin + n;
    int* iin = (int*)ws.knn[4].p;
    int* iout = iin + n;
    double* xs = (double*)ws.knn[5].p;
    double *ys = xs + n, *zs = ys + n;
    const unsigned nb = (unsigned)std::min<long long>(kRedBlocks, (n + kKnnBlock - 1) / kKnnBlock);
    const unsigned grid = (unsigned)((n + kKnnBlock - 1) / kKnnBlock);
    hipLaunchKernelGGL(k_bbox, dim3(nb), dim3(kKnnBlock), 0, st, dpos, (long long)n, part);
    ASP_LAUNCHED();
    hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(kKnnBlock), 0, st, (const double*)part, (int)nb, dg);
    ASP_LAUNCHED();
    hipLaunchKernelGGL(k_keys, dim3(grid), dim3(kKnnBlock), 0, st, dpos, (long long)n,
                       (const KGrid*)dg, kin, iin);
    ASP_LAUNCHED();
    size_t tmp = 0;
    ASP_HIP(rocprim::radix_sort_pairs(nullptr, tmp, kin, kout, iin, iout, (size_t)n, 0, 3 * kQBits,
                                      st));
    ASP_TRY(ensure(ws.knn[6], tmp));
    ASP_HIP(rocprim::radix_sort_pairs(ws.knn[6].p, tmp, kin, kout, iin, iout, (size_t)n, 0,
                                      3 * kQBits, st));
    hipLaunchKernelGGL(k_gather, dim3(grid), dim3(kKnnBlock), 0, st, dpos, (long long)n,
                       (const int*)iout, xs, ys, zs);
    ASP_LAUNCHED();
    if (k <= 32)
        hipLaunchKernelGGL(k_knn<32>, dim3(grid), dim3(kKnnBlock), 0, st, (const double*)xs,
                           (const double*)ys, (const double*)zs, (const unsigned long long*)kout,
                           (const int*)iout, (long long)n, k, (const KGrid*)dg, dh);
    else
        hipLaunchKernelGGL(k_knn<64>, dim3(grid), dim3(kKnnBlock), 0, st, (const double*)xs,
                           (const double*)ys, (const double*)zs, (const unsigned long long*)kout,
                           (const int*)iout, (long long)n, k, (const KGrid*)dg, dh);
    ASP_LAUNCHED();
    if (!dev) {
        ASP_HIP(hipMemcpyAsync(h, dh, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    return ASP_OK;
}

}  // namespace asp

using namespace asp;

extern "C" int asp_knn_smoothing_lengths(const double* positions, int64_t n, int32_t k,
                                         double* h, int32_t flags, int32_t device,
                                         void* stream) {
    t_err.clear();
    return knn(positions, n, k, h, flags, device, (hipStream_t)stream);
}
