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
// bounding cube; rocPRIM radix sort), positions gathered into sorted fp64 SoA.  One wave
// takes 64 consecutive particles of the curve (k_knn_wave):
//   1. the curve window of W = 64 entries either side is streamed once per wave through
//      LDS (coalesced), every lane testing every entry; candidates below a lane's k-th
//      distance so far are buffered in registers and merged into its register top-k a
//      few at a time (the O(k) insertion does not run per candidate for the whole wave);
//   2. each lane then checks its ball (radius = its k-th distance so far) against the
//      cells of edge >= half that radius: cells whose Morton key range lies inside the
//      window's span are complete; any other cell the ball reaches is scanned by the
//      lane (binary-searched key range, minus the window).
// The k-th smallest d2 over a superset of the ball is the exact answer.  (k_knn: the
// one-lane-per-particle form, kept as a diagnostic; DESIGN.md §12 has the measurements.)
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/asp.h"
#include "asp_host.hpp"

namespace asp {

constexpr int kKnnBlock = 256;
#ifndef ASP_KNN_QBITS
#define ASP_KNN_QBITS 21
#endif
constexpr int kQBits = ASP_KNN_QBITS;            // quantisation bits per axis
constexpr int kKeyBits = 3 * kQBits;             // Morton key bits (keys < 2^kKeyBits)
constexpr long long kQMax = (1LL << kQBits) - 1;
static_assert(kQBits >= 12 && kQBits <= 21, "3 x kQBits key bits in 64; >= the tables' 12 levels");
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

// The k smallest d2 seen, in registers (static indexing only), kept sorted ascending in
// the LAST k of K slots (the first K - k hold -inf and never move), so the k-th smallest is
// v[K - 1].  Inserting d (< v[K - 1]) is a branch-free merge step:
//   v'[q] = min(v[q], max(v[q - 1], d)),  v[-1] = -inf
// = the q-th smallest of v and d (v[q] if d > v[q], else max(v[q - 1], d)): 2K min / max.
// v_min_f64 / v_max_f64 as plain instructions.  fmin / fmax lower to the same instructions
// plus a v_max_f64 x, x quieting each loop-carried operand (IEEE mode: a signalling NaN
// must not pass through), a third instruction per slot of the insertion.  The top-k never
// holds a NaN (insert() admits only d < mx), so the quieting is dead weight.
__device__ __forceinline__ double hw_min(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double hw_max(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

typedef float kf2 __attribute__((ext_vector_type(2)));  // packed fp32 pair (v_pk_* ops)
typedef float kf4 __attribute__((ext_vector_type(4)));

template <int K>
struct TopK {
    double v[K];
    double mx;  // the k-th smallest so far (+inf until k values are in)
    int nins;   // insertions (diagnostic counter, ASP_KNN_COUNT)
    __device__ __forceinline__ void init(int k) {
#pragma unroll
        for (int q = 0; q < K; ++q) v[q] = q < K - k ? -INFINITY : INFINITY;
        mx = INFINITY;
        nins = 0;
    }
    __device__ __forceinline__ void insert(double d) {
        if (!(d < mx)) return;
        ++nins;
#pragma unroll
        for (int q = K - 1; q > 0; --q) v[q] = hw_min(v[q], hw_max(v[q - 1], d));
        v[0] = hw_min(v[0], d);
        mx = v[K - 1];
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

// Cell table of one Morton level L (the finest level with about one particle per cell):
// tab[c] = the first sorted index whose key lies in cell c or later (c < 8^L), tab[8^L] = n.
// A cell of any level <= L is then a range [tab[.], tab[.]) by two loads instead of two
// binary searches over the whole array.  The grid spans the bounding cube, so in a
// centrally concentrated set the level-L cells of the dense part hold thousands of
// particles (10^7 Plummer: median 5400 per particle's cell at L = 8); a level-L cell with
// more than kSubMin particles gets a sub-table over its 8^3 cells three levels down
// (same form: the first index of each sub-cell, entry 512 = the cell's end), so a finer
// cell is two table loads plus a binary search inside its sub-cell (median 11 particles
// at L + 3) instead of one over the whole level-L cell.
constexpr int kSubLevels = 3;
constexpr int kSubCells = 1 << (3 * kSubLevels);  // 512 sub-cells per sub-table
constexpr int kSubMin = 64;                       // level-L cells above this get one
struct CellTab {
    const int* tab;
    const int* sub;     // per level-L cell: its sub-table, or -1
    const int* subtab;  // sub-tables, kSubCells + 1 entries each
    int sh;  // kKeyBits - 3 L: key >> sh = the level-L cell
};

// Built in two steps (round 5): each occupied cell's first particle writes its index, then a
// suffix minimum over the table (initialised to n) gives every empty cell the next occupied
// cell's start.  The round-4 form had each particle write the empty cells before its own,
// so the particle after a long empty stretch of the bounding cube wrote millions of entries
// on its own (3.5 ms of the 10^7 k-NN's 4.8-ms set-up).
__global__ __launch_bounds__(kKnnBlock) void k_cell_starts(const unsigned long long* __restrict__ keys,
                                                            long long n, int sh, int* __restrict__ tab) {
    long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (i >= n) return;
    const long long c = (long long)(keys[i] >> sh);
    if (i == 0 || (long long)(keys[i - 1] >> sh) != c) tab[c] = (int)i;
}

// Suffix minimum of v[0, m): blocks of kSfxPer x kSfxBlock entries.  k_sfx_block forms the
// block-local suffix minima in place and the block's minimum; k_sfx_top the suffix minima
// of those (one workgroup); k_sfx_apply folds the next blocks' minimum into each block.
constexpr int kSfxBlock = 1024, kSfxPer = 4, kSfxSpan = kSfxBlock * kSfxPer;
__device__ __forceinline__ int block_suffix_min(int x, int* sh) {  // min over threads >= t
    const int t = threadIdx.x;
    sh[t] = x;
    __syncthreads();
    for (int d = 1; d < kSfxBlock; d <<= 1) {
        const int y = t + d < kSfxBlock ? sh[t + d] : INT_MAX;
        __syncthreads();
        x = min(x, y);
        sh[t] = x;
        __syncthreads();
    }
    return x;
}
__global__ __launch_bounds__(kSfxBlock) void k_sfx_block(int* __restrict__ v, long long m,
                                                          int* __restrict__ bmin) {
    __shared__ int sh[kSfxBlock];
    const long long j0 = (long long)blockIdx.x * kSfxSpan + (long long)threadIdx.x * kSfxPer;
    int e[kSfxPer];
#pragma unroll
    for (int q = 0; q < kSfxPer; ++q) e[q] = j0 + q < m ? v[j0 + q] : INT_MAX;
#pragma unroll
    for (int q = kSfxPer - 2; q >= 0; --q) e[q] = min(e[q], e[q + 1]);
    const int incl = block_suffix_min(e[0], sh);                        // this and later threads
    const int later = threadIdx.x + 1 < kSfxBlock ? sh[threadIdx.x + 1] : INT_MAX;
#pragma unroll
    for (int q = 0; q < kSfxPer; ++q)
        if (j0 + q < m) v[j0 + q] = min(e[q], later);
    if (threadIdx.x == 0) bmin[blockIdx.x] = incl;
}
__global__ __launch_bounds__(kSfxBlock) void k_sfx_top(int* __restrict__ bmin, int nb) {
    __shared__ int sh[kSfxBlock];
    int carry = INT_MAX;  // minimum of the chunks after this one
    for (int c0 = ((nb - 1) / kSfxBlock) * kSfxBlock; c0 >= 0; c0 -= kSfxBlock) {
        const int j = c0 + (int)threadIdx.x;
        const int x = j < nb ? bmin[j] : INT_MAX;
        const int s = min(block_suffix_min(x, sh), carry);
        if (j < nb) bmin[j] = s;
        carry = min(carry, sh[0]);
        __syncthreads();
    }
}
__global__ __launch_bounds__(kSfxBlock) void k_sfx_apply(int* __restrict__ v, long long m,
                                                          const int* __restrict__ bmin, int nb) {
    const int b = blockIdx.x;
    if (b + 1 >= nb) return;
    const int nx = bmin[b + 1];
    const long long j0 = (long long)b * kSfxSpan + (long long)threadIdx.x * kSfxPer;
#pragma unroll
    for (int q = 0; q < kSfxPer; ++q)
        if (j0 + q < m) v[j0 + q] = min(v[j0 + q], nx);
}

// Sub-table slots of the dense level-L cells (slot order does not matter).
__global__ __launch_bounds__(kKnnBlock) void k_sub_slots(const int* __restrict__ tab, long long ncell,
                                                          int submin, int* __restrict__ sub,
                                                          int* __restrict__ nslot) {
    long long c = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (c >= ncell) return;
    sub[c] = tab[c + 1] - tab[c] > submin ? atomicAdd(nslot, 1) : -1;
}

// Per particle of a dense cell: the sub-cells starting at it (as k_cell_table), and the
// cell's last particle closes the table.
__global__ __launch_bounds__(kKnnBlock) void k_sub_table(const unsigned long long* __restrict__ keys,
                                                          long long n, int sh,
                                                          const int* __restrict__ tab,
                                                          const int* __restrict__ sub,
                                                          int* __restrict__ subtab) {
    long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (i >= n) return;
    const long long c = (long long)(keys[i] >> sh);
    const int s = sub[c];
    if (s < 0) return;
    const int sh2 = sh - 3 * kSubLevels;
    int* st = subtab + (long long)s * (kSubCells + 1);
    const int q = (int)((keys[i] >> sh2) & (kSubCells - 1));
    const int first = tab[c], end = tab[c + 1];
    const int qp = i == first ? -1 : (int)((keys[i - 1] >> sh2) & (kSubCells - 1));
    for (int r = qp + 1; r <= q; ++r) st[r] = (int)i;
    if (i == end - 1)
        for (int r = q + 1; r <= kSubCells; ++r) st[r] = end;
}

// First index with key >= k0 (k0 < 2^kKeyBits), through the tables.
__device__ __forceinline__ long long cell_lower(const unsigned long long* __restrict__ keys,
                                                long long n, const CellTab& T,
                                                unsigned long long k0) {
    const long long c = (long long)(k0 >> T.sh);
    const long long a = T.tab[c];
    if ((unsigned long long)c << T.sh == k0) return a;  // k0 starts a level-L cell
    const int s = T.sub[c];
    if (s >= 0) {
        const int sh2 = T.sh - 3 * kSubLevels;
        const int* st = T.subtab + (long long)s * (kSubCells + 1);
        const int q = (int)((k0 >> sh2) & (kSubCells - 1));
        const long long a2 = st[q];
        if ((k0 >> sh2) << sh2 == k0) return a2;  // k0 starts a sub-cell
        return a2 + lower_bound(keys + a2, st[q + 1] - a2, k0);
    }
    const long long b = T.tab[c + 1];
    return a + lower_bound(keys + a, b - a, k0);
}

// Two lookups (the ends of one key range) with their loads interleaved: the table, slot and
// sub-table loads of both issued together, then both binary searches in lock step -- one
// chain of dependent loads instead of two.  Same results as cell_lower.
__device__ __forceinline__ void cell_lower2(const unsigned long long* __restrict__ keys, long long n,
                                            const CellTab& T, unsigned long long k0,
                                            unsigned long long k1, long long& j0, long long& j1) {
    const long long c0 = (long long)(k0 >> T.sh), c1 = (long long)(k1 >> T.sh);
    const long long a0 = T.tab[c0], a1 = T.tab[c1];
    const long long e0 = T.tab[c0 + 1], e1 = T.tab[c1 + 1];
    const int s0 = T.sub[c0], s1 = T.sub[c1];
    const int sh2 = T.sh - 3 * kSubLevels;
    const bool al0 = (unsigned long long)c0 << T.sh == k0, al1 = (unsigned long long)c1 << T.sh == k1;
    long long lo0 = a0, len0 = al0 ? 0 : e0 - a0, lo1 = a1, len1 = al1 ? 0 : e1 - a1;
    if (!al0 && s0 >= 0) {
        const int* st = T.subtab + (long long)s0 * (kSubCells + 1);
        const int q = (int)((k0 >> sh2) & (kSubCells - 1));
        lo0 = st[q];
        len0 = (k0 >> sh2) << sh2 == k0 ? 0 : st[q + 1] - lo0;
    }
    if (!al1 && s1 >= 0) {
        const int* st = T.subtab + (long long)s1 * (kSubCells + 1);
        const int q = (int)((k1 >> sh2) & (kSubCells - 1));
        lo1 = st[q];
        len1 = (k1 >> sh2) << sh2 == k1 ? 0 : st[q + 1] - lo1;
    }
    while (len0 > 0 || len1 > 0) {
        const long long h0 = len0 >> 1, h1 = len1 >> 1;
        const unsigned long long v0 = len0 > 0 ? keys[lo0 + h0] : 0ULL;
        const unsigned long long v1 = len1 > 0 ? keys[lo1 + h1] : 0ULL;
        if (len0 > 0) {
            if (v0 < k0) {
                lo0 += h0 + 1;
                len0 -= h0 + 1;
            } else {
                len0 = h0;
            }
        }
        if (len1 > 0) {
            if (v1 < k1) {
                lo1 += h1 + 1;
                len1 -= h1 + 1;
            } else {
                len1 = h1;
            }
        }
    }
    j0 = lo0;
    j1 = lo1;
}

// The whole search for particle i by one lane: returns its k-th smallest d2.
template <int K>
__device__ __forceinline__ double knn_thread(long long i, const double* __restrict__ xs,
                                             const double* __restrict__ ys,
                                             const double* __restrict__ zs,
                                             const unsigned long long* __restrict__ keys,
                                             long long n, int k, const KGrid& G) {
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
            const unsigned long long pre = sh >= kKeyBits ? 0ULL : key >> sh;
            auto same = [&](long long j) { return sh >= kKeyBits || (keys[j] >> sh) == pre; };
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
                        unsigned long long k0 = sh3 >= kKeyBits ? 0ULL : p << sh3;
                        unsigned long long k1 = sh3 >= kKeyBits ? ~0ULL : (p + 1) << sh3;
                        long long j0 = lower_bound(keys, n, k0);
                        long long j1 = sh3 >= kKeyBits ? n : lower_bound(keys + j0, n - j0, k1) + j0;
                        // [w0, w1) is in already
                        for (long long j = j0; j < std::min(j1, w0); ++j)
                            T.insert(dist2(x, y, z, xs[j], ys[j], zs[j]));
                        for (long long j = std::max(j0, w1); j < j1; ++j)
                            T.insert(dist2(x, y, z, xs[j], ys[j], zs[j]));
                    }
        }
    }
    return T.mx;
}

template <int K>
__global__ __launch_bounds__(kKnnBlock) void k_knn(const double* __restrict__ xs,
                                                   const double* __restrict__ ys,
                                                   const double* __restrict__ zs,
                                                   const unsigned long long* __restrict__ keys,
                                                   const int* __restrict__ idx, long long n,
                                                   int k, const KGrid* __restrict__ g,
                                                   double* __restrict__ h) {
    long long i = (long long)blockIdx.x * kKnnBlock + threadIdx.x;
    if (i >= n) return;
    const KGrid G = *g;
    h[idx[i]] = sqrt(knn_thread<K>(i, xs, ys, zs, keys, n, k, G));
}

// ----------------------------------------------------------------------------------
// Wave-cooperative search: one wave takes 64 consecutive particles of the Morton order
// (spatially compact).
//   1. The curve window [base - W, base + 64 + W) is streamed ONCE per wave: 64 coalesced
//      loads into LDS per chunk, each lane testing the 64 entries against its own
//      particle (LDS broadcast reads).  Candidates below a lane's current k-th distance go
//      to a small register buffer, merged into the top-k when some lane's buffer is full,
//      so the O(k) insertion runs a few times per chunk, not per candidate for the wave.
//   2. Each lane then checks its ball (radius = its k-th distance so far, plus slack)
//      against the cells of the level with edge >= that radius: a cell whose key range
//      lies strictly inside the window's key span is complete already; any other cell the
//      ball reaches is scanned by the lane alone (binary-searched range minus the window).
// Exact: every particle within the final k-th distance is in the window or in a scanned
// cell.  Far from jumps of the curve the window covers the whole ball and step 2 scans
// nothing.
// ----------------------------------------------------------------------------------
constexpr int kBufSlots = 8;
constexpr int kWinHalf = 256;  // W: curve window each side of the wave (round 6, with the shared pass: 64-448 swept)
constexpr int kCellFine = 1;   // verification cells >= half the ball radius (swept: 0-3)
constexpr int kWindowF32 = 1;  // the window pass with the fp32 prefilter (wave_scan32)
constexpr bool kMaskTest = true;  // the entry test's form (wave_stream32 MASK)
constexpr int kUnionQ = 64;
constexpr int kNearFirst = 1;  // window chunks nearest first (wave_scan32_near)
#ifndef ASP_KNN_WGROUP
#define ASP_KNN_WGROUP 32
#endif
#ifndef ASP_KNN_UGROUP
#define ASP_KNN_UGROUP 64
#endif
constexpr int kWGroup = ASP_KNN_WGROUP;  // mask test: entries per candidate walk, window pass
constexpr int kUGroup = ASP_KNN_UGROUP;  // ... and shared pass     // the shared cell pass's lane quantile (of 64; 0: off)

template <int K>
struct Cand {
    TopK<K> T;
    double buf[kBufSlots];
    int cnt;
    __device__ __forceinline__ void push(double d) {  // d < T.mx already
#pragma unroll
        for (int q = 0; q < kBufSlots; ++q)
            if (q == cnt) buf[q] = d;
        ++cnt;
    }
    __device__ __forceinline__ void flush() {
#pragma unroll
        for (int q = 0; q < kBufSlots; ++q)
            if (q < cnt) T.insert(buf[q]);
        cnt = 0;
    }
};

template <int K>
__device__ __forceinline__ void wave_scan(long long a, long long b, const double* __restrict__ xs,
                                          const double* __restrict__ ys,
                                          const double* __restrict__ zs, double* lx, double* ly,
                                          double* lz, int lane, double x, double y, double z,
                                          Cand<K>& C) {
    for (long long c = a; c < b; c += 64) {
        const int m = (int)min(64LL, b - c);
        if (lane < m) {
            lx[lane] = xs[c + lane];
            ly[lane] = ys[c + lane];
            lz[lane] = zs[c + lane];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int q = 0; q < m; ++q) {
            double d = dist2(x, y, z, lx[q], ly[q], lz[q]);
            if (d < C.T.mx) C.push(d);
            if (__builtin_amdgcn_ballot_w64(C.cnt == kBufSlots)) C.flush();
        }
        __builtin_amdgcn_wave_barrier();  // the chunk is rewritten next
    }
}

// One lane's scan of sorted particles [a, b): four particles' coordinates are loaded
// before any of them is inserted, so the lane has 12 loads in flight instead of 3
// (57 -> 54 ms at 10^7; 8 or 16 at a time: 69-70 ms, register pressure).
constexpr int kScanUnroll = 4;
template <int K>
__device__ __forceinline__ void scan_range(long long a, long long b, const double* __restrict__ xs,
                                           const double* __restrict__ ys,
                                           const double* __restrict__ zs, double x, double y,
                                           double z, TopK<K>& T) {
    long long j = a;
    for (; j + kScanUnroll <= b; j += kScanUnroll) {
        double px[kScanUnroll], py[kScanUnroll], pz[kScanUnroll];
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
            px[u] = xs[j + u];
            py[u] = ys[j + u];
            pz[u] = zs[j + u];
        }
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) T.insert(dist2(x, y, z, px[u], py[u], pz[u]));
    }
    for (; j < b; ++j) T.insert(dist2(x, y, z, xs[j], ys[j], zs[j]));
}

// Wave reductions by DPP (quad_perm xor 1 / xor 2, row_half_mirror, row_mirror, then
// row_bcast15 / row_bcast31 into lane 63) and one v_readlane: six dependent VALU steps where
// __shfl_xor took six ds_bpermute round trips through LDS (the shared pass's cell
// enumeration reduces twice per column).  Every lane of the wave must be active; the result
// is uniform.
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(v, v, CTRL, RM, 0xf, false);
}
template <class Op>
__device__ __forceinline__ int wave_reduce_i(int v, Op op) {
    v = op(v, dpp_i<0xb1>(v));       // quad_perm [1, 0, 3, 2]
    v = op(v, dpp_i<0x4e>(v));       // quad_perm [2, 3, 0, 1]
    v = op(v, dpp_i<0x141>(v));      // row_half_mirror
    v = op(v, dpp_i<0x140>(v));      // row_mirror
    v = op(v, dpp_i<0x142, 0xa>(v)); // row_bcast15 into rows 1, 3
    v = op(v, dpp_i<0x143, 0xc>(v)); // row_bcast31 into rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ double dpp_d(double v, int which) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    int lo = (int)(unsigned)b, hi = (int)(unsigned)(b >> 32);
    switch (which) {
        case 0: lo = dpp_i<0xb1>(lo); hi = dpp_i<0xb1>(hi); break;
        case 1: lo = dpp_i<0x4e>(lo); hi = dpp_i<0x4e>(hi); break;
        case 2: lo = dpp_i<0x141>(lo); hi = dpp_i<0x141>(hi); break;
        case 3: lo = dpp_i<0x140>(lo); hi = dpp_i<0x140>(hi); break;
        case 4: lo = dpp_i<0x142, 0xa>(lo); hi = dpp_i<0x142, 0xa>(hi); break;
        default: lo = dpp_i<0x143, 0xc>(lo); hi = dpp_i<0x143, 0xc>(hi); break;
    }
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_max(double v) {  // v >= 0 or NaN-free
#pragma unroll
    for (int w = 0; w < 6; ++w) v = fmax(v, dpp_d(v, w));
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, 63);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), 63);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// The window pass with an fp32 prefilter.  Entries go to LDS twice: fp64 (for the exact
// distance) and fp32 relative to a wave origin O (lane 0's particle).  Every lane tests
// every entry in fp32, d32 = ((dx dx + dy dy) + dz dz) from fl32(x - O) - fl32(e - O),
// against a bound T that no pair with fp64 d < mx can exceed: with u = 2^-24 and M the
// largest |coordinate - O| of the chunk and the wave's particles, each fp32 difference is
// within 2.01 u M + 1.01 u |dx| of the exact one and the rounded sum within (1 + 5u), so
// d32 <= (1 + 5u) (sqrt(mx) (1 + 1.01u) + 3.49 u M)^2 < T := (sqrt(mx) (1 + 2^-22) +
// 2^-21 M)^2 (1 + 2^-21), rounded up to fp32.  Passing entries are buffered by LDS index
// (8 per lane); a flush computes their exact fp64 distances (the reference's expression)
// and inserts them -- lanes in step, so the fp64 work runs once per candidate, not once
// per entry for every lane whenever any lane has a candidate.  The buffer is flushed
// before the chunk's LDS is rewritten.  Results are the fp64 path's exactly (mx only
// shrinks, so a bound from an earlier mx stays valid).
// The stream is entries f = 0 .. nent - 1 of the sorted arrays, entry f at sorted index
// at(f) (-1: skip it -- its fp32 copy is NaN, which no bound passes); lanes with part false
// take no candidates (their bound is -1).
template <int K, bool MASK, int GRP, class At>
__device__ __forceinline__ void wave_stream32(long long nent, At at, const double* __restrict__ xs,
                                              const double* __restrict__ ys,
                                              const double* __restrict__ zs, double* lx, double* ly,
                                              double* lz, float* fx, float* fy, float* fz, int lane,
                                              double x, double y, double z, bool part, TopK<K>& T,
                                              bool fill = false, int sdiag = 0) {
    const double ox = __shfl(x, 0, 64), oy = __shfl(y, 0, 64), oz = __shfl(z, 0, 64);
    const double rx = x - ox, ry = y - oy, rz = z - oz;
    const float qx = (float)rx, qy = (float)ry, qz = (float)rz;
    const kf2 qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
    const double mq = wave_max(fmax(fabs(rx), fmax(fabs(ry), fabs(rz))));
    // chunk c + 64's entries are loaded (clamped index, unconditional loads) before chunk c
    // is tested, so the gathers' latency overlaps the tests
    auto entry = [&](long long c, int& g, double& ex, double& ey, double& ez) {
        g = c + lane < nent ? (int)at(c + lane) : -1;  // sorted indices < 2^31
        const int gi = g >= 0 ? g : 0;
        ex = xs[gi];
        ey = ys[gi];
        ez = zs[gi];
    };
    // (two chunks ahead measured slower: 18.81 vs 18.59 ms at 10^7, same box)
    int gn;
    double exn, eyn, ezn;
    entry(0, gn, exn, eyn, ezn);
    for (long long c = 0; c < nent; c += 64) {
        const int m = (int)min(64LL, nent - c);
        double me = 0.0;
        const int g = gn;
        const double ex = exn, ey = eyn, ez = ezn;
        if (c + 64 < nent) entry(c + 64, gn, exn, eyn, ezn);
        if (g >= 0) {
            lx[lane] = ex;
            ly[lane] = ey;
            lz[lane] = ez;
            const double dx = ex - ox, dy = ey - oy, dz = ez - oz;
            fx[lane] = (float)dx;
            fy[lane] = (float)dy;
            fz[lane] = (float)dz;
            me = fmax(fabs(dx), fmax(fabs(dy), fabs(dz)));
        } else {  // no entry (past the chunk's end, or skipped): NaN passes no bound
            fx[lane] = __builtin_nanf("");
            fy[lane] = 0.0f;
            fz[lane] = 0.0f;
        }
        const double M = fmax(mq, wave_max(me));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float Mf = (float)M * (1.0f + 0x1p-22f);  // >= M
        auto bound = [&]() -> float {
            if (!part) return -1.0f;
            if (!(T.mx < INFINITY)) return INFINITY;
            if (T.mx < 0x1p-100) {  // fp32 would lose the radius: the fp64 form
                const double r = sqrt(T.mx) * (1.0 + 0x1p-22) + 0x1p-21 * M;
                return (float)(r * r * (1.0 + 0x1p-21)) * (1.0f + 0x1p-22f);
            }
            // the same bound in fp32 (round 6): sqrt of fl32(mx) is within ~2^-23 of
            // sqrt(mx); widened by 2^-18 (and Mf >= M (1 + 2^-23)), the fp32 sum is >= the
            // fp64 form's (1 + 2^-22) sqrt(mx) + 2^-21 M, and its square times (1 + 2^-18)
            // >= that squared times (1 + 2^-21): never below the fp64 bound
            const float r = __builtin_amdgcn_sqrtf((float)T.mx) * (1.0f + 0x1p-18f) + 0x1p-21f * Mf;
            return r * r * (1.0f + 0x1p-18f);
        };
        float tb = bound();
        if constexpr (MASK) {
            // GRP entries at a time (16 / 32): their fp32 copies by 16-byte LDS reads
            // (every slot of the chunk is written, NaN past its end), the passing ones as a
            // bit mask, then each lane walks its own bits (exact fp64 distance, insert) --
            // the wave pays one walk per group in which any lane has a candidate
            static_assert(GRP == 16 || GRP == 32 || GRP == 64, "group of 16, 32 or 64 entries");
            int gstart = 0;
            if (fill && c == 0 && m >= K) {
                // the first K entries straight into the empty top-k (k == K: no -inf slots):
                // their exact distances (an entry without a particle, or a NaN distance,
                // as +inf -- what insert() would not take), sorted by a bitonic network
                // (K/2 log2 K (log2 K + 1)/2 compare-exchanges, 480 min / max for K = 32)
                // instead of K insertions of 2K min / max each
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    const double d = fx[q] == fx[q] ? dist2(x, y, z, lx[q], ly[q], lz[q]) : INFINITY;
                    T.v[q] = d < INFINITY ? d : INFINITY;
                }
#pragma unroll
                for (int sz = 2; sz <= K; sz <<= 1)
#pragma unroll
                    for (int st = sz >> 1; st > 0; st >>= 1)
#pragma unroll
                        for (int i = 0; i < K; ++i) {
                            const int j = i ^ st;
                            if (j > i) {
                                const double lo = hw_min(T.v[i], T.v[j]), hi = hw_max(T.v[i], T.v[j]);
                                const bool up = (i & sz) == 0;
                                T.v[i] = up ? lo : hi;
                                T.v[j] = up ? hi : lo;
                            }
                        }
                T.mx = T.v[K - 1];
                T.nins += K;
                tb = bound();
                gstart = K;
            }
            // sdiag (timing only): 1 = the chunks staged but not tested, 2 = tested, no walks
            // entries [off, off + 32) of the chunk (at most GRP) into a 32-bit mask
            auto test32 = [&](int off, int cnt, unsigned& pm) {
#pragma unroll 1
                for (int u = 0; u < cnt; u += 4) {
                    // entries (u, u + 1) and (u + 2, u + 3) as packed pairs
                    const kf4 X = *(const kf4*)(fx + off + u);
                    const kf4 Y = *(const kf4*)(fy + off + u);
                    const kf4 Z = *(const kf4*)(fz + off + u);
#pragma unroll
                    for (int v = 0; v < 4; v += 2) {
                        const kf2 ex = v == 0 ? X.xy : X.zw, ey = v == 0 ? Y.xy : Y.zw,
                                  ez = v == 0 ? Z.xy : Z.zw;
                        const kf2 dx = qx2 - ex, dy = qy2 - ey, dz = qz2 - ez;
                        // fused (v_pk_fma_f32): three roundings instead of five, inside the
                        // (1 + 5u) the bound allows for the sum of squares (same box, 10^7:
                        // 17.49-17.56 -> 17.10-17.17 ms)
                        const kf2 d = __builtin_elementwise_fma(
                            dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
                        pm |= (d.x <= tb ? 1u : 0u) << (u + v);
                        pm |= (d.y <= tb ? 1u : 0u) << (u + v + 1);
                    }
                }
            };
            // sdiag (timing only): 1 = the chunks staged but not tested, 2 = tested, no walks
            for (int g0 = sdiag == 1 ? m : gstart; g0 < m; g0 += GRP) {
                unsigned pm = 0, pm2 = 0;  // entries g0 + [0, 32), g0 + 32 + [0, 32) (GRP 64)
                test32(g0, GRP < 32 ? GRP : 32, pm);
                if (GRP == 64 && g0 + 32 < m) test32(g0 + 32, 32, pm2);
                if (sdiag == 2) {
                    asm volatile("" ::"v"(pm), "v"(pm2));
                    pm = pm2 = 0;
                }
                if (__builtin_amdgcn_ballot_w64((pm | pm2) != 0)) {
                    while (pm | pm2) {
                        int q;
                        if (pm) {
                            q = g0 + __builtin_ctz(pm);
                            pm &= pm - 1;
                        } else {
                            q = g0 + 32 + __builtin_ctz(pm2);
                            pm2 &= pm2 - 1;
                        }
                        T.insert(dist2(x, y, z, lx[q], ly[q], lz[q]));
                    }
                    tb = bound();
                }
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        int ib[kBufSlots];
        int cnt = 0;
        auto flush = [&]() {
#pragma unroll
            for (int q = 0; q < kBufSlots; ++q)
                if (q < cnt) T.insert(dist2(x, y, z, lx[ib[q]], ly[ib[q]], lz[ib[q]]));
            cnt = 0;
        };
        for (int q = 0; q < m; ++q) {
            const float dx = qx - fx[q], dy = qy - fy[q], dz = qz - fz[q];
            const float d32 = (dx * dx + dy * dy) + dz * dz;
            if (d32 <= tb) {
#pragma unroll
                for (int t = 0; t < kBufSlots; ++t)
                    if (t == cnt) ib[t] = q;
                ++cnt;
            }
            if (__builtin_amdgcn_ballot_w64(cnt == kBufSlots)) {
                flush();
                tb = bound();
            }
        }
        flush();  // the chunk is rewritten next
        __builtin_amdgcn_wave_barrier();
    }
}

template <int K, bool MASK>
__device__ __forceinline__ void wave_scan32(long long a, long long b, const double* __restrict__ xs,
                                            const double* __restrict__ ys,
                                            const double* __restrict__ zs, double* lx, double* ly,
                                            double* lz, float* fx, float* fy, float* fz, int lane,
                                            double x, double y, double z, TopK<K>& T) {
    wave_stream32<K, MASK, kWGroup>(b - a, [&](long long f) { return a + f; }, xs, ys, zs, lx, ly, lz,
                                    fx, fy, fz, lane, x, y, z, true, T);
}

// The window [a, b) around the wave's own 64 particles [base, base + 64), streamed
// nearest chunks first: the wave's own chunk, then the chunks 64 below and above it, then
// 128 below and above, ...  In random order a lane's top-k takes about k (1 + ln(N / k))
// insertions for N entries; curve neighbours first, its k-th distance falls early and
// fewer of the later entries pass.
template <int K, bool MASK>
__device__ __forceinline__ void wave_scan32_near(long long a, long long b, long long base,
                                                 const double* __restrict__ xs,
                                                 const double* __restrict__ ys,
                                                 const double* __restrict__ zs, double* lx,
                                                 double* ly, double* lz, float* fx, float* fy,
                                                 float* fz, int lane, double x, double y, double z,
                                                 TopK<K>& T, bool fill) {
    const long long below = (base - a + 63) >> 6, above = (b - base - 1) >> 6;  // chunks each side
    const long long nch = 1 + 2 * max(below, above);
    wave_stream32<K, MASK, kWGroup>(nch * 64, [&](long long f) -> long long {
        const long long j = f >> 6, o = f & 63;
        const long long s = j == 0 ? 0 : (j & 1 ? -((j + 1) >> 1) : (j >> 1));  // 0, -1, +1, -2, +2, ...
        const long long g = base + s * 64 + o;
        return g >= a && g < b ? g : -1;
    }, xs, ys, zs, lx, ly, lz, fx, fy, fz, lane, x, y, z, true, T, fill);
}

__device__ __forceinline__ int wave_min_i(int v) {
    return wave_reduce_i(v, [](int a, int b) { return min(a, b); });
}
__device__ __forceinline__ int wave_max_i(int v) {
    return wave_reduce_i(v, [](int a, int b) { return max(a, b); });
}
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// The shared cell pass (round 6).  Each lane's cell pass below looks up and scans its own
// cells, one dependent load chain after another, while the other lanes of the wave, whose
// balls overlap its own, look up the same cells.  Here the wave takes the cells ONCE:
//   * a common level: the finest level whose edge is >= half the ball radius for uq / 64 of
//     the lanes (the others keep their own pass: one loose radius must not coarsen the
//     cells for all);
//   * the cells of that level meeting any such lane's ball (the per-lane test, ballot) and
//     not inside the window's key span, listed in LDS;
//   * their index ranges looked up by the lanes in parallel (64 lookups in flight), prefix
//     offsets formed by a wave scan;
//   * the concatenated ranges streamed once through LDS with the window pass's fp32
//     prefilter (indices inside the window skipped: they are in already).
// Exact for the same reason as the per-lane pass: any level's cells meeting a ball cover it.
constexpr int kUCells = 512;      // cells listed per wave (LDS); more: the per-lane pass
constexpr int kUScan = 4096;      // cells of the common box tested per wave at most
constexpr int kUMaxEnt = (1 << 16) - 1;  // entries streamed per wave at most (16-bit la)

#ifndef ASP_KNN_WPE
#define ASP_KNN_WPE 0  // waves per SIMD the search is compiled for (0: the compiler's choice)
#endif
#if ASP_KNN_WPE
#define ASP_KNN_OCC __attribute__((amdgpu_waves_per_eu(ASP_KNN_WPE)))
#else
#define ASP_KNN_OCC
#endif
template <int K, bool MASK>
__global__ __launch_bounds__(kKnnBlock, (K == 32 ? 3 : 1)) ASP_KNN_OCC void k_knn_wave(const double* __restrict__ xs,
                                                        const double* __restrict__ ys,
                                                        const double* __restrict__ zs,
                                                        const unsigned long long* __restrict__ keys,
                                                        const int* __restrict__ idx, long long n,
                                                        int k, const KGrid* __restrict__ g,
                                                        double* __restrict__ h, int diag,
                                                        int whalf, int fine, CellTab CT,
                                                        int f32, int uq, int near, int fill,
                                                        unsigned long long* evc) {
    __shared__ double sx[kKnnBlock / 64][64], sy[kKnnBlock / 64][64], sz[kKnnBlock / 64][64];
    __shared__ __attribute__((aligned(16))) float fx[kKnnBlock / 64][64], fy[kKnnBlock / 64][64],
        fz[kKnnBlock / 64][64];
    __shared__ unsigned long long ucl[kKnnBlock / 64][kUCells];  // shared pass: range keys, then (offset, start)
    __shared__ unsigned short ucn[kKnnBlock / 64][kUCells];      // ... cells per key range
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long base = ((long long)blockIdx.x * (kKnnBlock / 64) + wv) * 64;
    if (base >= n) return;  // wave-uniform
    const long long i = base + lane;
    const bool act = i < n;
    const long long ic = act ? i : n - 1;  // idle lanes shadow the last particle, write nothing
    const KGrid G = *g;
    const double x = xs[ic], y = ys[ic], z = zs[ic];
    Cand<K> C;
    C.T.init(k);
    C.cnt = 0;
    const long long win0 = max(0LL, base - whalf), win1 = min(n, base + 64 + whalf);
    if (f32) {
        if (near)
            wave_scan32_near<K, MASK>(win0, win1, base, xs, ys, zs, sx[wv], sy[wv], sz[wv], fx[wv],
                                      fy[wv], fz[wv], lane, x, y, z, C.T, fill && k == K);
        else
            wave_scan32<K, MASK>(win0, win1, xs, ys, zs, sx[wv], sy[wv], sz[wv], fx[wv], fy[wv],
                                 fz[wv], lane, x, y, z, C.T);
    } else {
        wave_scan<K>(win0, win1, xs, ys, zs, sx[wv], sy[wv], sz[wv], lane, x, y, z, C);
        C.flush();
    }
    // key span the window covers completely (open at the ends of the array)
    const unsigned long long klo = win0 == 0 ? 0ULL : keys[win0] + 1;
    const unsigned long long khi = win1 == n ? ~0ULL : keys[win1 - 1];
    bool shared = false;  // this lane's ball is covered by the shared cell pass
    // diag (timing only, wrong results): 2 = the shared pass's cell list and lookups without
    // its stream, 3 = the shared pass without the per-lane pass, 4 = the cell list alone,
    // 5 = the stream's chunks staged but not tested, 6 = tested without candidate walks
    if (uq > 0 && f32 && n >= k && (diag == 0 || diag >= 2)) {  // wave-uniform
        const bool ok = act && C.T.mx < INFINITY;
        const double R = sqrt(C.T.mx) * (1.0 + 0x1p-40);
        int sft = 99;  // this lane's own cell level (as the per-lane pass)
        if (ok) {
            int e;
            frexp(R * G.scale + 1.0, &e);
            sft = max(0, min(e, kQBits) - fine);
        }
        const int nact = __popcll(__ballot(ok));
        if (nact > 0) {
            const int need = (nact * uq + 63) >> 6;
            int sw = wave_min_i(sft);
            while (__popcll(__ballot(ok && sft <= sw)) < need) ++sw;
            const bool rg = ok && sft <= sw;
            const double c3[3] = {x, y, z};
            // the common box of cells (uniform: scalar loops), this lane's position and
            // squared radius in quanta (the per-lane pass's slack: one quantum per cell face)
            int A[3], B[3];
            double tq[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const int lo = (int)(max(0LL, quant(c3[a] - R, G.lo[a], G.scale) - 1) >> sw);
                const int hi = (int)(min(kQMax, quant(c3[a] + R, G.lo[a], G.scale) + 1) >> sw);
                A[a] = __builtin_amdgcn_readfirstlane(wave_min_i(rg ? lo : INT_MAX));
                B[a] = __builtin_amdgcn_readfirstlane(wave_max_i(rg ? hi : -1));
                tq[a] = (c3[a] - G.lo[a]) * G.scale;
            }
            const double r2q = rg ? C.T.mx * G.scale * G.scale * (1.0 + 0x1p-36) : -1.0;
            const double ed = (double)(1 << sw), ied = 1.0 / ed;  // cell edge in quanta (a power of two)
            // distance (quanta) from this lane's particle to the slab of cell cc on axis a,
            // the cell widened by one quantum each side
            auto gapq = [&](int a, int cc) {
                const double l = (double)cc * ed - 1.0 - tq[a], h = tq[a] - ((double)cc + 1.0) * ed - 1.0;
                return fmax(fmax(l, h), 0.0);
            };
            const int sh3 = 3 * sw;
            int nc = 0, ncol = 0;
            // cells p with k0 = p << sh3 >= klo and k1 = (p + 1) << sh3 <= khi lie inside the
            // window's key span: p >= ceil(klo / 2^sh3), p < floor(khi / 2^sh3)
            const unsigned long long plo = sh3 >= kKeyBits ? 1ULL : (klo >> sh3) + ((klo & ((1ULL << sh3) - 1)) != 0);
            const unsigned long long phi = sh3 >= kKeyBits ? 0ULL : (khi >> sh3);
            bool ovf = (long long)(B[0] - A[0] + 1) * (B[1] - A[1] + 1) > kUScan;
            for (int cx = A[0]; cx <= B[0] && !ovf; ++cx) {
                const double gx = gapq(0, cx), sx2 = gx * gx;
                if (!__ballot(sx2 <= r2q)) continue;
                for (int cy = A[1]; cy <= B[1] && !ovf; ++cy) {
                    ++ncol;
                    const double gy = gapq(1, cy), s2 = sx2 + gy * gy;
                    // this lane's cells of the column: gap_z^2 <= r2q - s2, i.e. cz in
                    // [(t - 1 - w) / ed - 1, (t + 1 + w) / ed], w = sqrt(r2q - s2) (fp32,
                    // widened by 2^-18 relative + 2 quanta)
                    int z0 = INT_MAX, z1 = -1;
                    if (s2 <= r2q) {
                        const double w = (double)(__builtin_amdgcn_sqrtf((float)(r2q - s2)) * (1.0f + 0x1p-18f)) + 2.0;
                        z0 = (int)floor((tq[2] - 1.0 - w) * ied) - 1;  // ied = 1 / ed exactly
                        z1 = (int)floor((tq[2] + 1.0 + w) * ied);
                    }
                    const int cz0 = max(A[2], __builtin_amdgcn_readfirstlane(wave_min_i(z0)));
                    const int cz1 = min(B[2], __builtin_amdgcn_readfirstlane(wave_max_i(z1)));
                    // the column's cells, one per lane: Morton code, the window test, and
                    // the key-adjacent (even z, z + 1) pairs merged into one range -- the
                    // only cells of a column adjacent in key order (z is the lowest bit)
                    const unsigned long long pxy = (spread21(cx) << 2) | (spread21(cy) << 1);
                    for (int zb = cz0; zb <= cz1 && !ovf; zb += 64) {
                        const int cz = zb + lane;
                        const unsigned long long p = pxy | spread21(cz);
                        const bool inc = cz <= cz1 && !(p >= plo && p < phi);
                        const unsigned long long I = __ballot(inc);
                        const bool prev = lane > 0 && ((I >> (lane - 1)) & 1);
                        const bool next = lane < 63 && ((I >> (lane + 1)) & 1);
                        const bool start = inc && !((cz & 1) && prev);
                        const unsigned long long S = __ballot(start);
                        const int idx = nc + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(S >> 32),
                                                                         __builtin_amdgcn_mbcnt_lo((unsigned)S, 0u));
                        const int cnt = __popcll(S);
                        if (nc + cnt > kUCells) {
                            ovf = true;
                            break;
                        }
                        if (start) {
                            ucl[wv][idx] = sh3 >= kKeyBits ? 0ULL : p << sh3;
                            ucn[wv][idx] = (unsigned short)(1 + ((cz & 1) == 0 && next));
                        }
                        nc += cnt;
                    }
                }
            }
            if (evc && lane == 0) {  // diagnostic: columns and list entries of the shared pass
                atomicAdd(&evc[4], (unsigned long long)ncol);
                atomicAdd(&evc[5], (unsigned long long)nc);
                atomicAdd(&evc[6], 1ULL);
            }
            long long tot = 0;
            if (!ovf && nc > 0 && diag != 4) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // lookups, 64 entries at a time: each entry's index range minus the window,
                // as the part below it (la entries from j0) and the part above it (from
                // max(j0, win1)); entry = offset << 47 | la << 31 | j0
                for (int c0 = 0; c0 < nc; c0 += 64) {
                    const int c = c0 + lane;
                    long long j0 = 0, la = 0, len = 0;
                    if (c < nc) {
                        const unsigned long long k0 = ucl[wv][c];
                        const unsigned long long span = (unsigned long long)ucn[wv][c] << sh3;
                        const unsigned long long k1 = sh3 >= kKeyBits ? ~0ULL : k0 + span;
                        long long j1;
                        if (sh3 >= kKeyBits || (k1 >> kKeyBits)) {  // the range runs to the end of the keys
                            j0 = cell_lower(keys, n, CT, k0);
                            j1 = n;
                        } else {
                            cell_lower2(keys, n, CT, k0, k1, j0, j1);
                        }
                        la = max(0LL, min(j1, win0) - j0);
                        len = la + max(0LL, j1 - max(j0, win1));
                    }
                    const int l32 = (int)min(len, (long long)kUMaxEnt + 1);
                    const long long incl = tot + wave_incl_scan(l32, lane);
                    if (c < nc)
                        ucl[wv][c] = ((unsigned long long)min(incl - l32, (long long)kUMaxEnt + 1) << 47) |
                                     ((unsigned long long)min(la, 0xffffLL) << 31) | (unsigned long long)j0;
                    tot = __shfl(incl, 63, 64);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (!ovf && tot <= kUMaxEnt && diag != 2 && diag != 4) {
                const unsigned long long* L = ucl[wv];
                int cur = 0;  // this lane's range of its previous entry (entries come in order)
                auto at = [&](long long f) -> long long {  // the last range starting at or before f
                    // exponential search forward from the previous entry's range (a chunk
                    // advances a lane by 64 entries, a few ranges), then binary search
                    int lo = cur, step = 1;
                    while (lo + step < nc && (long long)(L[lo + step] >> 47) <= f) {
                        lo += step;
                        step <<= 1;
                    }
                    int hi = min(lo + step, nc) - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if ((long long)(L[mid] >> 47) <= f) lo = mid;
                        else hi = mid - 1;
                    }
                    cur = lo;
                    const unsigned long long e = L[lo];
                    const long long o = f - (long long)(e >> 47), la = (long long)((e >> 31) & 0xffff);
                    const long long j0 = (long long)(e & 0x7fffffffULL);
                    return o < la ? j0 + o : max(j0, win1) + (o - la);
                };
                wave_stream32<K, MASK, kUGroup>(tot, at, xs, ys, zs, sx[wv], sy[wv], sz[wv], fx[wv], fy[wv], fz[wv],
                                 lane, x, y, z, rg, C.T, false, diag >= 5 ? diag - 4 : 0);
                shared = rg;
                if (evc && lane == 0) atomicAdd(&evc[2], (unsigned long long)tot);
            }
        }
    }
    if (act && !shared && n >= k && diag == 0) {
        const double R = sqrt(C.T.mx) * (1.0 + 0x1p-40);
        int e;
        frexp(R * G.scale + 1.0, &e);  // cell edge 2^shift >= R + 1 quantum ...
        const int shift = max(0, min(e, kQBits) - fine), sh3 = 3 * shift;  // ... / 2^fine
        const double c3[3] = {x, y, z};
        long long ca[3], cb[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            ca[a] = max(0LL, quant(c3[a] - R, G.lo[a], G.scale) - 1) >> shift;
            cb[a] = min(kQMax, quant(c3[a] + R, G.lo[a], G.scale) + 1) >> shift;
        }
        long long pj1 = 0;           // the last lookup's end index ...
        unsigned long long pk1 = 1;  // ... and key (1: none yet -- no range ends there)
        long long nscan = 0;         // ASP_KNN_COUNT: fp64 distances of the cell scans
        for (long long cx = ca[0]; cx <= cb[0]; ++cx)
            for (long long cy = ca[1]; cy <= cb[1]; ++cy)
                for (long long cz = ca[2]; cz <= cb[2]; ++cz) {
                    const long long cc[3] = {cx, cy, cz};
                    double md = 0.0;
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        double clo = G.lo[a] + (double)(cc[a] << shift) * G.quantum - G.quantum;
                        double chi = G.lo[a] + (double)((cc[a] + 1) << shift) * G.quantum + G.quantum;
                        double d = c3[a] < clo ? clo - c3[a] : (c3[a] > chi ? c3[a] - chi : 0.0);
                        md += d * d;
                    }
                    if (md * (1.0 - 0x1p-40) > C.T.mx) continue;  // beyond the k-th distance
                    unsigned long long p = morton3(cx, cy, cz);
                    unsigned long long k0 = sh3 >= kKeyBits ? 0ULL : p << sh3;
                    unsigned long long k1 = sh3 >= kKeyBits ? ~0ULL : (p + 1) << sh3;  // exclusive
                    if (k0 >= klo && k1 <= khi) continue;  // inside the window already
                    // a cell adjacent in key order to the last one looked up (the z pairs
                    // of a column, ...) starts where that one ended: one lookup instead of two
                    const long long j0 = k0 == pk1 ? pj1 : cell_lower(keys, n, CT, k0);
                    const long long j1 = sh3 >= kKeyBits || (k1 >> kKeyBits) ? n : cell_lower(keys, n, CT, k1);
                    pk1 = k1;
                    pj1 = j1;
                    scan_range<K>(j0, min(j1, win0), xs, ys, zs, x, y, z, C.T);
                    scan_range<K>(max(j0, win1), j1, xs, ys, zs, x, y, z, C.T);
                    if (evc) nscan += max(0LL, min(j1, win0) - j0) + max(0LL, j1 - max(j0, win1));
                }
        if (evc) atomicAdd(&evc[1], (unsigned long long)nscan);  // diagnostic: cell-scan distances
    }
    if (evc && act) {
        atomicAdd(&evc[0], (unsigned long long)(win1 - win0));  // window distances
        atomicAdd(&evc[3], (unsigned long long)C.T.nins);       // top-k insertions
    }
    if (act) h[idx[i]] = sqrt(C.T.mx);
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
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
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
    if (ws.prof) ASP_TRY(prof_next(ws));
    StageMark mprep(ws, kSKnnPrep, st);  // bounding box, keys, sort, gather, cell tables
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
    // level-L cell table: about one particle per cell, at most 8^9 cells (512 MiB)
    int L = 1;
    while (L < 9 && (1LL << (3 * L)) < n) ++L;
    const long long ncell = 1LL << (3 * L);
    ASP_TRY(ensure(ws.knn[7], (size_t)(ncell + 1) * sizeof(int)));
    int* tab = (int*)ws.knn[7].p;
    ASP_HIP(hipMemsetD32Async((hipDeviceptr_t)tab, (int)n, (size_t)(ncell + 1), st));
    hipLaunchKernelGGL(k_cell_starts, dim3(grid), dim3(kKnnBlock), 0, st,
                       (const unsigned long long*)kout, (long long)n, kKeyBits - 3 * L, tab);
    ASP_LAUNCHED();
    {  // the empty cells: suffix minimum over the ncell + 1 entries
        const long long m = ncell + 1;
        const int nbs = (int)((m + kSfxSpan - 1) / kSfxSpan);
        ASP_TRY(ensure(ws.knn[10], (size_t)nbs * sizeof(int)));
        int* bmin = (int*)ws.knn[10].p;
        hipLaunchKernelGGL(k_sfx_block, dim3(nbs), dim3(kSfxBlock), 0, st, tab, m, bmin);
        ASP_LAUNCHED();
        hipLaunchKernelGGL(k_sfx_top, dim3(1), dim3(kSfxBlock), 0, st, bmin, nbs);
        ASP_LAUNCHED();
        hipLaunchKernelGGL(k_sfx_apply, dim3(nbs), dim3(kSfxBlock), 0, st, tab, m,
                           (const int*)bmin, nbs);
        ASP_LAUNCHED();
    }
    // sub-tables of the dense level-L cells: at most n / (kSubMin + 1) of them
    const int submin = getenv("ASP_KNN_SUBMIN") ? std::max(8, atoi(getenv("ASP_KNN_SUBMIN"))) : kSubMin;
    const long long nslot_max = n / (submin + 1) + 1;
    ASP_TRY(ensure(ws.knn[8], (size_t)(ncell + 1) * sizeof(int)));
    ASP_TRY(ensure(ws.knn[9], (size_t)nslot_max * (kSubCells + 1) * sizeof(int)));
    int* sub = (int*)ws.knn[8].p;
    int* nslot = sub + ncell;
    int* subtab = (int*)ws.knn[9].p;
    ASP_HIP(hipMemsetAsync(nslot, 0, sizeof(int), st));
    hipLaunchKernelGGL(k_sub_slots, dim3((unsigned)((ncell + kKnnBlock - 1) / kKnnBlock)),
                       dim3(kKnnBlock), 0, st, (const int*)tab, ncell, submin, sub, nslot);
    ASP_LAUNCHED();
    hipLaunchKernelGGL(k_sub_table, dim3(grid), dim3(kKnnBlock), 0, st,
                       (const unsigned long long*)kout, (long long)n, kKeyBits - 3 * L,
                       (const int*)tab, (const int*)sub, subtab);
    ASP_LAUNCHED();
    const CellTab CT{tab, sub, subtab, kKeyBits - 3 * L};
    mprep.done();
    // diagnostics only: ASP_KNN_THREAD = one lane per particle throughout;
    // ASP_KNN_DIAG = 1: the window pass alone (wrong results, timing)
    const bool per_thread = getenv("ASP_KNN_THREAD") != nullptr;
    const int diag = getenv("ASP_KNN_DIAG") ? atoi(getenv("ASP_KNN_DIAG")) : 0;
    const int whalf = getenv("ASP_KNN_WINDOW") ? atoi(getenv("ASP_KNN_WINDOW")) : kWinHalf;
    const int fine = getenv("ASP_KNN_FINE") ? atoi(getenv("ASP_KNN_FINE")) : kCellFine;
    const int f32 = getenv("ASP_KNN_F32") ? atoi(getenv("ASP_KNN_F32")) : kWindowF32;
    // the shared cell pass: the common level covers uq / 64 of a wave's lanes (0: off)
    // the window / shared passes' entry test: 16 entries per step into a bit mask (1) or
    // one entry per step into an 8-slot buffer (0)
    const bool mask = getenv("ASP_KNN_MASK") ? atoi(getenv("ASP_KNN_MASK")) != 0 : kMaskTest;
    // the window pass's chunk order: nearest to the wave's own first (1) or in array order (0)
    const int near = getenv("ASP_KNN_NEAR") ? atoi(getenv("ASP_KNN_NEAR")) : kNearFirst;
    // the window's first k entries sorted into the empty top-k (k == 32 / 64 only)
    const int fill = getenv("ASP_KNN_FILL") ? atoi(getenv("ASP_KNN_FILL")) : 1;
    const int uq = getenv("ASP_KNN_UNION") ? std::min(64, std::max(0, atoi(getenv("ASP_KNN_UNION")))) : kUnionQ;
    // ASP_KNN_COUNT: count the distances the search evaluates (bench.py's k-NN roofline;
    // one atomic per lane, so off in timed runs) -> asp_last_stats [9] window, [10] cells,
    // [11] entries the shared cell pass streamed (once per wave), [12] top-k insertions
    unsigned long long* evc = nullptr;
    if (getenv("ASP_KNN_COUNT")) {
        ASP_TRY(ensure(ws.knn[11], 8 * sizeof(unsigned long long)));
        evc = (unsigned long long*)ws.knn[11].p;
        ASP_HIP(hipMemsetAsync(evc, 0, 8 * sizeof(unsigned long long), st));
    }
    StageMark msearch(ws, kSKnnSearch, st);
#define ASP_KNN(KN)                                                                               \
    do {                                                                                          \
        if (per_thread)                                                                           \
            hipLaunchKernelGGL(k_knn<KN>, dim3(grid), dim3(kKnnBlock), 0, st, (const double*)xs,  \
                               (const double*)ys, (const double*)zs,                              \
                               (const unsigned long long*)kout, (const int*)iout, (long long)n,   \
                               k, (const KGrid*)dg, dh);                                          \
        else if (mask)                                                                            \
            hipLaunchKernelGGL((k_knn_wave<KN, true>), dim3((unsigned)((n + 255) / 256)),          \
                               dim3(kKnnBlock), 0, st, (const double*)xs, (const double*)ys,      \
                               (const double*)zs, (const unsigned long long*)kout,                \
                               (const int*)iout, (long long)n, k, (const KGrid*)dg, dh, diag,     \
                               whalf, fine, CT, f32, uq, near, fill, evc);                        \
        else                                                                                      \
            hipLaunchKernelGGL((k_knn_wave<KN, false>), dim3((unsigned)((n + 255) / 256)),         \
                               dim3(kKnnBlock), 0, st, (const double*)xs, (const double*)ys,      \
                               (const double*)zs, (const unsigned long long*)kout,                \
                               (const int*)iout, (long long)n, k, (const KGrid*)dg, dh, diag,     \
                               whalf, fine, CT, f32, uq, near, fill, evc);                        \
    } while (0)
    if (k <= 32)
        ASP_KNN(32);
    else
        ASP_KNN(64);
#undef ASP_KNN
    ASP_LAUNCHED();
    msearch.done();
    for (int j = 9; j <= 12; ++j) ws.stats[j] = 0;
    if (evc) {
        unsigned long long e[8];
        ASP_HIP(hipMemcpyAsync(e, evc, sizeof(e), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
        ws.stats[9] = (long long)e[0];
        ws.stats[10] = (long long)e[1];
        ws.stats[11] = (long long)e[2];
        ws.stats[12] = (long long)e[3];
        if (getenv("ASP_KNN_COUNT_PRINT"))
            fprintf(stderr, "knn shared pass: %llu waves, %.1f columns and %.1f ranges per wave\n", e[6],
                    e[6] ? (double)e[4] / e[6] : 0.0, e[6] ? (double)e[5] / e[6] : 0.0);
    }
    if (!dev) {
        ASP_HIP(hipMemcpyAsync(h, dh, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    return ws_end_.finish();
}

}  // namespace asp

using namespace asp;

extern "C" int asp_knn_smoothing_lengths(const double* positions, int64_t n, int32_t k,
                                         double* h, int32_t flags, int32_t device,
                                         void* stream) {
    t_err.clear();
    return knn(positions, n, k, h, flags, device, (hipStream_t)stream);
}
