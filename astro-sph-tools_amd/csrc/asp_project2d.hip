// asp_project2d.hip -- MI355X (gfx950) SPH particle -> pixel-grid projection.
//
// Replaces the reference's create_image / process_chunk / calculate_pixel_value /
// quartic_spline_kernel path (/root/reference/src/astro_sph_tools/tools/projections/
// _projector.py:13-120, _pixel_calculations.pyx:9-36, _kernels.pyx:9-20) with a
// scatter formulation built for CDNA4:
//
//   K1 count     one streaming pass over (u, v, h): per-workgroup LDS histogram of
//                (particle, GPU tile) insertions -> hist[block][tile]
//   K2a colscan  per tile, exclusive prefix over blocks (in place) + tile totals
//   K2b tilescan one workgroup: tile start offsets in Morton order of the tiles, the
//                deposit work list (runs of <= CH records of one tile; empty tiles get
//                a zero item) and the merge list of tiles split over several items
//   K3 scatter   second streaming pass: each insertion written as a 16/32-byte record
//                into its tile's run (LDS cursors) + per-(block, tile) max|A W_norm|
//   K3b scale    per tile: max over blocks -> power-of-two fixed-point scale
//   K4 deposit   one workgroup per work item: records -> int64 LDS tile accumulators
//                (ds_add_u64), small footprints lane-per-record, large ones swept by a
//                whole wave; the tile is converted and written once, or (split tiles)
//                stored as an int64 partial slab
//   K5 merge     split tiles: exact int64 sum of their slabs, convert, write
//   K6 wide      particles overlapping > kWideTiles tiles, per tile, gathered
//   K7 ratio     out0 / out1 (mass-weighted maps) when not fused into K4/K5
//
// No MFMA: this is gather/scatter work; the bounds are HBM bytes and VALU/LDS-atomic
// issue.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/asp.h"
#include "asp_binning.hpp"
#include "asp_device.hpp"
#include "asp_host.hpp"

namespace asp {

#ifndef ASP_COUNT_BLOCK
#define ASP_COUNT_BLOCK 256
#endif
constexpr int kCountBlock = ASP_COUNT_BLOCK;  // count workgroup
#ifndef ASP_SCATTER_BLOCK
#define ASP_SCATTER_BLOCK 1024
#endif
#ifndef ASP_SCATTER_GROUP
#define ASP_SCATTER_GROUP 4
#endif
// Scatter workgroup and how many consecutive count workgroups' particles it takes over:
// fewer, wider scatter workgroups keep fewer partially written record lines open at a
// time (each workgroup appends to its own segment of every tile), so more of them fill
// in the caches before they are written back.
constexpr int kScatterBlock = ASP_SCATTER_BLOCK;
constexpr int kScatterGroup = ASP_SCATTER_GROUP;

#ifndef ASP_ABLATE_SCATTER
#define ASP_ABLATE_SCATTER 0  // diagnostic builds only: 1 = no first-record stores,
                              // 2 = first records stored to coalesced slots (wrong map)
#endif

// A record whose box clipped to its tile spans >= g.band_cols columns is WIDE: it is
// binned into a second run per tile (histogram column t + ntiles) and deposited by row
// bands (K4b: lanes own columns, register accumulation, no atomics), which beats the
// atomic-bound wave sweep only when most of a wave's 64 lanes have work.
__device__ __forceinline__ int tile_column(const Grid& g, const Box& b, bool maybe_wide, int tx,
                                           int ty) {
    int t = tx * g.nty + ty;
    if (!maybe_wide) return t;
    int hh = min(b.y1, ty * kTile + kTile - 1) - max(b.y0, ty * kTile) + 1;
    return hh >= g.band_cols ? t + g.ntiles : t;
}
constexpr int kUnroll = 2;        // particles in flight per thread in scatter
#ifndef ASP_COUNT_UNROLL
#define ASP_COUNT_UNROLL 8
#endif
constexpr int kCountUnroll = ASP_COUNT_UNROLL;  // ... and in count
// Particles per loop iteration of a count / scatter workgroup (a "batch").
constexpr long long kBatch = (long long)kCountBlock * kCountUnroll;
static_assert(kBatch == (long long)kScatterBlock * kUnroll, "count and scatter batches differ");
#ifndef ASP_INTERLEAVE
#define ASP_INTERLEAVE 1
#endif
// ASP_INTERLEAVE: batches are dealt to the count workgroups round-robin (batch j to
// workgroup j % nblk; the scatter workgroup of count workgroups sb*grp.. takes their
// batches in order), so at any moment the whole grid streams one window of the particle
// arrays instead of nblk far-apart runs.  0: each workgroup owns one contiguous run.

// Vector of U floats (one 4 U-byte load per lane).
template <int U>
using vecf = float __attribute__((ext_vector_type(U)));

// Load U CONSECUTIVE particles per lane (particle base + U * lane + k) with one U-wide
// load per array when the arrays are 4 U-byte aligned (`al`, the caller checks the base
// pointers; base is a multiple of U): a quarter of the load instructions of lane-strided
// dword loads, which kept the count pass at 3.7 TB/s.  h = 0 past the end, which has no
// footprint.
template <int U>
__device__ __forceinline__ void load_vec(const float* __restrict__ a, long long p, long long p1,
                                         bool al, float* out) {
    if (al && p + U <= p1) {
        vecf<U> x = *(const vecf<U>*)(a + p);
#pragma unroll
        for (int k = 0; k < U; ++k) out[k] = x[k];
    } else {
#pragma unroll
        for (int k = 0; k < U; ++k) out[k] = p + k < p1 ? a[p + k] : 0.0f;
    }
}
template <int U>
__device__ __forceinline__ bool aligned_vec(const void* a, const void* b, const void* c) {
    return (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & (4 * U - 1)) == 0;
}

template <int NT, int U = kUnroll>
__device__ __forceinline__ void load_batch(const float* __restrict__ u,
                                           const float* __restrict__ v,
                                           const float* __restrict__ h, long long base,
                                           long long p1, bool al, float* pu, float* pv,
                                           float* ph) {
    long long p = base + (long long)threadIdx.x * U;
    load_vec<U>(u, p, p1, al, pu);
    load_vec<U>(v, p, p1, al, pv);
    load_vec<U>(h, p, p1, al, ph);
}

// Record store (plain: non-temporal stores measured 2x slower for this pattern).
__device__ __forceinline__ void put_rec(float4* p, float4 v) { *p = v; }

// ----------------------------------------------------------------------------------
// K1: count insertions per (block, tile)
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(kCountBlock) void k_count(const float* __restrict__ u,
                                                       const float* __restrict__ v,
                                                       const float* __restrict__ h,
                                                       long long n, long long per_block, Grid g,
                                                       int* __restrict__ hist,
                                                       int* __restrict__ ctr) {
    extern __shared__ __attribute__((aligned(16))) int lh[];  // 2 * ntiles columns
    for (int t = threadIdx.x; t < g.nstream * g.ntiles; t += kCountBlock) lh[t] = 0;
    __syncthreads();
    int nwide = 0;
    constexpr long long kStep = kBatch;
#if ASP_INTERLEAVE
    // batch j (kBatch particles) belongs to count workgroup j % nblk
    const long long p0 = (long long)blockIdx.x * kStep, p1 = n, stride = per_block * kStep;
#else
    const long long p0 = (long long)blockIdx.x * per_block, p1 = min(n, p0 + per_block),
                    stride = kStep;
#endif
    // Software pipeline: the next batch's loads are in flight while this batch is binned.
    float pu[kCountUnroll], pv[kCountUnroll], ph[kCountUnroll];
    const bool al = aligned_vec<kCountUnroll>(u, v, h);
    load_batch<kCountBlock, kCountUnroll>(u, v, h, p0, p1, al, pu, pv, ph);
    for (long long base = p0; base < p1; base += stride) {
        float nu[kCountUnroll], nv[kCountUnroll], nh[kCountUnroll];
        load_batch<kCountBlock, kCountUnroll>(u, v, h, base + stride, p1, al, nu, nv, nh);
#pragma unroll
        for (int k = 0; k < kCountUnroll; ++k) {
            Box b;
            if (!footprint(g, pu[k], pv[k], ph[k], b)) continue;
            int tx0 = b.x0 >> kTileShift, tx1 = b.x1 >> kTileShift;
            int ty0 = b.y0 >> kTileShift, ty1 = b.y1 >> kTileShift;
            if ((tx1 - tx0 + 1) * (ty1 - ty0 + 1) > g.wide_tiles) {
                ++nwide;
                continue;
            }
            bool mb = g.nstream == 2 && b.y1 - b.y0 + 1 >= g.band_cols;
            for (int tx = tx0; tx <= tx1; ++tx)
                for (int ty = ty0; ty <= ty1; ++ty)
                    atomicAdd(&lh[tile_column(g, b, mb, tx, ty)], 1);
        }
#pragma unroll
        for (int k = 0; k < kCountUnroll; ++k) {
            pu[k] = nu[k];
            pv[k] = nv[k];
            ph[k] = nh[k];
        }
    }
    if (nwide) atomicAdd(&ctr[cWideCount], nwide);
    __syncthreads();
    int* row = hist + (long long)blockIdx.x * g.nstream * g.ntiles;
    for (int t = threadIdx.x; t < g.nstream * g.ntiles; t += kCountBlock) row[t] = lh[t];
}

// A record's candidate box clipped to tile (tx, ty), tile-local, one byte per bound:
// x0 | x1 << 8 | y0 << 16 | y1 << 24 (carried as the bits of a float).
__device__ __forceinline__ float tile_box(const Box& b, int tx, int ty) {
    int X0 = tx * kTile, Y0 = ty * kTile;
    unsigned x0 = max(b.x0, X0) - X0, x1 = min(b.x1, X0 + kTile - 1) - X0;
    unsigned y0 = max(b.y0, Y0) - Y0, y1 = min(b.y1, Y0 + kTile - 1) - Y0;
    return __uint_as_float(x0 | (x1 << 8) | (y0 << 16) | (y1 << 24));
}

template <int NOUT, int NT>
__device__ __forceinline__ void load_props(const float* __restrict__ a0,
                                           const float* __restrict__ a1, long long base,
                                           long long p1, bool al, float* pa0, float* pa1) {
    long long p = base + (long long)threadIdx.x * kUnroll;
    load_vec<kUnroll>(a0, p, p1, al, pa0);
    if constexpr (NOUT == 2) {
        load_vec<kUnroll>(a1, p, p1, al, pa1);
    } else {
#pragma unroll
        for (int k = 0; k < kUnroll; ++k) pa1[k] = 0.0f;
    }
}

// ----------------------------------------------------------------------------------
// K3: scatter records into their tiles' runs.  Same particle partition as K1.
// Record layout: NOUT == 1 -> float4 {u, v, h, a0};  NOUT == 2 -> the PREPARED record,
// 2 x float4 {u, v, h, c0}, {c1, thr, band, box} (prep2_record): the deposit's per-record
// set-up (candidate box, clip, error band, fp64 kernel normalisation) is done here, where
// the store-bound scatter has VALU to spare, instead of in the VALU-bound deposit.  Also
// the per-(block, tile) max |c| (fp32 bits) of the records it inserted, the fixed-point
// bound of K3b.
// ----------------------------------------------------------------------------------
template <int KID, int NOUT, int ACC>
__global__ __launch_bounds__(kScatterBlock) void k_scatter(
    const float* __restrict__ u, const float* __restrict__ v, const float* __restrict__ h,
    const float* __restrict__ a0, const float* __restrict__ a1, long long n, long long per_block,
    Grid g, const int* __restrict__ hist, const long long* __restrict__ tile_start,
    float4* __restrict__ recs, unsigned* __restrict__ cmx, int* __restrict__ wide_list,
    int* __restrict__ ctr, int blk0, int grp, long long rec_cap, int wide_cap) {
    // Speculative launch (enqueued before the host has read the counters): the record and
    // wide-list buffers were sized by an earlier call; if this call needs more, every
    // workgroup leaves at once and the host relaunches after growing them.
    if (ctr[cRecs] > rec_cap || ctr[cWideCount] > wide_cap) return;
    // absolute record cursors, regular runs then large runs (2 * ntiles)
    extern __shared__ __attribute__((aligned(16))) int cur[];
    // per-wave staging for the paired record stores (NOUT == 2): 64 records x 32 B
    float4* stage = (float4*)(cur + g.nstream * g.ntiles);
    unsigned* cm = (unsigned*)(stage + (NOUT == 2 ? (kScatterBlock / 64) * 128 : 0));
    // this workgroup (global index sb = blk0 + blockIdx.x) takes over count workgroups
    // grp * sb ..: its cursors start at the prefix row of the first of them
    const long long sb = blk0 + (long long)blockIdx.x;
    const int* row = hist + sb * grp * g.nstream * g.ntiles;
    for (int t = threadIdx.x; t < g.nstream * g.ntiles; t += kScatterBlock)
        cur[t] = (int)tile_start[t] + row[t];  // n_recs < 2^31 (checked on the host)
    if constexpr (ACC == kAccFix)
        for (int t = threadIdx.x; t < g.ntiles * NOUT; t += kScatterBlock) cm[t] = 0u;
    __syncthreads();
    constexpr long long kStep = kBatch;
#if ASP_INTERLEAVE
    // the batches of count workgroups sb * grp .. (< nblk = per_block here), in order:
    // batch it * nblk + sb * grp + j for j < gcnt, it = 0, 1, ...
    const long long gcnt = min((long long)grp, per_block - sb * grp);
    auto batch_base = [&](long long c) {
        return ((c / gcnt) * per_block + sb * grp + c % gcnt) * kStep;
    };
    const long long p1 = n;
    long long c = 0;
    const long long p0 = batch_base(0);
#else
    const long long p0 = sb * per_block;
    const long long p1 = min(n, p0 + per_block);
#endif
    // Software pipeline: issue the next batch's loads BEFORE this batch's record stores,
    // so waiting for them (vmcnt counts loads and stores in issue order) never waits on
    // the scattered stores.
    float pu[kUnroll], pv[kUnroll], ph[kUnroll], pa0[kUnroll], pa1[kUnroll];
    int first_slot[kUnroll];
    // the prepared fields of every particle's first record (the paired store's payload)
    float first_c0[kUnroll], first_c1[kUnroll], first_thr[kUnroll], first_band[kUnroll],
        first_box[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
        first_slot[k] = -1;
        first_c0[k] = first_c1[k] = first_thr[k] = first_band[k] = first_box[k] = 0.0f;
    }
    const bool al = aligned_vec<kUnroll>(u, v, h) && aligned_vec<kUnroll>(a0, NOUT == 2 ? a1 : a0, a0);
    load_batch<kScatterBlock>(u, v, h, p0, p1, al, pu, pv, ph);
    load_props<NOUT, kScatterBlock>(a0, a1, p0, p1, al, pa0, pa1);
#if ASP_INTERLEAVE
    for (long long base = p0, next; base < p1; base = next) {
        next = batch_base(++c);
#else
    for (long long base = p0, next; base < p1; base = next) {
        next = base + kStep;
#endif
        float nu[kUnroll], nv[kUnroll], nh[kUnroll], na0[kUnroll], na1[kUnroll];
        load_batch<kScatterBlock>(u, v, h, next, p1, al, nu, nv, nh);
        load_props<NOUT, kScatterBlock>(a0, a1, next, p1, al, na0, na1);
#pragma unroll
        for (int k = 0; k < kUnroll; ++k) {
            long long p = base + (long long)threadIdx.x * kUnroll + k;
            Box b;
            if (!footprint(g, pu[k], pv[k], ph[k], b)) continue;
            // NOUT == 2: the prepared record's fields (prep2_record); the fixed-point
            // bound is taken over the same fp32 coefficients the deposit scales
            float cf0 = NOUT == 2 ? (float)term_coef<KID>(pa0[k], ph[k]) : 0.0f;
            float cf1 = NOUT == 2 ? (float)term_coef<KID>(pa1[k], ph[k]) : 0.0f;
            unsigned c0 = 0u, c1 = 0u;
            if constexpr (ACC == kAccFix) {
                c0 = __float_as_uint(fabsf(NOUT == 2 ? cf0 : (float)term_coef<KID>(pa0[k], ph[k])));
                if (NOUT == 2) c1 = __float_as_uint(fabsf(cf1));
            }
            int tx0 = b.x0 >> kTileShift, tx1 = b.x1 >> kTileShift;
            int ty0 = b.y0 >> kTileShift, ty1 = b.y1 >> kTileShift;
            if ((tx1 - tx0 + 1) * (ty1 - ty0 + 1) > g.wide_tiles) {
                wide_list[atomicAdd(&ctr[cWideCursor], 1)] = (int)p;
                if constexpr (ACC == kAccFix) {
                    atomicMax((unsigned*)&ctr[cWideMax0], c0);
                    if (NOUT == 2) atomicMax((unsigned*)&ctr[cWideMax1], c1);
                }
                continue;
            }
            float thr = 0.0f, band = 0.0f;
            if constexpr (NOUT == 2) rec_band(g, ph[k], thr, band);
            float4 r0 = make_float4(pu[k], pv[k], ph[k], NOUT == 2 ? cf0 : pa0[k]);
            if constexpr (NOUT == 2) {
                first_c0[k] = cf0;
                first_c1[k] = cf1;
                first_thr[k] = thr;
                first_band[k] = band;
            }
            bool mb = g.nstream == 2 && b.y1 - b.y0 + 1 >= g.band_cols;
            for (int tx = tx0; tx <= tx1; ++tx)
                for (int ty = ty0; ty <= ty1; ++ty) {
                    int t = tx * g.nty + ty;
                    int slot = atomicAdd(&cur[tile_column(g, b, mb, tx, ty)], 1);
                    if constexpr (ACC == kAccFix) {
                        atomicMax(&cm[t * NOUT], c0);
                        if (NOUT == 2) atomicMax(&cm[t * NOUT + 1], c1);
                    }
#if ASP_ABLATE_SCATTER == 2
                    slot = (int)p;  // diagnostic: coalesced destinations, same bytes
#endif
                    if constexpr (NOUT == 2) {
                        float bp = tile_box(b, tx, ty);
                        if (tx == tx0 && ty == ty0) {
                            first_slot[k] = slot;  // written by the paired store below
                            first_box[k] = bp;
                        } else {
                            put_rec(&recs[2 * (long long)slot], r0);
                            put_rec(&recs[2 * (long long)slot + 1], make_float4(cf1, thr, band, bp));
                        }
                    } else {
                        put_rec(&recs[slot], r0);
                    }
                }
        }
        if constexpr (NOUT == 2) {
            // Paired store of every particle's first record: lanes 2j and 2j+1 write the
            // two 16-B halves of record j, so one store instruction covers 32 whole
            // 32-B records (32 lines) instead of 64 half records (64 lines).
            float4* st = stage + (threadIdx.x >> 6) * 128;
            int lane = threadIdx.x & 63;
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) {
                st[2 * lane] = make_float4(pu[k], pv[k], ph[k], first_c0[k]);
                st[2 * lane + 1] = make_float4(first_c1[k], first_thr[k], first_band[k], first_box[k]);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    int src = half * 32 + (lane >> 1);
                    int slot = __shfl(first_slot[k], src);
                    float4 val = st[2 * src + (lane & 1)];
#if ASP_ABLATE_SCATTER == 1
                    asm volatile("" ::"v"(val.x), "v"(val.y), "v"(val.z), "v"(val.w), "v"(slot));
#else
                    if (slot >= 0) put_rec(&recs[2 * (long long)slot + (lane & 1)], val);
#endif
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                first_slot[k] = -1;
            }
        }
#pragma unroll
        for (int k = 0; k < kUnroll; ++k) {
            pu[k] = nu[k];
            pv[k] = nv[k];
            ph[k] = nh[k];
            pa0[k] = na0[k];
            pa1[k] = na1[k];
        }
    }
    if constexpr (ACC == kAccFix) {
        __syncthreads();
        unsigned* out = cmx + (long long)blockIdx.x * g.ntiles * NOUT;  // per scatter block
        for (int t = threadIdx.x; t < g.ntiles * NOUT; t += kScatterBlock) out[t] = cm[t];
    }
}

// Power-of-two scale exponent so that n * cmax * 2^k <= 2^kScaleBits.
__device__ __forceinline__ int scale_exp(long long n, float cmax) {
    if (!(cmax > 0.0f) || n <= 0 || !__builtin_isfinite(cmax)) return 0;
    int e;
    frexp((double)n * (double)cmax, &e);  // n*cmax < 2^e
    return kScaleBits - e;
}

// ----------------------------------------------------------------------------------
// K3b: per tile, max over blocks of cmx -> fixed-point exponents tile_k[t] = {k0, k1}.
// ----------------------------------------------------------------------------------
template <int NOUT>
__global__ __launch_bounds__(kBlock) void k_tilescale(const unsigned* __restrict__ cmx, int nblk,
                                                      int ntiles, int nstream,
                                                      const int* __restrict__ tile_total,
                                                      int2* __restrict__ tile_k) {
    __shared__ unsigned part[4][64][NOUT];
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int t = blockIdx.x * 64 + lane;
    int b0 = (int)((long long)nblk * w / 4), b1 = (int)((long long)nblk * (w + 1) / 4);
    unsigned m[NOUT];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) m[o] = 0u;
    if (t < ntiles)
        for (int b = b0; b < b1; ++b)
#pragma unroll
            for (int o = 0; o < NOUT; ++o)
                m[o] = max(m[o], cmx[((long long)b * ntiles + t) * NOUT + o]);
#pragma unroll
    for (int o = 0; o < NOUT; ++o) part[w][lane][o] = m[o];
    __syncthreads();
    if (w == 0 && t < ntiles) {
        int k[2] = {0, 0};
#pragma unroll
        for (int o = 0; o < NOUT; ++o) {
            unsigned mm = max(max(part[0][lane][o], part[1][lane][o]),
                              max(part[2][lane][o], part[3][lane][o]));
            k[o] = scale_exp((long long)tile_total[t] + (nstream == 2 ? tile_total[t + ntiles] : 0),
                             __uint_as_float(mm));
        }
        tile_k[t] = make_int2(k[0], k[1]);
    }
}

// ----------------------------------------------------------------------------------
// Pair accumulation into the LDS tile (int64 fixed point)
// ----------------------------------------------------------------------------------
#ifndef ASP_ABLATE
#define ASP_ABLATE 0  // diagnostic builds only (tools/ablate.sh): 4 = conflict-free atomics, 1 = no LDS atomics,
                      // 2 = no pair loop, 3 = no record prep
#endif

template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void accumulate(const Prep& P, float r2, unsigned long long* acc0,
                                           unsigned long long* acc1, int k) {
    float q = __builtin_amdgcn_sqrtf(r2) * P.hinv;  // v_sqrt_f32, 1 ulp
    float w = kernel_shape<KID>(q);
#if ASP_ABLATE == 1
    float t0 = P.s0 * w, t1 = P.s1 * w;
    asm volatile("" ::"v"(t0), "v"(t1), "v"(k));
#else
    acc_add<ACC>(&acc0[k], P.s0 * w);
    if constexpr (NOUT == 2) acc_add<ACC>(&acc1[k], P.s1 * w);
#endif
}

// One wave sweeps the (clipped) box of one wave-uniform record: lanes along y (the
// contiguous image axis), so the LDS atomics of a wave hit distinct consecutive words.
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void sweep(const Grid& g, const Prep& P, int X0, int Y0,
                                      const float* xt, const float* yt,
                                      unsigned long long* acc0, unsigned long long* acc1,
                                      int lane) {
    int bh = P.b.y1 - P.b.y0 + 1;
    if (bh <= 64) {
        int rps = 64 / bh;
        int r = lane / bh, c = lane - r * bh;
        if (r < rps) {
            int yi = P.b.y0 + c;
            float Y = yt[yi - Y0];
            for (int xi = P.b.x0 + r; xi <= P.b.x1; xi += rps) {
                float r2;
                if (decide(g, P, xi, yi, xt[xi - X0], Y, r2))
                    accumulate<KID, NOUT, ACC>(P, r2, acc0, acc1, (xi - X0) * kTile + (yi - Y0));
            }
        }
    } else {
        for (int xi = P.b.x0; xi <= P.b.x1; ++xi) {
            float X = xt[xi - X0];
            for (int c = lane; c < bh; c += 64) {
                int yi = P.b.y0 + c;
                float r2;
                if (decide(g, P, xi, yi, X, yt[yi - Y0], r2))
                    accumulate<KID, NOUT, ACC>(P, r2, acc0, acc1, (xi - X0) * kTile + (yi - Y0));
            }
        }
    }
}

__device__ __forceinline__ Prep bcast_prep(const Prep& P, int l) {
    Prep Q;
    Q.u = bcast(P.u, l);
    Q.v = bcast(P.v, l);
    Q.h = bcast(P.h, l);
    Q.lo = bcast(P.lo, l);
    Q.hi = bcast(P.hi, l);
    Q.hinv = bcast(P.hinv, l);
    Q.s0 = bcast(P.s0, l);
    Q.s1 = bcast(P.s1, l);
    Q.b.x0 = bcast(P.b.x0, l);
    Q.b.x1 = bcast(P.b.x1, l);
    Q.b.y0 = bcast(P.b.y0, l);
    Q.b.y1 = bcast(P.b.y1, l);
    return Q;
}

__device__ __forceinline__ bool clip(Box& b, int X0, int Y0, int TW, int TH) {
    b.x0 = max(b.x0, X0);
    b.x1 = min(b.x1, X0 + TW - 1);
    b.y0 = max(b.y0, Y0);
    b.y1 = min(b.y1, Y0 + TH - 1);
    return b.x0 <= b.x1 && b.y0 <= b.y1;
}

// A record -> the pair loop's state, clipped to the tile (X0, Y0, TW, TH).  NOUT == 1:
// raw {u, v, h, a0}, prepared here.  NOUT == 2: the scatter's prepared record
// {u, v, h, c0}, {c1, thr, band, box}; only 1/h and the tile's fixed-point scale remain
// (ldexp of the fp32 coefficient: exact, the scale is a power of two).  False: no pair.
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ bool rec_prep(const Grid& g, const float4& r0, const float4& r1,
                                         int X0, int Y0, int TW, int TH, int2 kk, Prep& P) {
    if constexpr (NOUT == 1) {
        return prep_record<KID, ACC>(g, r0.x, r0.y, r0.z, r0.w, 0.0f, kk.x, kk.y, P) &&
               clip(P.b, X0, Y0, TW, TH);
    } else {
        P.u = r0.x;
        P.v = r0.y;
        P.h = r0.z;
        set_band(P, r1.y, r1.z);
        P.hinv = __builtin_amdgcn_rcpf(r0.z);
        if constexpr (ACC == kAccFix) {
            P.s0 = ldexpf(r0.w, kk.x);
            P.s1 = ldexpf(r1.x, kk.y);
        } else {
            P.s0 = r0.w;
            P.s1 = r1.x;
        }
        unsigned bp = __float_as_uint(r1.w);
        P.b.x0 = X0 + (int)(bp & 255u);
        P.b.x1 = X0 + (int)((bp >> 8) & 255u);
        P.b.y0 = Y0 + (int)((bp >> 16) & 255u);
        P.b.y1 = Y0 + (int)(bp >> 24);
        return true;
    }
}

template <int NOUT>
__device__ __forceinline__ void load_rec4(const float4* recs, long long i, float4& r0,
                                          float4& r1) {
    if constexpr (NOUT == 1) {
        r0 = recs[i];
    } else {
        r0 = recs[2 * i];
        r1 = recs[2 * i + 1];
    }
}

constexpr int kTilePix = kTile * kTile;
constexpr int kFlagAccumulate = 1;
constexpr int kFlagRatio = 2;  // fused ratio: out0 <- map0 / map1

// Tile prologue: zero accumulators, fp32 corner tables (exact fp64 corners rounded).
template <int NOUT, int NT>
__device__ __forceinline__ void tile_prologue(const Grid& g, int X0, int Y0,
                                              unsigned long long* acc, float* xt, float* yt) {
    for (int i = threadIdx.x; i < NOUT * kTilePix; i += NT) acc[i] = 0ull;
    if (threadIdx.x < kTile)
        xt[threadIdx.x] = (float)corner_x(g, X0 + threadIdx.x);
    else if (threadIdx.x < 2 * kTile)
        yt[threadIdx.x - kTile] = (float)corner_y(g, Y0 + threadIdx.x - kTile);
    __syncthreads();
}

// Convert a pixel's fixed-point sums and write it (plain store: the tile has one owner).
template <int NOUT, int ACC>
__device__ __forceinline__ void emit_pixel(long long o, unsigned long long s0,
                                           unsigned long long s1, int k0, int k1, float* out0,
                                           float* out1, int flags) {
    float v0 = acc_value<ACC>(s0, k0);
    float v1 = NOUT == 2 ? acc_value<ACC>(s1, k1) : 0.0f;
    if (flags & kFlagAccumulate) {
        v0 += out0[o];
        if (NOUT == 2) v1 += out1[o];
    }
    if (NOUT == 2) {
        out1[o] = v1;
        out0[o] = (flags & kFlagRatio) ? (v1 != 0.0f ? v0 / v1 : 0.0f) : v0;
    } else {
        out0[o] = v0;
    }
}

// ----------------------------------------------------------------------------------
// Gather form for large records (clipped box >= kGatherArea pixels).  A sweep costs one
// LDS atomic per pair and map; here every thread OWNS 8 pixels of the tile (row
// t >> 3, columns (t & 7) * 8 .. + 7), walks a block-wide LDS list of large records and
// sums their terms in registers -- no atomics per pair, only a flush per list round.
// ----------------------------------------------------------------------------------
constexpr int kBandCols2 = kTile + 1;  // row-band threshold for two-map maps (off)
constexpr int kGatherCap = 128;  // list entries per round (5 KiB of LDS)

struct GRec {  // 40 bytes; all lanes read the same entry (LDS broadcast)
    float u, v, lo, hi, hinv, s0, s1, h;
    int xr, yr;  // tile-local box: x0 | x1 << 16, y0 | y1 << 16
};

__device__ __forceinline__ GRec make_grec(const Prep& P, int X0, int Y0) {
    GRec r;
    r.u = P.u; r.v = P.v; r.lo = P.lo; r.hi = P.hi; r.hinv = P.hinv;
    r.s0 = P.s0; r.s1 = P.s1; r.h = P.h;
    r.xr = (P.b.x0 - X0) | ((P.b.x1 - X0) << 16);
    r.yr = (P.b.y0 - Y0) | ((P.b.y1 - Y0) << 16);
    return r;
}

// Register accumulators of one thread's 8 pixels: fp32 partial sums (flushed into the
// fp64 LDS tile every list round, <= kGatherCap terms each) or exact int64 fixed point.
template <int NOUT, int ACC>
struct GAcc {
    using T = typename std::conditional<ACC == kAccFix, unsigned long long, float>::type;
    T a0[8], a1[8];
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int j = 0; j < 8; ++j) { a0[j] = 0; a1[j] = 0; }
    }
    __device__ __forceinline__ void add(int j, float t0, float t1) {
        if constexpr (ACC == kAccFix) {
            a0[j] += f2fix(t0);
            if (NOUT == 2) a1[j] += f2fix(t1);
        } else {
            a0[j] += t0;
            if (NOUT == 2) a1[j] += t1;
        }
    }
    // add into the LDS tile (atomics: other waves may still be depositing there)
    __device__ __forceinline__ void flush(unsigned long long* acc0, unsigned long long* acc1,
                                          int pix0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (ACC == kAccFix) {
                if (a0[j]) atomicAdd(&acc0[pix0 + j], a0[j]);
                if (NOUT == 2 && a1[j]) atomicAdd(&acc1[pix0 + j], a1[j]);
            } else {
                if (a0[j] != 0.0f) atomicAdd((double*)&acc0[pix0 + j], (double)a0[j]);
                if (NOUT == 2 && a1[j] != 0.0f) atomicAdd((double*)&acc1[pix0 + j], (double)a1[j]);
            }
        }
        zero();
    }
};

// One list record against this thread's 8 pixels (row lx, columns ly0 .. ly0 + 7).
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void gather_rec(const Grid& g, const GRec& R, int X0, int Y0, int lx,
                                           int ly0, float X, const float* Yc,
                                           GAcc<NOUT, ACC>& ra) {
    int x0 = R.xr & 0xffff, x1 = R.xr >> 16, y0 = R.yr & 0xffff, y1 = R.yr >> 16;
    if (lx < x0 || lx > x1 || ly0 + 7 < y0 || ly0 > y1) return;
    float dx = R.u - X;
    float dx2 = dx * dx;
    unsigned amb = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float dy = R.v - Yc[j];
        float r2 = dx2 + dy * dy;
        bool inb = ly0 + j >= y0 && ly0 + j <= y1;
        bool a = inb && r2 >= R.lo && r2 <= R.hi;
        bool in = inb && r2 < R.lo;
        amb |= a ? (1u << j) : 0u;
        float w = kernel_shape<KID>(__builtin_amdgcn_sqrtf(r2) * R.hinv);
        ra.add(j, in ? R.s0 * w : 0.0f, in ? R.s1 * w : 0.0f);
    }
    if (amb) {  // band pairs (rare): the reference's fp64 decision
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // static indices: ra and Yc stay in registers
            if (!(amb & (1u << j))) continue;
            if (exact_pair(g, R.u, R.v, R.h, X0 + lx, Y0 + ly0 + j)) {
                float dy = R.v - Yc[j];
                float w = kernel_shape<KID>(__builtin_amdgcn_sqrtf(dx2 + dy * dy) * R.hinv);
                ra.add(j, R.s0 * w, R.s1 * w);
            }
        }
    }
}

// Block-wide: append this thread's large record (if any) to the LDS list and let the
// whole workgroup gather it, kGatherCap records per round.  Every thread of the block
// must call this (it contains barriers).
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void gather_rounds(const Grid& g, bool large, const Prep& P, int X0,
                                              int Y0, GRec* list, int* s_n, const float* xt,
                                              const float* yt, unsigned long long* acc0,
                                              unsigned long long* acc1) {
    const int lx = threadIdx.x >> 3, ly0 = (threadIdx.x & 7) << 3;
    // (registers live only inside a round: nothing is held across the record loop)
    const float X = xt[lx];
    float Yc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Yc[j] = yt[ly0 + j];
    GAcc<NOUT, ACC> ra;
    ra.zero();
    bool pending = large;
    for (;;) {
        if (threadIdx.x == 0) *s_n = 0;
        __syncthreads();
        if (pending) {
            int slot = atomicAdd(s_n, 1);
            if (slot < kGatherCap) {
                list[slot] = make_grec(P, X0, Y0);
                pending = false;
            }
        }
        __syncthreads();
        int total = *s_n;
        int n = min(total, kGatherCap);
        if (lx < kTile)
            for (int k = 0; k < n; ++k)
                gather_rec<KID, NOUT, ACC>(g, list[k], X0, Y0, lx, ly0, X, Yc, ra);
        if (lx < kTile) ra.flush(acc0, acc1, lx * kTile + ly0);
        __syncthreads();  // the list is rewritten next round
        if (total <= kGatherCap) break;
    }
}

// ----------------------------------------------------------------------------------
// K4 mode 1: a run of non-small records of one tile, deposited by ROW BANDS.  Wave w
// owns tile rows 8w .. 8w+7, lane l owns column l: every wave streams all records of the
// item, keeps those whose clipped box meets its rows and adds their terms to its own
// register accumulators -- no atomics, no LDS tile, waves never wait for each other.
// fp32 partial sums of one 64-record batch are folded into fp64 registers (kAccF64) or
// terms go straight to int64 fixed point (kAccFix).
// ----------------------------------------------------------------------------------
template <int NOUT, int ACC>
struct RowAcc {
    using W = typename std::conditional<ACC == kAccFix, unsigned long long, double>::type;
    W s0[8], s1[8];
    float f0[8], f1[8];
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            s0[r] = 0; s1[r] = 0; f0[r] = 0.0f; f1[r] = 0.0f;
        }
    }
    __device__ __forceinline__ void add(int r, float t0, float t1) {
        if constexpr (ACC == kAccFix) {
            s0[r] += f2fix(t0);
            if (NOUT == 2) s1[r] += f2fix(t1);
        } else {
            f0[r] += t0;
            if (NOUT == 2) f1[r] += t1;
        }
    }
    __device__ __forceinline__ void fold() {
        if constexpr (ACC != kAccFix) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                s0[r] += (double)f0[r];
                f0[r] = 0.0f;
                if (NOUT == 2) {
                    s1[r] += (double)f1[r];
                    f1[r] = 0.0f;
                }
            }
        }
    }
    __device__ __forceinline__ unsigned long long word0(int r) const {
        if constexpr (ACC == kAccFix) return s0[r];
        else return (unsigned long long)__double_as_longlong(s0[r]);
    }
    __device__ __forceinline__ unsigned long long word1(int r) const {
        if constexpr (ACC == kAccFix) return s1[r];
        else return (unsigned long long)__double_as_longlong(s1[r]);
    }
};

template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void band_item(const Grid& g, const float4* __restrict__ recs,
                                          const Item& it, int X0, int Y0, int TW, int TH,
                                          int2 kk, const float* xt, const float* yt,
                                          unsigned long long* __restrict__ slabs,
                                          float* __restrict__ out0, float* __restrict__ out1,
                                          int flags) {
    const int lane = threadIdx.x & 63, rb0 = blockIdx.y * 32 + (threadIdx.x >> 6) * 8;
    const float Yl = yt[lane];
    float Xr[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) Xr[r] = xt[rb0 + r];
    RowAcc<NOUT, ACC> ra;
    ra.zero();
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0;
    if (lane < it.count) load_rec4<NOUT>(recs, it.start + lane, r0, r1);
    for (int base = 0; base < it.count; base += 64) {
        float4 n0 = make_float4(0.f, 0.f, 0.f, 0.f), n1 = n0;
        if (base + 64 + lane < it.count) load_rec4<NOUT>(recs, it.start + base + 64 + lane, n0, n1);
        Prep P;
        bool hit = base + lane < it.count &&
                   rec_prep<KID, NOUT, ACC>(g, r0, r1, X0, Y0, TW, TH, kk, P) &&
                   P.b.x0 - X0 <= rb0 + 7 && P.b.x1 - X0 >= rb0;
        r0 = n0;
        r1 = n1;
        unsigned long long m = __ballot(hit);
        while (m) {
            int l = __builtin_ctzll(m);
            m &= m - 1;
            Prep Q = bcast_prep(P, l);
            const int ra0 = max(Q.b.x0 - X0 - rb0, 0), ra1 = min(Q.b.x1 - X0 - rb0, 7);
            const bool col = Y0 + lane >= Q.b.y0 && Y0 + lane <= Q.b.y1;
            const float dy = Q.v - Yl;
            const float dy2 = dy * dy;
            unsigned amb = 0u;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (r < ra0 || r > ra1) continue;  // wave-uniform
                float dx = Q.u - Xr[r];
                float r2 = dx * dx + dy2;
                bool a = col && r2 >= Q.lo && r2 <= Q.hi;
                bool in = col && r2 < Q.lo;
                amb |= a ? (1u << r) : 0u;
                float w = kernel_shape<KID>(__builtin_amdgcn_sqrtf(r2) * Q.hinv);
                ra.add(r, in ? Q.s0 * w : 0.0f, in ? Q.s1 * w : 0.0f);
            }
            if (amb) {  // band pairs (rare): the reference's fp64 decision
#pragma unroll
                for (int r = 0; r < 8; ++r) {  // static indices: ra stays in registers
                    if (!(amb & (1u << r))) continue;
                    if (exact_pair(g, Q.u, Q.v, Q.h, X0 + rb0 + r, Y0 + lane)) {
                        float dx = Q.u - Xr[r];
                        float w =
                            kernel_shape<KID>(__builtin_amdgcn_sqrtf(dx * dx + dy2) * Q.hinv);
                        ra.add(r, Q.s0 * w, Q.s1 * w);
                    }
                }
            }
        }
        ra.fold();
    }
    if (lane >= TH) return;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        int lx = rb0 + r;
        if (lx >= TW) break;
        if (it.slab >= 0) {
            unsigned long long* dst = slabs + (long long)it.slab * NOUT * kTilePix;
            dst[lx * kTile + lane] = ra.word0(r);
            if (NOUT == 2) dst[kTilePix + lx * kTile + lane] = ra.word1(r);
        } else {
            long long o = (long long)(X0 + lx) * g.ny + (Y0 + lane);
            emit_pixel<NOUT, ACC>(o, ra.word0(r), NOUT == 2 ? ra.word1(r) : 0ull, kk.x, kk.y,
                                  out0, out1, flags);
        }
    }
}

// Lane-per-record deposit of a box of at most S x S pixels: dy^2 per column in
// registers, an unrolled S x S pass decides every pair whose fp32 r2 is outside the error
// band and accumulates it; band pairs (~0.1 %) only set a bit, resolved afterwards in
// fp64 -- keeping the rare slow path out of the unrolled body.
template <int KID, int NOUT, int ACC, int S>
__device__ __forceinline__ void small_box(const Grid& g, const Prep& P, int bw, int bh, int X0,
                                          int Y0, const float* xt, const float* yt,
                                          unsigned long long* acc0, unsigned long long* acc1) {
    const int base = (P.b.x0 - X0) * kTile + (P.b.y0 - Y0);  // LDS word of pixel (0, 0)
    float dy2[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
        float dy = P.v - yt[min(P.b.y0 + j, P.b.y1) - Y0];
        dy2[j] = dy * dy;
    }
    unsigned amb = 0u;
#pragma unroll
    for (int ii = 0; ii < S; ++ii) {
        if (ii < bw) {
            int xi = P.b.x0 + ii;
            float dx = P.u - xt[xi - X0];
            float dx2 = dx * dx;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                if (j < bh) {
                    float r2 = dx2 + dy2[j];
                    bool a = r2 >= P.lo && r2 <= P.hi;
                    amb |= a ? (1u << (ii * S + j)) : 0u;
                    if (r2 < P.lo)
                        accumulate<KID, NOUT, ACC>(P, r2, acc0, acc1, base + ii * kTile + j);
                }
            }
        }
    }
    while (amb) {
        int bit = __builtin_ctz(amb);
        amb &= amb - 1u;
        int ii = bit / S, j = bit - (bit / S) * S;
        int xi = P.b.x0 + ii, yi = P.b.y0 + j;
        if (exact_pair(g, P.u, P.v, P.h, xi, yi)) {
            float dx = P.u - xt[xi - X0], dy = P.v - yt[yi - Y0];
            accumulate<KID, NOUT, ACC>(P, dx * dx + dy * dy, acc0, acc1,
                                       (xi - X0) * kTile + (yi - Y0));
        }
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) {  // v_pk_fma_f32
    return __builtin_elementwise_fma(a, b, c);
}

// Kernel shape on two pairs at once (packed fp32: v_pk_fma_f32 / v_pk_mul_f32).  Only
// pairs with fp32 r2 < (2h)^2 use the result, so q < 2 up to rounding and the Wendland
// clamp is not needed there (a q a few ulp over 2 gives a term ~1e-28 of the peak).
template <int KID>
__device__ __forceinline__ f2v kernel_shape2(f2v q) {
    if constexpr (KID == 0) {
        f2v q2 = q * q;
        f2v a = fma2(q2, fma2(q, f2v{0.75f, 0.75f}, f2v{-1.5f, -1.5f}), f2v{1.0f, 1.0f});
        f2v t = f2v{2.0f, 2.0f} - q;
        f2v b = (t * t) * (t * 0.25f);
        return f2v{q.x < 1.0f ? a.x : b.x, q.y < 1.0f ? a.y : b.y};
    } else if constexpr (KID == 1) {
        f2v t = fma2(q, f2v{-0.5f, -0.5f}, f2v{1.0f, 1.0f});
        f2v t2 = t * t;
        return (t2 * t2) * fma2(q, f2v{2.0f, 2.0f}, f2v{1.0f, 1.0f});
    } else {
        return f2v{1.0f, 1.0f};
    }
}

__device__ __forceinline__ f2v sqrt2(f2v x) {
    return f2v{__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
}

// Lane-per-record deposit of a box of at most 3 x 3 pixel corners (pixel-scale h), the
// common case: the nine fp32 r2 and kernel values are computed branch-free in packed
// fp32, and every pair with r2 < (2h)^2 is added.  Valid only when no pair lies in the
// error band (min |r2 - thr| > band): returns false for such a record WITHOUT touching the
// tile; the caller defers it to the exact path (small_box).
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ bool small3_fast(const Prep& P, int bw, int bh, int X0, int Y0,
                                            const float* xt, const float* yt,
                                            unsigned long long* acc0, unsigned long long* acc1) {
    constexpr float kFar = 1e18f;  // outside the box: r2 ~ 1e36, far from any threshold
    float dx2[3];
    f2v dy2;
    float dyc2;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float d = P.u - xt[min(P.b.x0 + i, P.b.x1) - X0];
        d = i < bw ? d : kFar;
        dx2[i] = d * d;
    }
    {
        float d0 = P.v - yt[P.b.y0 - Y0];
        float d1 = P.v - yt[min(P.b.y0 + 1, P.b.y1) - Y0];
        float d2 = P.v - yt[min(P.b.y0 + 2, P.b.y1) - Y0];
        d1 = bh > 1 ? d1 : kFar;
        d2 = bh > 2 ? d2 : kFar;
        f2v d = f2v{d0, d1};
        dy2 = d * d;
        dyc2 = d2 * d2;
    }
    f2v r2[3];
    float r2c[3];
    float m = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        r2[i] = dy2 + dx2[i];
        r2c[i] = dx2[i] + dyc2;
        f2v e = r2[i] - P.thr;
        m = fminf(m, fminf(fminf(fabsf(e.x), fabsf(e.y)), fabsf(r2c[i] - P.thr)));
    }
    if (!(m > P.band)) return false;  // a pair in the band (or NaN): exact path
#if ASP_ABLATE == 4  // diagnostic: lanes of each 32-lane half on distinct LDS banks (wrong map)
    const int base = ((P.b.x0 - X0) & 60) * kTile + (threadIdx.x & 31);
#else
    const int base = (P.b.x0 - X0) * kTile + (P.b.y0 - Y0);
#endif
    const f2v hv = f2v{P.hinv, P.hinv};
    // column j = 2 of rows 0, 1 as one packed pair, row 2 with a dummy partner
    f2v wc01 = kernel_shape2<KID>(sqrt2(f2v{r2c[0], r2c[1]}) * hv);
    f2v wc2 = kernel_shape2<KID>(sqrt2(f2v{r2c[2], 0.0f}) * hv);
    const float wc[3] = {wc01.x, wc01.y, wc2.x};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        f2v w = kernel_shape2<KID>(sqrt2(r2[i]) * hv);
        f2v t0 = w * P.s0, t1 = w * P.s1;
        f2v c = f2v{wc[i], wc[i]} * f2v{P.s0, P.s1};
        const int k = base + i * kTile;
        if (r2[i].x < P.thr) {
            acc_add<ACC>(&acc0[k], t0.x);
            if constexpr (NOUT == 2) acc_add<ACC>(&acc1[k], t1.x);
        }
        if (r2[i].y < P.thr) {
            acc_add<ACC>(&acc0[k + 1], t0.y);
            if constexpr (NOUT == 2) acc_add<ACC>(&acc1[k + 1], t1.y);
        }
        if (r2c[i] < P.thr) {
            acc_add<ACC>(&acc0[k + 2], c.x);
            if constexpr (NOUT == 2) acc_add<ACC>(&acc1[k + 2], c.y);
        }
    }
    return true;
}

#ifndef ASP_FAST3
#define ASP_FAST3 1  // 0: diagnostic builds only, the unpacked 3 x 3 body with in-loop band pairs
#endif

#ifndef ASP_DEP_THREADS
#define ASP_DEP_THREADS 512
#endif
// k_deposit workgroup: two per CU (64 KiB fp64 LDS tile each)
constexpr int kDepThreads = ASP_DEP_THREADS;

// Per-wave list of records deferred to the exact path (a pair in the error band).
constexpr int kDeferCap = 128;

// Exact body for deferred records: lanes 0 .. cnt-1 take list entries first .. first+cnt-1
// (record indices within the item), reload and re-prepare them and decide every pair
// with the error-band / fp64 logic of small_box.  Wave-level: no block barrier.
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void deferred(const Grid& g, const float4* __restrict__ recs,
                                      long long start, const int* dlist, int first, int cnt,
                                      int X0, int Y0, int TW, int TH, int2 kk, const float* xt,
                                      const float* yt, unsigned long long* acc0,
                                      unsigned long long* acc1, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int idx = lane < cnt ? dlist[first + lane] : -1;
    __builtin_amdgcn_wave_barrier();
    if (idx < 0) return;
    float4 r0, r1 = make_float4(0.f, 0.f, 0.f, 0.f);
    load_rec4<NOUT>(recs, start + idx, r0, r1);
    Prep P;
    if (!rec_prep<KID, NOUT, ACC>(g, r0, r1, X0, Y0, TW, TH, kk, P)) return;
    small_box<KID, NOUT, ACC, 4>(g, P, P.b.x1 - P.b.x0 + 1, P.b.y1 - P.b.y0 + 1, X0, Y0, xt, yt,
                                 acc0, acc1);
}

// ----------------------------------------------------------------------------------
// K4: deposit one work item (a run of records of one tile) into LDS, then write the
// tile (single-item tiles) or its int64 partial slab (split tiles).
// ----------------------------------------------------------------------------------
// Gathered large records (GATHER): a batch's large-box records go to an LDS list (SoA,
// one batch = kDepThreads records at most); after a block barrier every thread tests the
// list against the 8 pixels it owns (row = tid / 8, columns 8 (tid % 8) ..), with the
// same fp32 decision + fp64 band fallback as decide(), and keeps register sums, added to
// its own LDS words once per batch: no per-pair atomics.  fp64 accumulation only.
constexpr int kGFields = 10;  // u v h lo hi hinv s0 s1 box(x0|x1<<8|y0<<16|y1<<24, tile-local)
constexpr size_t kGatherLds = (size_t)kGFields * kDepThreads * 4 + 2 * sizeof(int);

template <int KID, int NOUT>
__device__ __forceinline__ void gather_list(const Grid& g, const float* gl, int nl, int X0,
                                            int Y0, int TW, int TH, const float* xt,
                                            const float* yt, unsigned long long* acc0,
                                            unsigned long long* acc1) {
    const int row = threadIdx.x >> 3, col0 = (threadIdx.x & 7) * 8;
    if (row >= TW || col0 >= TH) return;
    const float X = xt[row];
    float Yv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Yv[j] = yt[min(col0 + j, kTile - 1)];
    double s0[8], s1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.0;
    const float *gu = gl, *gv = gl + kDepThreads, *gh = gl + 2 * kDepThreads,
                *glo = gl + 3 * kDepThreads, *ghi = gl + 4 * kDepThreads,
                *ghv = gl + 5 * kDepThreads, *gs0 = gl + 6 * kDepThreads,
                *gs1 = gl + 7 * kDepThreads;
    const unsigned* gb = (const unsigned*)(gl + 8 * kDepThreads);
    for (int e = 0; e < nl; ++e) {
        unsigned bx = gb[e];
        int x0 = bx & 255, x1 = (bx >> 8) & 255, y0 = (bx >> 16) & 255, y1 = bx >> 24;
        if (row < x0 || row > x1 || col0 + 7 < y0 || col0 > y1) continue;
        const float u = gu[e], v = gv[e], lo = glo[e], hi = ghi[e];
        const float dx = u - X;
        const float dx2 = dx * dx;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = col0 + j;
            if (c < y0 || c > y1) continue;
            float dy = v - Yv[j];
            float r2 = dx2 + dy * dy;
            bool in = r2 < lo;
            if (r2 >= lo && r2 <= hi) in = exact_pair(g, u, v, gh[e], X0 + row, Y0 + c);
            if (in) {
                float w = kernel_shape<KID>(__builtin_amdgcn_sqrtf(r2) * ghv[e]);
                s0[j] += (double)(gs0[e] * w);
                if constexpr (NOUT == 2) s1[j] += (double)(gs1[e] * w);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (col0 + j >= TH) continue;
        const int k = row * kTile + col0 + j;
        double* a0 = (double*)&acc0[k];
        *a0 += s0[j];
        if constexpr (NOUT == 2) {
            double* a1 = (double*)&acc1[k];
            *a1 += s1[j];
        }
    }
}

template <int KID, int NOUT, int ACC, bool GATHER = false>
__global__ __launch_bounds__(kDepThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_deposit(
    Grid g, const float4* __restrict__ recs, const Item* __restrict__ items,
    const int2* __restrict__ tile_k, unsigned long long* __restrict__ slabs,
    float* __restrict__ out0, float* __restrict__ out1, int flags) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];
    unsigned long long* acc0 = acc;
    unsigned long long* acc1 = acc + kTilePix;
    float* xt = (float*)(acc + NOUT * kTilePix);
    float* yt = xt + kTile;
    float* gl = yt + kTile;                          // GATHER: the list (SoA)
    int* gcnt = (int*)(gl + kGFields * kDepThreads);  // GATHER: two list counters
    const Item it = items[blockIdx.x];
    if (it.mode != 0) return;  // K4b's
    int tx = it.tile / g.nty, ty = it.tile - (it.tile / g.nty) * g.nty;
    int X0 = tx * kTile, Y0 = ty * kTile;
    int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    if (it.count == 0) {  // empty tile: the map is 0 there
        if (flags & kFlagAccumulate) {
            // last chunk of a chunked mass-weighted map: the earlier chunks left the two
            // raw sums here, the ratio is still to be taken
            if constexpr (NOUT == 2) {
                if (flags & kFlagRatio) {
                    for (int k = threadIdx.x; k < kTilePix; k += kDepThreads) {
                        int lx = k >> kTileShift, ly = k & (kTile - 1);
                        if (lx >= TW || ly >= TH) continue;
                        long long o = (long long)(X0 + lx) * g.ny + (Y0 + ly);
                        float v1 = out1[o];
                        out0[o] = v1 != 0.0f ? out0[o] / v1 : 0.0f;
                    }
                }
            }
            return;
        }
        for (int k = threadIdx.x; k < kTilePix; k += kDepThreads) {
            int lx = k >> kTileShift, ly = k & (kTile - 1);
            if (lx >= TW || ly >= TH) continue;
            long long o = (long long)(X0 + lx) * g.ny + (Y0 + ly);
            out0[o] = 0.0f;
            if (NOUT == 2) out1[o] = 0.0f;
        }
        return;
    }
    const int2 kk = ACC == kAccFix ? tile_k[it.tile] : make_int2(0, 0);
    if (GATHER && threadIdx.x == 0) gcnt[0] = gcnt[1] = 0;  // the prologue's barrier orders it
    tile_prologue<NOUT, kDepThreads>(g, X0, Y0, acc, xt, yt);
    {
        __shared__ int defer_lds[kDepThreads / 64][kDeferCap];
        int lane = threadIdx.x & 63;
        int* dlist = defer_lds[threadIdx.x >> 6];
        int ndef = 0;  // wave-uniform
        // Software pipeline, two batches deep: batches i+1 and i+2 load while batch i deposits
        // (16 waves/CU x 64 lanes x 32 B x 2 in flight per CU).
        float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, q0 = r0, q1 = r0;
        if ((int)threadIdx.x < it.count) load_rec4<NOUT>(recs, it.start + threadIdx.x, r0, r1);
        if ((int)threadIdx.x + kDepThreads < it.count)
            load_rec4<NOUT>(recs, it.start + threadIdx.x + kDepThreads, q0, q1);
        for (int base = 0; base < it.count; base += kDepThreads) {
            int i = base + threadIdx.x;
            float4 n0 = make_float4(0.f, 0.f, 0.f, 0.f), n1 = n0;
            if (i + 2 * kDepThreads < it.count)
                load_rec4<NOUT>(recs, it.start + i + 2 * kDepThreads, n0, n1);
            Prep P;
            P.b = Box{0, -1, 0, -1};
            bool live = false;
    #if ASP_ABLATE == 3
            asm volatile("" ::"v"(r0.x), "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x));
            r0 = q0; r1 = q1; q0 = n0; q1 = n1;
            continue;
    #endif
            if (i < it.count)
                live = rec_prep<KID, NOUT, ACC>(g, r0, r1, X0, Y0, TW, TH, kk, P);
            r0 = q0;
            r1 = q1;
            q0 = n0;
            q1 = n1;
    #if ASP_ABLATE == 2
            asm volatile("" ::"v"(P.u), "v"(P.v), "v"(P.lo), "v"(P.hi), "v"(P.s0), "v"(P.s1),
                         "v"(P.b.x0), "v"(P.b.y1), "v"(live ? 1 : 0));
            continue;
    #endif
            int bw = P.b.x1 - P.b.x0 + 1, bh = P.b.y1 - P.b.y0 + 1;
            bool small = live && bw <= 4 && bh <= 4;
            bool amb = false;
            if (small) {
                // lane-per-record.  Boxes of <= 3 x 3 corners (pixel-scale h: a 2h = 1.5 px
                // disc spans 3 corners per axis unless its centre sits within the box
                // margin of a half-pixel) take the packed body; 4-wide boxes and records
                // with a pair in the error band are deferred to the exact body, a full
                // wave of them at a time
#if ASP_FAST3
                if (bw <= 3 && bh <= 3)
                    amb = !small3_fast<KID, NOUT, ACC>(P, bw, bh, X0, Y0, xt, yt, acc0, acc1);
                else
                    amb = true;
#else
                if (__ballot(bw > 3 || bh > 3) == 0ull)
                    small_box<KID, NOUT, ACC, 3>(g, P, bw, bh, X0, Y0, xt, yt, acc0, acc1);
                else
                    small_box<KID, NOUT, ACC, 4>(g, P, bw, bh, X0, Y0, xt, yt, acc0, acc1);
#endif
            }
            {
                unsigned long long am = __ballot(amb);
                if (am) {
                    if (amb) dlist[ndef + __popcll(am & ((1ull << lane) - 1ull))] = i;
                    ndef += __popcll(am);
                    if (ndef >= 64) {  // a full wave of deferred records
                        ndef -= 64;
                        deferred<KID, NOUT, ACC>(g, recs, it.start, dlist, ndef, 64, X0, Y0, TW, TH, kk,
                                                 xt, yt, acc0, acc1, lane);
                    }
                }
            }
            if constexpr (GATHER) {
                // list counter of this batch: gcnt[parity]; the other one is reset here for
                // the next batch (nobody touches it before the barrier that ends this one)
                const int par = (base / kDepThreads) & 1;
                if (live && !small) {
                    int e = atomicAdd(&gcnt[par], 1);
                    gl[e] = P.u;
                    gl[kDepThreads + e] = P.v;
                    gl[2 * kDepThreads + e] = P.h;
                    gl[3 * kDepThreads + e] = P.lo;
                    gl[4 * kDepThreads + e] = P.hi;
                    gl[5 * kDepThreads + e] = P.hinv;
                    gl[6 * kDepThreads + e] = P.s0;
                    gl[7 * kDepThreads + e] = P.s1;
                    gl[8 * kDepThreads + e] = __uint_as_float(
                        (unsigned)(P.b.x0 - X0) | ((unsigned)(P.b.x1 - X0) << 8) |
                        ((unsigned)(P.b.y0 - Y0) << 16) | ((unsigned)(P.b.y1 - Y0) << 24));
                }
                __syncthreads();
                const int nl = gcnt[par];
                if (threadIdx.x == 0) gcnt[par ^ 1] = 0;
                if (nl) gather_list<KID, NOUT>(g, gl, nl, X0, Y0, TW, TH, xt, yt, acc0, acc1);
                __syncthreads();
            } else {
                unsigned long long big = __ballot(live && !small);
                while (big) {
                    int l = __builtin_ctzll(big);
                    big &= big - 1;
                    Prep Q = bcast_prep(P, l);
                    sweep<KID, NOUT, ACC>(g, Q, X0, Y0, xt, yt, acc0, acc1, lane);
                }
            }
        }
        if (ndef > 0)
            deferred<KID, NOUT, ACC>(g, recs, it.start, dlist, 0, ndef, X0, Y0, TW, TH, kk, xt, yt,
                                     acc0, acc1, lane);
    }
    __syncthreads();
    if (it.slab >= 0) {  // split tile: exact partial sums, merged by K5
        unsigned long long* dst = slabs + (long long)it.slab * NOUT * kTilePix;
        for (int k = threadIdx.x; k < NOUT * kTilePix; k += kDepThreads) dst[k] = acc[k];
        return;
    }
    for (int k = threadIdx.x; k < kTilePix; k += kDepThreads) {
        int lx = k >> kTileShift, ly = k & (kTile - 1);
        if (lx >= TW || ly >= TH) continue;
        long long o = (long long)(X0 + lx) * g.ny + (Y0 + ly);
        emit_pixel<NOUT, ACC>(o, acc0[k], NOUT == 2 ? acc1[k] : 0ull, kk.x, kk.y, out0, out1,
                              flags);
    }
}

// K4b: mode-1 items (non-small records), row bands; grid (items, 2): blockIdx.y picks
// the tile half, each of the 4 waves 8 rows of it.  Writes the tile (or its slab half).
template <int KID, int NOUT, int ACC>
__global__ __launch_bounds__(kBlock) void k_band(Grid g, const float4* __restrict__ recs,
                                                 const Item* __restrict__ items,
                                                 const int2* __restrict__ tile_k,
                                                 unsigned long long* __restrict__ slabs,
                                                 float* __restrict__ out0,
                                                 float* __restrict__ out1, int flags) {
    __shared__ float xt[kTile], yt[kTile];
    const Item it = items[blockIdx.x];
    if (it.mode != 1) return;
    int tx = it.tile / g.nty, ty = it.tile - (it.tile / g.nty) * g.nty;
    int X0 = tx * kTile, Y0 = ty * kTile;
    int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    if ((int)blockIdx.y * 32 >= TW) return;
    const int2 kk = ACC == kAccFix ? tile_k[it.tile] : make_int2(0, 0);
    if (threadIdx.x < kTile)
        xt[threadIdx.x] = (float)corner_x(g, X0 + threadIdx.x);
    else if (threadIdx.x < 2 * kTile)
        yt[threadIdx.x - kTile] = (float)corner_y(g, Y0 + threadIdx.x - kTile);
    __syncthreads();
    static_assert(kBlock == 4 * 64, "row bands: 4 waves x 8 rows per tile half");
    band_item<KID, NOUT, ACC>(g, recs, it, X0, Y0, TW, TH, kk, xt, yt, slabs, out0, out1, flags);
}

// ----------------------------------------------------------------------------------
// K5: split tiles -- exact int64 sum of the item slabs, convert, write.  Grid
// (merges, kTilePix / kBlock): each workgroup one 4-row strip of a tile, one pixel per
// thread; the slab loop issues kMergeBatch independent loads per map before summing them
// in slab order (deterministic), so a thread has up to 2 x kMergeBatch loads in flight.
// ----------------------------------------------------------------------------------
constexpr int kMergeBatch = 8;
template <int NOUT, int ACC>
__global__ __launch_bounds__(kBlock) void k_merge(Grid g, const Merge* __restrict__ merges,
                                                  const unsigned long long* __restrict__ slabs,
                                                  const int2* __restrict__ tile_k,
                                                  float* __restrict__ out0,
                                                  float* __restrict__ out1, int flags) {
    const Merge m = merges[blockIdx.x];
    int tx = m.tile / g.nty, ty = m.tile - (m.tile / g.nty) * g.nty;
    int X0 = tx * kTile, Y0 = ty * kTile;
    int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    const int k = blockIdx.y * kBlock + threadIdx.x;
    int lx = k >> kTileShift, ly = k & (kTile - 1);
    if (lx >= TW || ly >= TH) return;
    const int2 kk = ACC == kAccFix ? tile_k[m.tile] : make_int2(0, 0);
    const unsigned long long* src = slabs + (long long)m.slab0 * NOUT * kTilePix + k;
    unsigned long long s0 = 0, s1 = 0;  // +0.0 in fp64 as well
    int j = 0;
    for (; j + kMergeBatch <= m.nslab; j += kMergeBatch) {
        unsigned long long b0[kMergeBatch], b1[kMergeBatch];
#pragma unroll
        for (int q = 0; q < kMergeBatch; ++q) {
            const unsigned long long* p = src + (long long)(j + q) * NOUT * kTilePix;
            b0[q] = p[0];
            b1[q] = NOUT == 2 ? p[kTilePix] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < kMergeBatch; ++q) {  // fixed slab order: deterministic
            s0 = acc_sum<ACC>(s0, b0[q]);
            if (NOUT == 2) s1 = acc_sum<ACC>(s1, b1[q]);
        }
    }
    for (; j < m.nslab; ++j) {
        const unsigned long long* p = src + (long long)j * NOUT * kTilePix;
        s0 = acc_sum<ACC>(s0, p[0]);
        if (NOUT == 2) s1 = acc_sum<ACC>(s1, p[kTilePix]);
    }
    long long o = (long long)(X0 + lx) * g.ny + (Y0 + ly);
    emit_pixel<NOUT, ACC>(o, s0, s1, kk.x, kk.y, out0, out1, flags);
}

// ----------------------------------------------------------------------------------
// K6: wide particles (footprint over > kWideTiles tiles): they are never binned.  One
// workgroup per tile walks the wide list kGatherCap particles at a time, keeps those
// whose clipped box meets the tile and gathers them (register sums, no per-pair
// atomics); fixed point with the wide particles' own bound.  Adds onto the tile K4/K5
// wrote (this workgroup is its only writer).
// ----------------------------------------------------------------------------------
template <int KID, int NOUT, int ACC>
__global__ __launch_bounds__(kDepBlock) void k_wide(Grid g, const float* __restrict__ u,
                                                    const float* __restrict__ v,
                                                    const float* __restrict__ h,
                                                    const float* __restrict__ a0,
                                                    const float* __restrict__ a1,
                                                    const int* __restrict__ wide_list, int n_wide,
                                                    const int* __restrict__ ctr,
                                                    float* __restrict__ out0,
                                                    float* __restrict__ out1) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];
    unsigned long long* acc0 = acc;
    unsigned long long* acc1 = acc + kTilePix;
    float* xt = (float*)(acc + NOUT * kTilePix);
    float* yt = xt + kTile;
    __shared__ GRec glist[kGatherCap];
    __shared__ int gcount;
    int t = blockIdx.x;
    int tx = t / g.nty, ty = t - (t / g.nty) * g.nty;
    int X0 = tx * kTile, Y0 = ty * kTile;
    int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    tile_prologue<NOUT, kDepBlock>(g, X0, Y0, acc, xt, yt);
    int k0 = ACC == kAccFix ? scale_exp(n_wide, __uint_as_float((unsigned)ctr[cWideMax0])) : 0;
    int k1 = (ACC == kAccFix && NOUT == 2)
                 ? scale_exp(n_wide, __uint_as_float((unsigned)ctr[cWideMax1])) : 0;
    bool any = false;
    for (int c = 0; c < n_wide; c += kGatherCap) {
        Prep P;
        bool live = false;
        int k = c + (int)threadIdx.x;
        if (threadIdx.x < kGatherCap && k < n_wide) {
            int p = wide_list[k];
            live = prep_record<KID, ACC>(g, u[p], v[p], h[p], a0[p], NOUT == 2 ? a1[p] : 0.0f, k0,
                                         k1, P) &&
                   clip(P.b, X0, Y0, TW, TH);
        }
        if (__syncthreads_or(live)) {
            any = true;
            gather_rounds<KID, NOUT, ACC>(g, live, P, X0, Y0, glist, &gcount, xt, yt, acc0, acc1);
        }
    }
    if (!any) return;  // uniform: every thread saw the same __syncthreads_or results
    __syncthreads();
    for (int k = threadIdx.x; k < kTilePix; k += kDepBlock) {
        int lx = k >> kTileShift, ly = k & (kTile - 1);
        if (lx >= TW || ly >= TH) continue;
        long long o = (long long)(X0 + lx) * g.ny + (Y0 + ly);
        emit_pixel<NOUT, ACC>(o, acc0[k], NOUT == 2 ? acc1[k] : 0ull, k0, k1, out0, out1,
                              kFlagAccumulate);
    }
}

// K7: out0 <- out0 / out1 (0 where out1 == 0).
__global__ __launch_bounds__(kBlock) void k_ratio(float* __restrict__ out0,
                                                  const float* __restrict__ out1, long long m) {
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long stride = (long long)gridDim.x * kBlock;
    for (; i < m; i += stride) {
        float d = out1[i];
        out0[i] = d != 0.0f ? out0[i] / d : 0.0f;
    }
}

// ----------------------------------------------------------------------------------
// Auxiliary entry points: kernel evaluation, chunk ranges, neighbour lists.
// ----------------------------------------------------------------------------------
__global__ void k_kernel_eval(int kid, const double* __restrict__ r, const double* __restrict__ h,
                              double* __restrict__ w, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double q = r[i] / h[i];
    double res = 0.0;
    if (kid == ASP_KERNEL_CUBIC_SPLINE) {  // _kernels.pyx:13-19, same branch order
        if (q < 1.0)
            res = (1 - 1.5 * pow(q, 2.0) + 0.75 * pow(q, 3.0)) / (M_PI * pow(h[i], 3.0));
        else if (q < 2.0)
            res = (0.25 * pow((2 - q), 3.0)) / (M_PI * pow(h[i], 3.0));
    } else if (kid == ASP_KERNEL_WENDLAND_C2) {
        if (q < 2.0) {
            double t = 1.0 - 0.5 * q;
            res = 21.0 / (16.0 * M_PI * pow(h[i], 3.0)) * pow(t, 4.0) * (1.0 + 2.0 * q);
        }
    } else {
        res = 1.0;
    }
    w[i] = res;
}

__global__ void k_chunk_ranges(Grid g, const float* __restrict__ u, const float* __restrict__ v,
                               const float* __restrict__ h, long long n, int* cx0, int* cx1,
                               int* cy0, int* cy1) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int a, b, c, d;
    chunk_range((double)u[i], (double)h[i], g.x_min, g.psx, g.nx, g.cs, a, b);
    chunk_range((double)v[i], (double)h[i], g.y_min, g.psy_cull, g.ny, g.cs, c, d);
    cx0[i] = a;
    cx1[i] = b;
    cy0[i] = c;
    cy1[i] = d;
}

// Neighbour lists: one workgroup per pixel, particles in ascending order.  The decision
// is the deposit's (footprint box, then decide()), so this lists exactly the pairs the
// deposit accumulates.  pass 0 counts, pass 1 writes at offsets[pixel].
__global__ __launch_bounds__(kBlock) void k_neighbours(Grid g, const float* __restrict__ u,
                                                       const float* __restrict__ v,
                                                       const float* __restrict__ h, long long n,
                                                       const long long* __restrict__ pixels,
                                                       long long* __restrict__ counts,
                                                       const long long* __restrict__ offsets,
                                                       int* __restrict__ index, long long cap,
                                                       int pass) {
    __shared__ int wsum[kBlock / 64];
    __shared__ long long run;
    long long pix = pixels[blockIdx.x];
    int xi = (int)(pix / g.ny), yi = (int)(pix - (pix / g.ny) * g.ny);
    float X = (float)corner_x(g, xi), Y = (float)corner_y(g, yi);
    if (threadIdx.x == 0) run = pass ? offsets[blockIdx.x] : 0;
    __syncthreads();
    int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (long long base = 0; base < n; base += kBlock) {
        long long p = base + threadIdx.x;
        bool in = false;
        if (p < n) {
            Prep P;
            if (prep_record<2>(g, u[p], v[p], h[p], 0.0f, 0.0f, 0, 0, P) && xi >= P.b.x0 &&
                xi <= P.b.x1 && yi >= P.b.y0 && yi <= P.b.y1) {
                float r2;
                in = decide(g, P, xi, yi, X, Y, r2);
            }
        }
        unsigned long long m = __ballot(in);
        if (lane == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int before = 0, tot = 0;
        for (int k = 0; k < kBlock / 64; ++k) {
            if (k < wv) before += wsum[k];
            tot += wsum[k];
        }
        if (pass && in) {
            long long slot = run + before + __popcll(m & ((1ull << lane) - 1ull));
            if (slot < cap) index[slot] = (int)p;
        }
        __syncthreads();
        if (threadIdx.x == 0) run += tot;
        __syncthreads();
    }
    if (!pass && threadIdx.x == 0) counts[blockIdx.x] = run;
}

static uint32_t spread_bits(uint32_t x) {
    x &= 0xffff;
    x = (x | (x << 8)) & 0x00ff00ff;
    x = (x | (x << 4)) & 0x0f0f0f0f;
    x = (x | (x << 2)) & 0x33333333;
    x = (x | (x << 1)) & 0x55555555;
    return x;
}

static int ensure_morton(Workspace& ws, int ntx, int nty, hipStream_t st) {
    if (ws.morton_ntx == ntx && ws.morton_nty == nty) return ASP_OK;
    std::vector<std::pair<uint32_t, int>> key((size_t)ntx * nty);
    for (int tx = 0; tx < ntx; ++tx)
        for (int ty = 0; ty < nty; ++ty)
            key[(size_t)tx * nty + ty] = {spread_bits(tx) << 1 | spread_bits(ty), tx * nty + ty};
    std::sort(key.begin(), key.end());
    std::vector<int> order(key.size());
    for (size_t i = 0; i < key.size(); ++i) order[i] = key[i].second;
    ASP_TRY(ensure(ws.morton, order.size() * sizeof(int)));
    ASP_HIP(hipMemcpyAsync(ws.morton.p, order.data(), order.size() * sizeof(int),
                           hipMemcpyHostToDevice, st));
    ASP_HIP(hipStreamSynchronize(st));
    ws.morton_ntx = ntx;
    ws.morton_nty = nty;
    return ASP_OK;
}

static bool make_grid(double x_min, double x_max, double y_min, double y_max, int nx, int ny,
                      int cs, Grid& g) {
    if (!(nx > 0 && ny > 0 && cs > 0)) return false;
    if (!(x_max > x_min) || !(y_max > y_min)) return false;
    if (!std::isfinite(x_min) || !std::isfinite(x_max) || !std::isfinite(y_min) ||
        !std::isfinite(y_max))
        return false;
    g.x_min = x_min;
    g.y_min = y_min;
    g.psx = (x_max - x_min) / nx;
    g.psy_pix = (y_max - y_min) / nx;
    g.psy_cull = (y_max - y_min) / ny;
    if (!(g.psx > 0.0) || !(g.psy_pix > 0.0) || !(g.psy_cull > 0.0)) return false;
    g.xminf = (float)x_min;
    g.yminf = (float)y_min;
    g.ipsx = (float)(1.0 / g.psx);
    g.ipsy = (float)(1.0 / g.psy_pix);
    if (!std::isfinite(g.ipsx) || !std::isfinite(g.ipsy)) return false;
    double mg = std::max({std::fabs(x_min), std::fabs(x_min + nx * g.psx), std::fabs(y_min),
                          std::fabs(y_min + ny * g.psy_pix)});
    g.mg = (float)(mg * (1.0 + 1e-6));
    g.nx = nx;
    g.ny = ny;
    g.cs = cs;
    g.ncx = (nx + cs - 1) / cs;
    g.ncy = (ny + cs - 1) / cs;
    g.ntx = (nx + kTile - 1) / kTile;
    g.nty = (ny + kTile - 1) / kTile;
    g.ntiles = g.ntx * g.nty;
    g.nonsquare = nx != ny;
    g.band_cols = kTile + 1;  // row bands off unless project2d enables them
    g.nstream = 1;
    g.wide_tiles = kWideTiles;
    return true;
}

constexpr int kMaxBinBlocks = 1024;  // count / scatter workgroups (hist rows)
constexpr int kMaxTiles = 4096;  // K1/K3 LDS: 2 cursors + per-tile max (16 B/tile at 2 maps)
static_assert(kMaxTiles <= kScanThreads * 4, "k_tilescan holds <= kScanPer tiles per thread");

// The particles are cut into nch chunks (contiguous runs of count workgroups).  Every
// chunk has its own tile-sorted record region, work list and slabs, so chunk c can be
// deposited (side stream) while chunk c + 1 is scattered: the scatter is bound by
// scattered-store issue, the deposit by VALU / LDS, and the two overlap.
struct Chunk {
    long long blk0, nblk_s;  // first scatter workgroup, scatter workgroups
    long long rec0, n_recs;  // record region
    int n_items, n_merges, n_slabs, slab0;
};

struct Plan {
    long long n, nblk, per_block;
    long long nblk_s;  // scatter workgroups (grp count workgroups each)
    int grp;           // count workgroups per scatter workgroup
    long long cb;      // count workgroups per chunk (a multiple of grp)
    int nch;           // chunks
    Chunk ch[kMarks];
    int n_items, n_merges, n_slabs, n_wide;
    long long n_recs;
};

constexpr long long kChunkMinParticles = 1LL << 22;  // below: one chunk
#ifndef ASP_CHUNKS
#define ASP_CHUNKS 1
#endif
constexpr int kChunks = ASP_CHUNKS;

// items / merges per chunk in the work-list buffers
static inline size_t item_cap(const Grid& g) { return (size_t)2 * g.ntiles + kTargetItems + kTargetItems1 + 16; }
static inline size_t merge_cap(const Grid& g) { return (size_t)g.ntiles + 16; }

// One chunk's scatter (K3) on stream st.  rec_cap / wide_cap: the capacities the kernel
// checks against the device counters (speculative launch; see project2d).
template <int KID, int NOUT, int ACC>
static int launch_scatter(const Grid& g, Workspace& ws, const Plan& pl, int c, const float* u,
                          const float* v, const float* h, const float* a0, const float* a1,
                          long long rec_cap, int wide_cap, hipStream_t st) {
    int* dc = (int*)ws.counters.p;
    const Chunk& ck = pl.ch[c];
    float4* recs = (float4*)ws.recs.p + ck.rec0 * NOUT;
    StageMark m(ws, kSScatter, st);
    size_t lds = (size_t)g.nstream * g.ntiles * sizeof(int) +
                 (NOUT == 2 ? (size_t)(kScatterBlock / 64) * 128 * sizeof(float4) : 0) +
                 (ACC == kAccFix ? (size_t)g.ntiles * NOUT * sizeof(unsigned) : 0);
    hipLaunchKernelGGL((k_scatter<KID, NOUT, ACC>), dim3((unsigned)ck.nblk_s), dim3(kScatterBlock),
                       lds, st, u, v, h, a0, a1, pl.n, ASP_INTERLEAVE ? pl.nblk : pl.per_block * pl.grp, g,
                       (const int*)ws.hist.p,
                       (const long long*)ws.tile_start.p + (long long)c * 2 * g.ntiles, recs,
                       (unsigned*)ws.cmx.p, (int*)ws.wide.p, dc, (int)ck.blk0, pl.grp,
                       rec_cap, wide_cap);
    ASP_LAUNCHED();
    m.done();
    return ASP_OK;
}

// K3..K7 for one kernel / map count.  Scatters run on the caller's stream st; with several
// chunks the deposits run on the workspace's side stream, each behind its chunk's scatter
// (one event per chunk), and st waits for the side stream at the end.
template <int KID, int NOUT, int ACC>
static int run_tail(const Grid& g, Workspace& ws, const Plan& pl, const float* u,
                    const float* v, const float* h, const float* a0, const float* a1, float* o0,
                    float* o1, int flags, hipStream_t st, bool pre_scattered) {
    int* dc = (int*)ws.counters.p;
    const bool ratio = (flags & ASP_F_RATIO) != 0;
    const bool fuse_ratio = ratio && pl.n_wide == 0;
    const bool piped = pl.nch > 1;
    hipStream_t sd = piped ? ws.side : st;
    const size_t icap = item_cap(g), mcap = merge_cap(g);
    for (int c = 0; c < pl.nch; ++c) {
        const Chunk& ck = pl.ch[c];
        float4* recs = (float4*)ws.recs.p + ck.rec0 * NOUT;
        unsigned long long* slabs = (unsigned long long*)ws.slabs.p + (long long)ck.slab0 * NOUT * kTilePix;
        const Item* items = (const Item*)ws.items.p + c * icap;
        const Merge* merges = (const Merge*)ws.merges.p + c * mcap;
        int dflags = ((flags & ASP_F_ACCUMULATE) || c > 0 ? kFlagAccumulate : 0) |
                     (fuse_ratio && c == pl.nch - 1 ? kFlagRatio : 0);
        if (!(c == 0 && pre_scattered))
            ASP_TRY((launch_scatter<KID, NOUT, ACC>(g, ws, pl, c, u, v, h, a0, a1, 0x7fffffffLL,
                                                    0x7fffffff, st)));
        if (piped) {
            ASP_HIP(hipEventRecord(ws.chunk_ev[c], st));
            ASP_HIP(hipStreamWaitEvent(sd, ws.chunk_ev[c], 0));
        }
        if (ACC == kAccFix) {  // one chunk only (project2d)
            StageMark m(ws, kSScale, sd);
            hipLaunchKernelGGL((k_tilescale<NOUT>), dim3((g.ntiles + 63) / 64), dim3(kBlock), 0, sd,
                               (const unsigned*)ws.cmx.p, (int)pl.nblk_s, g.ntiles, g.nstream,
                               (const int*)ws.tile_total.p, (int2*)ws.tile_k.p);
            ASP_LAUNCHED();
            m.done();
        }
        {
            StageMark m(ws, kSDeposit, sd);
            size_t lds = (size_t)NOUT * kTilePix * 8 + 2 * kTile * 4;
            // ASP_GATHER=1: gathered large records (fp64 accumulation)
            const bool gather = getenv("ASP_GATHER") && atoi(getenv("ASP_GATHER")) == 1;
            if (ACC == kAccF64 && gather)
                hipLaunchKernelGGL((k_deposit<KID, NOUT, ACC, true>), dim3(ck.n_items), dim3(kDepThreads),
                                   lds + kGatherLds, sd, g, (const float4*)recs, items,
                                   (const int2*)ws.tile_k.p, slabs, o0, o1, dflags);
            else
                hipLaunchKernelGGL((k_deposit<KID, NOUT, ACC>), dim3(ck.n_items), dim3(kDepThreads), lds, sd, g,
                                   (const float4*)recs, items, (const int2*)ws.tile_k.p, slabs, o0, o1,
                                   dflags);
            ASP_LAUNCHED();
            m.done();
        }
        if (g.nstream == 2) {  // one chunk only (project2d)
            StageMark m(ws, kSBand, sd);
            hipLaunchKernelGGL((k_band<KID, NOUT, ACC>), dim3(ck.n_items, 2), dim3(kBlock), 0, sd, g,
                               (const float4*)recs, items, (const int2*)ws.tile_k.p, slabs, o0, o1,
                               dflags);
            ASP_LAUNCHED();
            m.done();
        }
        if (ck.n_merges > 0) {
            StageMark m(ws, kSMerge, sd);
            hipLaunchKernelGGL((k_merge<NOUT, ACC>), dim3(ck.n_merges, kTilePix / kBlock), dim3(kBlock), 0, sd, g,
                               merges, (const unsigned long long*)slabs, (const int2*)ws.tile_k.p,
                               o0, o1, dflags);
            ASP_LAUNCHED();
            m.done();
        }
    }
    if (pl.n_wide > 0) {
        StageMark m(ws, kSWide, sd);
        size_t lds = (size_t)NOUT * kTilePix * 8 + 2 * kTile * 4;
        hipLaunchKernelGGL((k_wide<KID, NOUT, ACC>), dim3(g.ntiles), dim3(kDepBlock), lds, sd, g, u, v, h,
                           a0, a1, (const int*)ws.wide.p, pl.n_wide, (const int*)dc, o0, o1);
        ASP_LAUNCHED();
        m.done();
    }
    if (ratio && !fuse_ratio) {
        long long npix = (long long)g.nx * g.ny;
        long long blocks = std::min<long long>((npix + kBlock - 1) / kBlock, 8192);
        StageMark m(ws, kSRatio, sd);
        hipLaunchKernelGGL(k_ratio, dim3((unsigned)std::max<long long>(1, blocks)), dim3(kBlock),
                           0, sd, o0, (const float*)o1, npix);
        ASP_LAUNCHED();
        m.done();
    }
    if (piped) {
        ASP_HIP(hipEventRecord(ws.done_ev, sd));
        ASP_HIP(hipStreamWaitEvent(st, ws.done_ev, 0));
    }
    return ASP_OK;
}

static int project2d(const float* u, const float* v, const float* h, const float* a0,
                     const float* a1, long long n, double x_min, double x_max, double y_min,
                     double y_max, int nx, int ny, int cs, int kid, int flags, float* out0,
                     float* out1, int device, void* stream) {
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (kid < 0 || kid > 2) return fail(ASP_ERR_INVALID, "unknown kernel_id");
    if (!out0) return fail(ASP_ERR_INVALID, "out0 is NULL");
    if ((a1 == nullptr) != (out1 == nullptr))
        return fail(ASP_ERR_INVALID, "a1 and out1 must both be given or both be NULL");
    if ((flags & ASP_F_RATIO) && !out1) return fail(ASP_ERR_INVALID, "ASP_F_RATIO needs out1");
    if ((flags & ASP_F_RATIO) && (flags & ASP_F_ACCUMULATE))
        return fail(ASP_ERR_INVALID, "ASP_F_RATIO cannot be combined with ASP_F_ACCUMULATE");
    if (n > 0 && (!u || !v || !h || !a0)) return fail(ASP_ERR_INVALID, "NULL particle array");
    if (n > 0x7fffffffLL) return fail(ASP_ERR_UNSUPPORTED, "n >= 2^31 particles per call");
    Grid g;
    if (!make_grid(x_min, x_max, y_min, y_max, nx, ny, cs, g))
        return fail(ASP_ERR_INVALID,
                    "invalid grid: need nx, ny, chunk_size >= 1, finite x_max > x_min, "
                    "y_max > y_min");
    // Row bands (K4b) are correct for any threshold but, as measured so far, slower than
    // the LDS-atomic sweep even for full-width boxes, so they are off by
    // default; ASP_BAND_COLS=c routes records spanning >= c tile columns to them.
    g.band_cols = (out1 != nullptr) ? kBandCols2 : kTile + 1;
    if (const char* e = getenv("ASP_BAND_COLS")) g.band_cols = std::max(1, atoi(e));
    g.nstream = g.band_cols <= kTile ? 2 : 1;  // a second record run per tile for K4b
    if (const char* e = getenv("ASP_WIDE_TILES")) g.wide_tiles = std::max(1, atoi(e));
    if (g.ntiles > kMaxTiles)
        return fail(ASP_ERR_UNSUPPORTED, "grid too large (more than 4096 64x64 tiles)");
    if (device < 0 || device >= 64) return fail(ASP_ERR_INVALID, "bad device");
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device >= ndev) return fail(ASP_ERR_INVALID, "device index out of range");
    ASP_HIP(hipSetDevice(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    const int nout = out1 ? 2 : 1;
    const bool dev = flags & ASP_F_DEVICE_PTRS;
    const long long npix = (long long)nx * ny;

    // stage host inputs
    const float* du = u;
    const float* dv = v;
    const float* dh = h;
    const float* da0 = a0;
    const float* da1 = a1;
    float* d0 = out0;
    float* d1 = out1;
    if (!dev) {
        const float* src[5] = {u, v, h, a0, a1};
        for (int k = 0; k < 4 + (nout == 2); ++k) {
            ASP_TRY(ensure(ws.in[k], (size_t)n * sizeof(float)));
            if (n > 0)
                ASP_HIP(hipMemcpyAsync(ws.in[k].p, src[k], (size_t)n * sizeof(float),
                                       hipMemcpyHostToDevice, st));
        }
        du = (const float*)ws.in[0].p;
        dv = (const float*)ws.in[1].p;
        dh = (const float*)ws.in[2].p;
        da0 = (const float*)ws.in[3].p;
        da1 = nout == 2 ? (const float*)ws.in[4].p : nullptr;
        for (int k = 0; k < nout; ++k) ASP_TRY(ensure(ws.out[k], (size_t)npix * sizeof(float)));
        d0 = (float*)ws.out[0].p;
        d1 = nout == 2 ? (float*)ws.out[1].p : nullptr;
        if (flags & ASP_F_ACCUMULATE) {
            ASP_HIP(hipMemcpyAsync(d0, out0, npix * sizeof(float), hipMemcpyHostToDevice, st));
            if (d1)
                ASP_HIP(hipMemcpyAsync(d1, out1, npix * sizeof(float), hipMemcpyHostToDevice, st));
        }
    }
    if (ws.prof) ASP_TRY(prof_next(ws));

    Plan pl{};
    pl.n = n;
    if (n == 0) {  // all-zero map(s)
        if (!(flags & ASP_F_ACCUMULATE)) {
            StageMark m(ws, kSMemset, st);
            ASP_HIP(hipMemsetAsync(d0, 0, npix * sizeof(float), st));
            if (d1) ASP_HIP(hipMemsetAsync(d1, 0, npix * sizeof(float), st));
            m.done();
        }
    } else {
        ASP_TRY(ensure_morton(ws, g.ntx, g.nty, st));
        long long max_blk = kMaxBinBlocks;
        if (const char* e = getenv("ASP_BIN_BLOCKS")) max_blk = std::max(1, atoi(e));
        pl.nblk = std::min<long long>(max_blk, std::max<long long>(1, (n + 8191) / 8192));
        pl.per_block = (n + pl.nblk - 1) / pl.nblk;
        pl.per_block = (pl.per_block + 3) / 4 * 4;  // vector loads: block bases stay 16-B aligned
        pl.nblk = (n + pl.per_block - 1) / pl.per_block;
        const bool det = (flags & ASP_F_DETERMINISTIC) != 0;
        // chunks: the fp64 path with one record run per tile; fixed point needs one
        // per-tile scale over all particles and the row bands one work list
        int nch = n >= kChunkMinParticles ? kChunks : 1;
        if (const char* e = getenv("ASP_CHUNKS")) nch = atoi(e);
        if (det || g.nstream != 1) nch = 1;
        nch = (int)std::max<long long>(1, std::min<long long>({(long long)nch, (long long)kMarks, pl.nblk}));
        pl.grp = std::max(1, kScatterGroup / nch);
        pl.cb = (pl.nblk + nch - 1) / nch;
        pl.cb = (pl.cb + pl.grp - 1) / pl.grp * pl.grp;
        pl.nch = (int)((pl.nblk + pl.cb - 1) / pl.cb);
        pl.nblk_s = 0;
        for (int c = 0; c < pl.nch; ++c) {
            long long b0 = c * pl.cb, b1 = std::min(pl.nblk, b0 + pl.cb);
            pl.ch[c].blk0 = b0 / pl.grp;
            pl.ch[c].nblk_s = (b1 - b0 + pl.grp - 1) / pl.grp;
            pl.nblk_s += pl.ch[c].nblk_s;
        }
        if (pl.nch > 1) ASP_TRY(ensure_side(ws));
        ASP_TRY(ensure(ws.hist, (size_t)pl.nblk * g.nstream * g.ntiles * sizeof(int)));
        if (det) ASP_TRY(ensure(ws.cmx, (size_t)pl.nblk_s * g.ntiles * nout * sizeof(unsigned)));
        ASP_TRY(ensure(ws.tile_total, (size_t)pl.nch * 2 * g.ntiles * sizeof(int)));
        ASP_TRY(ensure(ws.tile_start, (size_t)pl.nch * 2 * g.ntiles * sizeof(long long)));
        ASP_TRY(ensure(ws.tile_k, (size_t)g.ntiles * sizeof(int2)));
        ASP_TRY(ensure(ws.items, (size_t)pl.nch * item_cap(g) * sizeof(Item)));
        ASP_TRY(ensure(ws.merges, (size_t)pl.nch * merge_cap(g) * sizeof(Merge)));
        ASP_TRY(ensure(ws.counters, (size_t)kMarks * cNum * sizeof(int)));
        if (!ws.h_counters) ASP_HIP(hipHostMalloc((void**)&ws.h_counters, kMarks * cNum * sizeof(int)));
        int* dc = (int*)ws.counters.p;
        ASP_HIP(hipMemsetAsync(dc, 0, (size_t)pl.nch * cNum * sizeof(int), st));
        {
            StageMark m(ws, kSCount, st);
            hipLaunchKernelGGL(k_count, dim3((unsigned)pl.nblk), dim3(kCountBlock),
                               (size_t)g.nstream * g.ntiles * sizeof(int), st, du, dv, dh, n,
                               ASP_INTERLEAVE ? pl.nblk : pl.per_block, g,
                               (int*)ws.hist.p, dc);
            ASP_LAUNCHED();
            m.done();
        }
        {
            StageMark m(ws, kSColscan, st);
            hipLaunchKernelGGL(k_colscan, dim3((g.nstream * g.ntiles + 63) / 64, pl.nch), dim3(kColscanBlock),
                               0, st, (int*)ws.hist.p, (int)pl.nblk, g.nstream * g.ntiles,
                               (int*)ws.tile_total.p, (int)pl.cb);
            ASP_LAUNCHED();
            m.done();
        }
        for (int c = 0; c < pl.nch; ++c) {
            StageMark m(ws, kSTilescan, st);
            hipLaunchKernelGGL(k_tilescan<4>, dim3(1), dim3(kScanThreads), 0, st,
                               (const int*)ws.tile_total.p + (long long)c * g.nstream * g.ntiles,
                               (const int*)ws.morton.p, g.ntiles, g.nstream,
                               (long long*)ws.tile_start.p + (long long)c * 2 * g.ntiles,
                               (Item*)ws.items.p + c * item_cap(g),
                               (Merge*)ws.merges.p + c * merge_cap(g), dc + c * cNum);
            ASP_LAUNCHED();
            m.done();
        }
        // One small read-back sizes the record / slab buffers.  With buffers
        // left by an earlier call, the scatter is enqueued BEFORE the host waits for it
        // (speculatively: it checks the counters against those capacities itself), so the
        // GPU does not idle across the host round trip.
        // The copy runs on the side stream, so the scatter behind it on st need not wait
        // for the copy's own latency.
        ASP_TRY(ensure_side(ws));
        ASP_HIP(hipEventRecord(ws.scan_ev, st));
        ASP_HIP(hipStreamWaitEvent(ws.side, ws.scan_ev, 0));
        ASP_HIP(hipMemcpyAsync(ws.h_counters, dc, (size_t)pl.nch * cNum * sizeof(int),
                               hipMemcpyDeviceToHost, ws.side));
        ASP_HIP(hipEventRecord(ws.cnt_ev, ws.side));
        const long long rec_cap = (long long)std::min<size_t>(ws.recs.cap / (nout * sizeof(float4)), 0x7fffffff);
        const int wide_cap = (int)std::min<size_t>(ws.wide.cap / sizeof(int), 0x7fffffff);
        const bool spec = pl.nch == 1 && ws.recs.p && ws.wide.p && getenv("ASP_NO_SPECULATE") == nullptr;
        if (spec) {
            pl.ch[0].rec0 = 0;
#define ASP_SC(K, N, A) \
    launch_scatter<K, N, A>(g, ws, pl, 0, du, dv, dh, da0, da1, rec_cap, wide_cap, st)
#define ASP_SC2(K, A) (nout == 1 ? ASP_SC(K, 1, A) : ASP_SC(K, 2, A))
#define ASP_SC3(A) (kid == 0 ? ASP_SC2(0, A) : kid == 1 ? ASP_SC2(1, A) : ASP_SC2(2, A))
            ASP_TRY(det ? ASP_SC3(kAccFix) : ASP_SC3(kAccF64));
#undef ASP_SC3
#undef ASP_SC2
#undef ASP_SC
        }
        ASP_HIP(hipEventSynchronize(ws.cnt_ev));
        pl.n_items = pl.n_slabs = pl.n_merges = 0;
        pl.n_recs = 0;
        for (int c = 0; c < pl.nch; ++c) {
            const int* hc = ws.h_counters + c * cNum;
            Chunk& ck = pl.ch[c];
            ck.rec0 = pl.n_recs;
            ck.n_recs = hc[cRecs];
            ck.n_items = hc[cItems];
            ck.n_merges = hc[cMerges];
            ck.n_slabs = hc[cSlabs];
            ck.slab0 = pl.n_slabs;
            if (ck.n_recs >= 0x7fffffffLL)
                return fail(ASP_ERR_UNSUPPORTED, "more than 2^31 particle-tile records");
            pl.n_recs += ck.n_recs;
            pl.n_items += ck.n_items;
            pl.n_slabs += ck.n_slabs;
            pl.n_merges += ck.n_merges;
        }
        pl.n_wide = ws.h_counters[cWideCount];
        if (pl.n_recs >= 0x7fffffffLL)
            return fail(ASP_ERR_UNSUPPORTED, "more than 2^31 particle-tile records");
        const bool pre = spec && pl.n_recs <= rec_cap && pl.n_wide <= wide_cap;
        if (spec && !pre) ASP_HIP(hipStreamSynchronize(st));  // its (no-op) scatter is done
        ASP_TRY(ensure(ws.recs, (size_t)pl.n_recs * nout * sizeof(float4)));
        ASP_TRY(ensure(ws.wide, (size_t)pl.n_wide * sizeof(int)));
        ASP_TRY(ensure(ws.slabs, (size_t)pl.n_slabs * nout * kTilePix * sizeof(long long)));
        int rc;
#define ASP_TAIL(K, N, A) \
    run_tail<K, N, A>(g, ws, pl, du, dv, dh, da0, da1, d0, d1, flags, st, pre)
#define ASP_TAIL2(K, A) (nout == 1 ? ASP_TAIL(K, 1, A) : ASP_TAIL(K, 2, A))
#define ASP_TAIL3(A) (kid == 0 ? ASP_TAIL2(0, A) : kid == 1 ? ASP_TAIL2(1, A) : ASP_TAIL2(2, A))
        rc = det ? ASP_TAIL3(kAccFix) : ASP_TAIL3(kAccF64);
#undef ASP_TAIL3
#undef ASP_TAIL2
#undef ASP_TAIL
        if (rc != ASP_OK) return rc;
    }
    if (n == 0 && (flags & ASP_F_RATIO)) {
        // 0 / 0 -> 0: the memset already wrote the ratio map
    }
    if (!dev) {
        ASP_HIP(hipMemcpyAsync(out0, d0, npix * sizeof(float), hipMemcpyDeviceToHost, st));
        if (out1)
            ASP_HIP(hipMemcpyAsync(out1, d1, npix * sizeof(float), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    ws.stats[0] = pl.n_recs;
    ws.stats[1] = pl.n_items;
    ws.stats[2] = pl.n_wide;
    ws.stats[3] = kTile;
    ws.stats[4] = g.ntiles;
    ws.stats[5] = n > 0 ? ws.h_counters[cChunk] : 0;
    ws.stats[6] = pl.n_merges;
    ws.stats[7] = pl.n_slabs;
    ws.stats[8] = n > 0 ? pl.nch : 0;
    return ASP_OK;
}

}  // namespace asp

// ==================================================================================
// C-ABI
// ==================================================================================
using namespace asp;

extern "C" {

int asp_version(void) { return ASP_API_VERSION * 10000 + 1; }

const char* asp_last_error(void) { return t_err.c_str(); }

int asp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int asp_project2d(const float* u, const float* v, const float* h, const float* a0,
                  const float* a1, int64_t n, double u_min, double u_max, double v_min,
                  double v_max, int32_t nx, int32_t ny, int32_t chunk_size, int32_t kernel_id,
                  int32_t flags, float* out0, float* out1, int32_t device, void* stream) {
    t_err.clear();
    return project2d(u, v, h, a0, a1, n, u_min, u_max, v_min, v_max, nx, ny, chunk_size,
                     kernel_id, flags, out0, out1, device, stream);
}

int asp_kernel_eval(int32_t kernel_id, const double* r, const double* h, double* w, int64_t n,
                    int32_t flags, int32_t device, void* stream) {
    t_err.clear();
    if (kernel_id < 0 || kernel_id > 2) return fail(ASP_ERR_INVALID, "unknown kernel_id");
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (n == 0) return ASP_OK;
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    const double *dr = r, *dh = h;
    double* dw = w;
    bool dev = flags & ASP_F_DEVICE_PTRS;
    if (!dev) {
        ASP_TRY(ensure(ws.aux[0], n * sizeof(double)));
        ASP_TRY(ensure(ws.aux[1], n * sizeof(double)));
        ASP_TRY(ensure(ws.aux[2], n * sizeof(double)));
        ASP_HIP(hipMemcpyAsync(ws.aux[0].p, r, n * sizeof(double), hipMemcpyHostToDevice, st));
        ASP_HIP(hipMemcpyAsync(ws.aux[1].p, h, n * sizeof(double), hipMemcpyHostToDevice, st));
        dr = (const double*)ws.aux[0].p;
        dh = (const double*)ws.aux[1].p;
        dw = (double*)ws.aux[2].p;
    }
    hipLaunchKernelGGL(k_kernel_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (int)kernel_id, dr, dh, dw, (long long)n);
    ASP_HIP(hipGetLastError());
    if (!dev) {
        ASP_HIP(hipMemcpyAsync(w, dw, n * sizeof(double), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    return ASP_OK;
}

int asp_chunk_ranges(const float* u, const float* v, const float* h, int64_t n, double u_min,
                     double u_max, double v_min, double v_max, int32_t nx, int32_t ny,
                     int32_t chunk_size, int32_t* cx0, int32_t* cx1, int32_t* cy0, int32_t* cy1,
                     int32_t flags, int32_t device, void* stream) {
    t_err.clear();
    Grid g;
    if (!make_grid(u_min, u_max, v_min, v_max, nx, ny, chunk_size, g))
        return fail(ASP_ERR_INVALID, "invalid grid");
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (n == 0) return ASP_OK;
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    bool dev = flags & ASP_F_DEVICE_PTRS;
    const float *du = u, *dv = v, *dh = h;
    int* o[4] = {cx0, cx1, cy0, cy1};
    if (!dev) {
        const float* src[3] = {u, v, h};
        for (int k = 0; k < 3; ++k) {
            ASP_TRY(ensure(ws.in[k], n * sizeof(float)));
            ASP_HIP(hipMemcpyAsync(ws.in[k].p, src[k], n * sizeof(float), hipMemcpyHostToDevice,
                                   st));
        }
        du = (const float*)ws.in[0].p;
        dv = (const float*)ws.in[1].p;
        dh = (const float*)ws.in[2].p;
        for (int k = 0; k < 4; ++k) {
            ASP_TRY(ensure(ws.aux[k], n * sizeof(int)));
            o[k] = (int*)ws.aux[k].p;
        }
    }
    hipLaunchKernelGGL(k_chunk_ranges, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g,
                       du, dv, dh, (long long)n, o[0], o[1], o[2], o[3]);
    ASP_HIP(hipGetLastError());
    if (!dev) {
        int* dst[4] = {cx0, cx1, cy0, cy1};
        for (int k = 0; k < 4; ++k)
            ASP_HIP(hipMemcpyAsync(dst[k], o[k], n * sizeof(int), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    return ASP_OK;
}

int asp_pixel_neighbours(const float* u, const float* v, const float* h, int64_t n,
                         double u_min, double u_max, double v_min, double v_max, int32_t nx,
                         int32_t ny, int32_t chunk_size, const int64_t* pixels, int64_t npix,
                         int64_t* offsets, int32_t* index, int64_t cap, int64_t* total,
                         int32_t device) {
    t_err.clear();
    Grid g;
    if (!make_grid(u_min, u_max, v_min, v_max, nx, ny, chunk_size, g))
        return fail(ASP_ERR_INVALID, "invalid grid");
    if (n < 0 || npix < 0 || cap < 0) return fail(ASP_ERR_INVALID, "negative size");
    for (int64_t k = 0; k < npix; ++k)
        if (pixels[k] < 0 || pixels[k] >= (int64_t)nx * ny)
            return fail(ASP_ERR_INVALID, "pixel id out of range");
    offsets[0] = 0;
    if (total) *total = 0;
    if (npix == 0) return ASP_OK;
    if (n == 0) {
        for (int64_t k = 0; k < npix; ++k) offsets[k + 1] = 0;
        return ASP_OK;
    }
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = nullptr;
    const float* src[3] = {u, v, h};
    for (int k = 0; k < 3; ++k) {
        ASP_TRY(ensure(ws.in[k], n * sizeof(float)));
        ASP_HIP(hipMemcpyAsync(ws.in[k].p, src[k], n * sizeof(float), hipMemcpyHostToDevice, st));
    }
    ASP_TRY(ensure(ws.aux[0], npix * sizeof(long long)));
    ASP_TRY(ensure(ws.aux[1], npix * sizeof(long long)));
    ASP_TRY(ensure(ws.aux[2], (npix + 1) * sizeof(long long)));
    ASP_HIP(hipMemcpyAsync(ws.aux[0].p, pixels, npix * sizeof(long long), hipMemcpyHostToDevice,
                           st));
    hipLaunchKernelGGL(k_neighbours, dim3((unsigned)npix), dim3(kBlock), 0, st, g,
                       (const float*)ws.in[0].p, (const float*)ws.in[1].p,
                       (const float*)ws.in[2].p, (long long)n, (const long long*)ws.aux[0].p,
                       (long long*)ws.aux[1].p, (const long long*)nullptr, (int*)nullptr, 0LL, 0);
    ASP_HIP(hipGetLastError());
    std::vector<long long> cnt(npix);
    ASP_HIP(hipMemcpyAsync(cnt.data(), ws.aux[1].p, npix * sizeof(long long),
                           hipMemcpyDeviceToHost, st));
    ASP_HIP(hipStreamSynchronize(st));
    for (int64_t k = 0; k < npix; ++k) offsets[k + 1] = offsets[k] + cnt[k];
    long long tot = offsets[npix];
    if (total) *total = tot;
    long long wcap = std::min<long long>(cap, tot);
    if (wcap > 0) {
        ASP_TRY(ensure(ws.aux[3], wcap * sizeof(int)));
        ASP_HIP(hipMemcpyAsync(ws.aux[2].p, offsets, npix * sizeof(long long),
                               hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_neighbours, dim3((unsigned)npix), dim3(kBlock), 0, st, g,
                           (const float*)ws.in[0].p, (const float*)ws.in[1].p,
                           (const float*)ws.in[2].p, (long long)n, (const long long*)ws.aux[0].p,
                           (long long*)ws.aux[1].p, (const long long*)ws.aux[2].p,
                           (int*)ws.aux[3].p, wcap, 1);
        ASP_HIP(hipGetLastError());
        ASP_HIP(hipMemcpyAsync(index, ws.aux[3].p, wcap * sizeof(int), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    return ASP_OK;
}

int asp_ratio(float* out0, const float* out1, int64_t n, int32_t device, void* stream) {
    t_err.clear();
    if (n < 0 || !out0 || !out1) return fail(ASP_ERR_INVALID, "bad argument");
    if (n == 0) return ASP_OK;
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    long long blocks = std::min<long long>((n + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_ratio, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       out0, out1, (long long)n);
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}

int asp_profile_stages(int32_t device, uint32_t stage_mask) {
    t_err.clear();
    int ndev = asp_device_count();
    if (device < 0 || device >= ndev) return fail(ASP_ERR_INVALID, "bad device");
    ASP_HIP(hipSetDevice(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    if (stage_mask && !ws.ev[0][0][0][0])
        for (int q = 0; q < 2; ++q)
            for (int k = 0; k < kStages; ++k)
                for (int j = 0; j < kMarks; ++j)
                    for (int e = 0; e < 2; ++e) ASP_HIP(hipEventCreate(&ws.ev[q][k][j][e]));
    for (int k = 0; k < kStages; ++k) {
        ws.stage_ms[k] = 0.0;
        ws.stage_n[k] = 0;
        ws.ev_live[0][k] = ws.ev_live[1][k] = 0;
    }
    ws.prof = stage_mask != 0u;
    ws.prof_mask = stage_mask;
    return ASP_OK;
}

int asp_profile(int32_t device, int32_t enable) {
    return asp_profile_stages(device, enable ? 0xffffffffu : 0u);
}

int asp_profile_read(int32_t device, double* ms_sum, int64_t* launches, int32_t nstages) {
    t_err.clear();
    if (device < 0 || device >= 64 || !ms_sum || !launches)
        return fail(ASP_ERR_INVALID, "bad argument");
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    if (ws.prof) {
        ASP_HIP(hipSetDevice(device));
        ASP_TRY(prof_fold(ws));
    }
    for (int k = 0; k < nstages; ++k) {
        ms_sum[k] = k < kStages ? ws.stage_ms[k] : 0.0;
        launches[k] = k < kStages ? ws.stage_n[k] : 0;
    }
    return ASP_OK;
}

int asp_last_stats(int32_t device, int64_t* stats, int32_t nstats) {
    if (device < 0 || device >= 64 || !stats) return fail(ASP_ERR_INVALID, "bad argument");
    for (int k = 0; k < nstats && k < 9; ++k) stats[k] = g_ws[device].stats[k];
    return ASP_OK;
}

int asp_release(int32_t device) {
    int lo = device < 0 ? 0 : device, hi = device < 0 ? 63 : device;
    int ndev = asp_device_count();
    for (int d = lo; d <= hi && d < ndev; ++d) {
        Workspace& ws = g_ws[d];
        std::lock_guard<std::mutex> lock(ws.mu);
        if (hipSetDevice(d) != hipSuccess) continue;
        Buf* all[] = {&ws.in[0], &ws.in[1], &ws.in[2], &ws.in[3], &ws.in[4], &ws.out[0],
                      &ws.out[1], &ws.hist, &ws.cmx, &ws.tile_total, &ws.tile_start,
                      &ws.tile_k, &ws.items, &ws.merges, &ws.counters, &ws.recs, &ws.wide,
                      &ws.slabs, &ws.morton, &ws.morton3, &ws.aux[0], &ws.aux[1], &ws.aux[2], &ws.aux[3],
                      &ws.aux[4], &ws.aux[5]};
        for (Buf* b : all) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
        if (ws.h_counters) (void)hipHostFree(ws.h_counters);
        ws.h_counters = nullptr;
        ws.morton_ntx = ws.morton_nty = -1;
        ws.morton3_key[0] = ws.morton3_key[1] = ws.morton3_key[2] = -1;
    }
    return ASP_OK;
}

}  // extern "C"
