// asp_project2d.hip -- MI355X (gfx950) SPH particle -> pixel-grid projection.
//
// Replaces the reference's create_image / process_chunk / calculate_pixel_value /
// quartic_spline_kernel path (/root/reference/src/astro_sph_tools/tools/projections/
// _projector.py:13-120, _pixel_calculations.pyx:9-36, _kernels.pyx:9-20) with a
// scatter formulation built for CDNA4:
//
//   K1 count     one streaming pass over (u, v, h): per-workgroup LDS histogram of
//                (particle, GPU tile) insertions -> hist[block][tile], two streams per
//                tile: records whose box clipped to the tile is small / mid-size, and
//                LARGE ones (>= gather_min pixels on both axes, or >= gather_area pixels)
//   K2a colscan  per tile, exclusive prefix over blocks (in place) + tile totals
//   K2b tilescan one workgroup: tile start offsets in Morton order of the tiles, the
//                deposit work list (runs of <= CH records of one tile; empty tiles get
//                a zero item) and the merge list of tiles split over several items
//   K3 scatter   second streaming pass: each insertion written as a 32-byte PREPARED
//                record into its tile's run of its stream (LDS cursors)
//   K3b scale    (deterministic mode) per tile: power-of-two fixed-point scale
//   K4 deposit   one workgroup per work item of the small/mid stream: records -> LDS tile
//                accumulators; boxes of <= 4 x 4 pixels lane-per-record, mid-size boxes
//                swept by a whole wave (LDS atomics); the tile is written once, or (split
//                tiles) stored as a partial slab
//   K4g gather   the large stream: one single-wave workgroup per (work item, 16 x 32
//                region of the tile); the wave streams the item's records into per-lane
//                entries, walks those meeting its region with v_readlane (fields in
//                SGPRs), each lane summing one pixel of each 8 x 8 block in registers
//                (packed fp32, no per-pair atomics); tile or slab written from registers
//   K5 merge     split tiles: sum of their slabs in slab order, write
//   K6 wide      particles overlapping > wide_tiles tiles, per tile region, gathered
//   K7 ratio     out0 / out1 (mass-weighted maps) when not fused into K4/K5
//   K8 pairs     the kernel_func plug-in: every included (pixel, particle, r^2) pair
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

constexpr int kCountBlock = 256;   // count workgroup
#ifndef ASP_COUNT_UNROLL
#define ASP_COUNT_UNROLL 4
#endif
constexpr int kCountUnroll = ASP_COUNT_UNROLL;  // particles per lane and batch in count
// Scatter workgroup and how many consecutive count workgroups' particles it takes over:
// fewer, wider scatter workgroups keep fewer partially written record lines open at a
// time (each workgroup appends to its own segment of every tile).
#ifndef ASP_SCATTER_BLOCK
#define ASP_SCATTER_BLOCK 512
#endif
#ifndef ASP_SCATTER_GROUP_DEF
#define ASP_SCATTER_GROUP_DEF 4
#endif
constexpr int kScatterBlock = ASP_SCATTER_BLOCK;
constexpr int kScatterGroup = ASP_SCATTER_GROUP_DEF;
constexpr int kUnroll = (int)(kCountBlock * kCountUnroll / kScatterBlock);  // particles per lane and batch in scatter
// Particles per loop iteration of a count / scatter workgroup (a "batch").  Batches are
// dealt to the count workgroups round-robin (batch j to workgroup j % nblk; the scatter
// workgroup of count workgroups sb*grp.. takes their batches in order), so at any moment
// the whole grid streams one window of the particle arrays.
constexpr long long kBatch = (long long)kCountBlock * kCountUnroll;
static_assert(kBatch == (long long)kScatterBlock * kUnroll, "count and scatter batches differ");

// Records whose box clipped to a tile is at least this wide on both axes go to the large
// stream (K4g); the threshold is a Grid field so it can be tuned per call
// (ASP_GATHER_MIN).
constexpr int kGatherMinDefault = 5;
// ... or at least this many pixels: the thin slivers of large discs clipped at tile edges,
// which K4 sweeps a whole wave per record (ASP_GATHER_AREA): cfg 2 at
// physical h 11.42-11.49 -> 11.10 ms (12-20 alike), the pixel-scale map unchanged at 20
// (16 sends its 4 x 4 boxes to K4g: 3.25 -> 3.32 ms)
constexpr int kGatherAreaDefault = 20;

// Vector of U floats (one 4 U-byte load per lane).
template <int U>
using vecf = float __attribute__((ext_vector_type(U)));

// Load U CONSECUTIVE particles per lane with one U-wide load per array when the arrays
// are 4 U-byte aligned (`al`); h = 0 past the end, which has no footprint.
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

template <int U>
__device__ __forceinline__ void load_batch(const float* __restrict__ u, const float* __restrict__ v,
                                           const float* __restrict__ h, long long base,
                                           long long p1, bool al, float* pu, float* pv,
                                           float* ph) {
    long long p = base + (long long)threadIdx.x * U;
    load_vec<U>(u, p, p1, al, pu);
    load_vec<U>(v, p, p1, al, pv);
    load_vec<U>(h, p, p1, al, ph);
}

// A record's candidate box clipped to tile (tx, ty), tile-local, one byte per bound:
// x0 | x1 << 8 | y0 << 16 | y1 << 24.
__device__ __forceinline__ unsigned tile_box(const Box& b, int tx, int ty) {
    int X0 = tx * kTile, Y0 = ty * kTile;
    unsigned x0 = max(b.x0, X0) - X0, x1 = min(b.x1, X0 + kTile - 1) - X0;
    unsigned y0 = max(b.y0, Y0) - Y0, y1 = min(b.y1, Y0 + kTile - 1) - Y0;
    return x0 | (x1 << 8) | (y0 << 16) | (y1 << 24);
}

__device__ __forceinline__ bool box_large(unsigned bp, const Grid& g) {
    int bw = (int)((bp >> 8) & 255u) - (int)(bp & 255u) + 1;
    int bh = (int)(bp >> 24) - (int)((bp >> 16) & 255u) + 1;
    return (bw >= g.gather_min && bh >= g.gather_min) || bw * bh >= g.gather_area;
}

// Histogram column of a (particle, tile) insertion: t (small / mid-size stream) or
// t + ntiles (large stream, gathered by K4g).  `maybe`: the unclipped box is large.
__device__ __forceinline__ int column(const Grid& g, const Box& b, bool maybe, int tx, int ty) {
    const int t = tx * g.nty + ty;
    return maybe && box_large(tile_box(b, tx, ty), g) ? t + g.ntiles : t;
}
__device__ __forceinline__ bool maybe_large(const Grid& g, const Box& b) {
    const int bw = b.x1 - b.x0 + 1, bh = b.y1 - b.y0 + 1;  // unclipped: an upper bound
    return (bw >= g.gather_min && bh >= g.gather_min) || (long long)bw * bh >= g.gather_area;
}

// ----------------------------------------------------------------------------------
// K1: count insertions per (block, tile)
// ----------------------------------------------------------------------------------
template <bool CULL>
__global__ __launch_bounds__(kCountBlock) void k_count(const float* __restrict__ u,
                                                       const float* __restrict__ v,
                                                       const float* __restrict__ h,
                                                       long long n, long long nblk, Grid g,
                                                       Src64 s, int* __restrict__ hist,
                                                       int* __restrict__ ctr) {
    extern __shared__ __attribute__((aligned(16))) int lh[];  // 2 * ntiles columns
    for (int t = threadIdx.x; t < 2 * g.ntiles; t += kCountBlock) lh[t] = 0;
    __syncthreads();
    int nwide = 0;
    const long long p0 = (long long)blockIdx.x * kBatch, stride = nblk * kBatch;
    // Software pipeline: the next batch's loads are in flight while this batch is binned.
    float pu[kCountUnroll], pv[kCountUnroll], ph[kCountUnroll];
    const bool al = aligned_vec<kCountUnroll>(u, v, h);
    load_batch<kCountUnroll>(u, v, h, p0, n, al, pu, pv, ph);
    for (long long base = p0; base < n; base += stride) {
        float nu[kCountUnroll], nv[kCountUnroll], nh[kCountUnroll];
        load_batch<kCountUnroll>(u, v, h, base + stride, n, al, nu, nv, nh);
#pragma unroll
        for (int k = 0; k < kCountUnroll; ++k) {
            Box b;
            const int p = (int)(base + (long long)threadIdx.x * kCountUnroll + k);
            if (!footprint<CULL>(g, s, p, pu[k], pv[k], ph[k], b)) continue;
            int tx0 = b.x0 >> kTileShift, tx1 = b.x1 >> kTileShift;
            int ty0 = b.y0 >> kTileShift, ty1 = b.y1 >> kTileShift;
            if ((tx1 - tx0 + 1) * (ty1 - ty0 + 1) > g.wide_tiles) {
                ++nwide;
                continue;
            }
            const bool mb = maybe_large(g, b);
            if (tx1 - tx0 <= 1 && ty1 - ty0 <= 1) {
                // at most 2 x 2 tiles (every pixel-scale particle): straight-line, so a wave
                // pays for the second column / row only when one of its lanes needs it
                atomicAdd(&lh[column(g, b, mb, tx0, ty0)], 1);
                if (tx1 > tx0) atomicAdd(&lh[column(g, b, mb, tx1, ty0)], 1);
                if (ty1 > ty0) {
                    atomicAdd(&lh[column(g, b, mb, tx0, ty1)], 1);
                    if (tx1 > tx0) atomicAdd(&lh[column(g, b, mb, tx1, ty1)], 1);
                }
            } else {
                for (int tx = tx0; tx <= tx1; ++tx)
                    for (int ty = ty0; ty <= ty1; ++ty) atomicAdd(&lh[column(g, b, mb, tx, ty)], 1);
            }
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
    int* row = hist + (long long)blockIdx.x * 2 * g.ntiles;
    for (int t = threadIdx.x; t < 2 * g.ntiles; t += kCountBlock) row[t] = lh[t];
}

// Record stores of the scatter: plain stores (non-temporal ones measured 2x slower, the
// L2 merges the 32-B halves of a line).
// ASP_SCATTER_ABLATE (experiment builds only, never the default): 1 -- the record stores
// become a store under a condition no record meets (the records are still formed), 2 -- as
// 1 and the cursor claims become a plain index (no LDS atomics).  The deposit kernels then
// return at once (the record buffer holds no records).  DESIGN.md §4, round 6.
#ifndef ASP_SCATTER_ABLATE
#define ASP_SCATTER_ABLATE 0
#endif
// batches of particle loads the scatter keeps in flight ahead of the one it bins (1, or 2
// as an A/B build switch)
#ifndef ASP_SCATTER_PREFETCH
#define ASP_SCATTER_PREFETCH 1
#endif
__device__ __forceinline__ void rec_store(float4* dst, float4 v) {
    // one global_store_dwordx4 per half record: the empty asm keeps the vectorizer from
    // regrouping two halves as dwordx3 + unaligned dwordx4 + dword
#if ASP_SCATTER_ABLATE
    if (v.x == 1.25e-37f && v.y == -1.25e-37f) *dst = v;
#else
    *dst = v;
#endif
    asm volatile("" ::: "memory");
}

template <int NOUT>
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
// The PREPARED record (32 B, both map counts): {u, v, h, c0}, {c1, p, band, box} --
// c = a * norm(h) the fp32 term coefficients, p the particle index (the fp64 re-decision
// reads the caller's arrays there), band the error band of §3, box the candidate box
// clipped to the tile (4 tile-local bytes).  The deposit's per-record set-up is done
// here, where the store-bound scatter has VALU to spare.  Also the per-(block, tile) max
// |c| (fp32 bits) of the records it inserted, the fixed-point bound of K3b.
// ----------------------------------------------------------------------------------
// SRC: where the record frame's exact coordinates come from -- 0: the fp32 arrays (fp32
// callers), 1: the resident fp64 arrays, loaded with the batch (s.u64 != null), 2: decided
// per particle (src_u: the chunk-cull kernels).  0 and 1 keep loads out of the per-particle
// branches (the fp32 kernels carry no fp64 load path at all).
// PROBE: 1 for the placement trials' launches (the same code under its own name, so that
// profiles of the steady state show them apart).
// Properties 2..5 of asp_project2d_props (NX = 1): their arrays (unused ones repeat
// a[0]) and the per-record coefficient array ext (float4 {c2, c3, c4, c5} at the record's
// slot), written beside the records so every further pair of maps deposits from the SAME
// binning.
struct XArgs {
    const float* a[4];
    float4* ext;
};

// Per-wave staging of the paired record stores: first halves at [lane], second halves at
// [72 + lane] (8 float4 apart: neither the b128 writes nor the b128 reads conflict).
constexpr int kStageF4 = 136;

template <int KID, int NOUT, int ACC, bool CULL, int SRC, int PROBE, int NX = 0>
__global__ __launch_bounds__(kScatterBlock) void k_scatter(
    const float* __restrict__ u, const float* __restrict__ v, const float* __restrict__ h,
    const float* __restrict__ a0, const float* __restrict__ a1, long long n, long long nblk,
    Grid g, Src64 s, const int* __restrict__ hist, const long long* __restrict__ tile_start,
    const int* __restrict__ tile_total, float4* __restrict__ recs, unsigned* __restrict__ cmx,
    int* __restrict__ wide_list, int* __restrict__ ctr, int grp, long long rec_cap,
    int wide_cap, XArgs xa) {
    // Speculative launch (enqueued before the host has read the counters): the record and
    // wide-list buffers were sized by an earlier call; if this call needs more, every
    // workgroup leaves at once and the host relaunches after growing them.
    if (ctr[cRecs] > rec_cap || ctr[cWideCount] > wide_cap) return;
    // absolute record cursors: the small / mid-size stream, then the large one
    extern __shared__ __attribute__((aligned(16))) int cur[];
    // per-wave staging for the paired record stores: 64 records x 32 B (second halves
    // 8 float4 further on, so neither the b128 writes nor the b128 reads conflict)
    float4* stage = (float4*)(cur + 2 * g.ntiles);
    unsigned* cm = (unsigned*)(stage + (kScatterBlock / 64) * kStageF4);
    // this workgroup takes over count workgroups grp * sb ..: its cursors start at the
    // prefix row of the first of them
    const long long sb = blockIdx.x;
    const int* row = hist + sb * grp * 2 * g.ntiles;
    for (int t = threadIdx.x; t < 2 * g.ntiles; t += kScatterBlock)
        cur[t] = (int)tile_start[t] + row[t];  // n_recs < 2^31 (checked on the host)
    if constexpr (ACC == kAccFix)
        for (int t = threadIdx.x; t < g.ntiles * NOUT; t += kScatterBlock) cm[t] = 0u;
    __syncthreads();
    // the batches of count workgroups sb * grp .. (< nblk), in order: batch q * nblk +
    // sb * grp + r for r < gcnt, q = 0, 1, ...  The loop steps (q, r) and carries the batch's
    // first particle index c: a division by gcnt per batch made the compiler emit two
    // 64-bit divisions per iteration (SALU was 147 instructions per wave and iteration,
    // round 6).  One batch per iteration: 2 and 4 batches measured slower (1.794 / 1.918 vs
    // 1.756 ms, round 5, DESIGN_LOG.md §18) -- the scatter is bound by its stores, not by
    // load latency.  Lane particle k of the batch at c: c + k * kScatterBlock + threadIdx.x
    // (coalesced dword loads).  Every load is unconditional -- index clamped to the last
    // particle, h = 0 past the end (no footprint) -- so the compiler can count the loads in
    // flight: with load_vec's vector-or-scalar branches it put s_waitcnt vmcnt(0) right after
    // issuing the NEXT batch's loads.
    const long long gcnt = min((long long)grp, nblk - sb * grp);
    auto base_of = [&](long long q, long long r) { return (q * nblk + sb * grp + r) * kBatch; };
    constexpr int kLane = kUnroll;
    auto pidx = [&](long long b, int k) {
        return b + (long long)k * kScatterBlock + threadIdx.x;
    };
    auto ld = [&](const float* __restrict__ a, long long c, float* out) {
#pragma unroll
        for (int k = 0; k < kLane; ++k) out[k] = a[min(pidx(c, k), n - 1)];
    };
    // Software pipeline: issue the next iteration's loads BEFORE this one's record stores.
    float pu[kLane], pv[kLane], ph[kLane], pa0[kLane], pa1[kLane];
    double pU[kLane], pV[kLane];  // SRC 1: the exact coordinates
    // SRC 1: the fp64 coordinates of the lane's particles (index clamped to the array:
    // unconditional loads; lanes past the end are never binned)
    auto load_src = [&](long long c, double* dU, double* dV) {
        if constexpr (SRC == 1) {
#pragma unroll
            for (int k = 0; k < kLane; ++k) {
                const long long q = min(pidx(c, k), n - 1) * s.stride;
                dU[k] = s.u64[q];
                dV[k] = s.v64[q];
            }
        } else {
#pragma unroll
            for (int k = 0; k < kLane; ++k) dU[k] = dV[k] = 0.0;
        }
    };
    auto load_all = [&](long long c, float* du, float* dv, float* dh, float* d0, float* d1) {
        ld(u, c, du);
        ld(v, c, dv);
        ld(h, c, dh);
        ld(a0, c, d0);
        if constexpr (NOUT == 2) ld(a1, c, d1);
        else
#pragma unroll
            for (int k = 0; k < kLane; ++k) d1[k] = 0.0f;
#pragma unroll
        for (int k = 0; k < kLane; ++k) dh[k] = pidx(c, k) < n ? dh[k] : 0.0f;
    };
    int first_slot[kLane];
    // the prepared fields of every particle's first record (the paired store's payload)
    float first_c0[kLane], first_c1[kLane], first_band[kLane], first_lu[kLane],
        first_lv[kLane];
    unsigned first_box[kLane];
#pragma unroll
    for (int k = 0; k < kLane; ++k) {
        first_slot[k] = -1;
        first_c0[k] = first_c1[k] = first_band[k] = first_lu[k] = first_lv[k] = 0.0f;
        first_box[k] = 0u;
    }
    // NX: properties 2..5, loaded with the batch (software-pipelined like the others)
    float px[NX ? 4 : 1][kLane];
    auto load_x = [&](long long c, float (&dst)[NX ? 4 : 1][kLane]) {
        if constexpr (NX) {
#pragma unroll
            for (int j = 0; j < 4; ++j) ld(xa.a[j], c, dst[j]);
        }
    };
    long long bq = 0, br = 0;
    auto step_batch = [&]() {
        const bool wrap = br + 1 == gcnt;
        bq += wrap ? 1 : 0;
        br = wrap ? 0 : br + 1;
        return base_of(bq, br);
    };
    long long c = base_of(0, 0);  // the current batch's first particle
    load_all(c, pu, pv, ph, pa0, pa1);
    load_src(c, pU, pV);
    load_x(c, px);
#if ASP_SCATTER_PREFETCH >= 2
    // A/B build switch: the batch after next in flight as well
    long long cmid = step_batch();
    float mu[kLane], mv[kLane], mh[kLane], ma0[kLane], ma1[kLane];
    load_all(cmid, mu, mv, mh, ma0, ma1);
    double mU[kLane], mV[kLane];
    load_src(cmid, mU, mV);
    float mx_[NX ? 4 : 1][kLane];
    load_x(cmid, mx_);
#endif
    while (c < n) {
        const long long cn = step_batch();  // the next batch to load
        float nu[kLane], nv[kLane], nh[kLane], na0[kLane], na1[kLane];
        load_all(cn, nu, nv, nh, na0, na1);
        double nU[kLane], nV[kLane];
        load_src(cn, nU, nV);
        float nx_[NX ? 4 : 1][kLane];
        load_x(cn, nx_);
#pragma unroll
        for (int k = 0; k < kLane; ++k) {
            const int p = (int)pidx(c, k);
            Box b;
            if (!footprint<CULL>(g, s, p, pu[k], pv[k], ph[k], b)) continue;
            // the fixed-point bound is taken over the same fp32 coefficients the deposit
            // scales
            const float cf0 = (float)term_coef<KID>(pa0[k], ph[k]);
            const float cf1 = NOUT == 2 ? (float)term_coef<KID>(pa1[k], ph[k]) : 0.0f;
            float4 cx = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if constexpr (NX)
                cx = make_float4((float)term_coef<KID>(px[0][k], ph[k]),
                                 (float)term_coef<KID>(px[1][k], ph[k]),
                                 (float)term_coef<KID>(px[2][k], ph[k]),
                                 (float)term_coef<KID>(px[3][k], ph[k]));
            unsigned c0 = 0u, c1 = 0u;
            if constexpr (ACC == kAccFix) {
                c0 = __float_as_uint(fabsf(cf0));
                c1 = __float_as_uint(fabsf(cf1));
            }
            int tx0 = b.x0 >> kTileShift, tx1 = b.x1 >> kTileShift;
            int ty0 = b.y0 >> kTileShift, ty1 = b.y1 >> kTileShift;
            if ((tx1 - tx0 + 1) * (ty1 - ty0 + 1) > g.wide_tiles) {
                wide_list[atomicAdd(&ctr[cWideCursor], 1)] = p;
                if constexpr (ACC == kAccFix) {
                    atomicMax((unsigned*)&ctr[cWideMax0], c0);
                    if (NOUT == 2) atomicMax((unsigned*)&ctr[cWideMax1], c1);
                }
                continue;
            }
            const float band = rec_band(g.mgl, ph[k]);  // decided in the box-origin frame
            // coordinates relative to the record's box origin, from the exact inputs: the
            // deposit's pair arithmetic then carries 2^-24 of the pair distance, not of |u|
            // 
            const double U = SRC == 0 ? (double)pu[k] : SRC == 1 ? pU[k] : src_u(s, p, pu[k]);
            const double V = SRC == 0 ? (double)pv[k] : SRC == 1 ? pV[k] : src_v(s, p, pv[k]);
            first_c0[k] = cf0;
            first_c1[k] = cf1;
            first_band[k] = band;
            first_lu[k] = (float)(U - corner_x(g, max(b.x0, tx0 * kTile)));
            first_lv[k] = (float)(V - corner_y(g, max(b.y0, ty0 * kTile)));
            const bool mb = maybe_large(g, b);
            auto insert = [&](int tx, int ty, bool first) {
                const int t = tx * g.nty + ty;
                const unsigned bp = tile_box(b, tx, ty);
                const int col = mb && box_large(bp, g) ? t + g.ntiles : t;
#if ASP_SCATTER_ABLATE >= 2
                int slot = col;
#else
                int slot = atomicAdd(&cur[col], 1);
#endif
                if constexpr (NX) rec_store(&xa.ext[slot], cx);
                if constexpr (ACC == kAccFix) {
                    atomicMax(&cm[t * NOUT], c0);
                    if (NOUT == 2) atomicMax(&cm[t * NOUT + 1], c1);
                }
                if (first) {
                    first_slot[k] = slot;  // written by the paired store below
                    first_box[k] = bp;
                } else {
                    rec_store(&recs[2 * (long long)slot],
                              make_float4((float)(U - corner_x(g, max(b.x0, tx * kTile))),
                                          (float)(V - corner_y(g, max(b.y0, ty * kTile))),
                                          ph[k], cf0));
                    rec_store(&recs[2 * (long long)slot + 1],
                              make_float4(cf1, __int_as_float(p), band, __uint_as_float(bp)));
                }
            };
            if (tx1 - tx0 <= 1 && ty1 - ty0 <= 1) {  // at most 2 x 2 tiles: straight-line
                insert(tx0, ty0, true);
                if (tx1 > tx0) insert(tx1, ty0, false);
                if (ty1 > ty0) {
                    insert(tx0, ty1, false);
                    if (tx1 > tx0) insert(tx1, ty1, false);
                }
            } else {
                for (int tx = tx0; tx <= tx1; ++tx)
                    for (int ty = ty0; ty <= ty1; ++ty) insert(tx, ty, tx == tx0 && ty == ty0);
            }
        }
        // Paired store of every particle's first record: lanes 2j and 2j+1 write the two
        // 16-B halves of record j, so one store instruction covers 32 whole 32-B records
        // (32 lines) instead of 64 half records (64 lines).
        float4* st = stage + (threadIdx.x >> 6) * kStageF4;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < kLane; ++k) {
            const int p = (int)pidx(c, k);
            st[lane] = make_float4(first_lu[k], first_lv[k], ph[k], first_c0[k]);
            st[72 + lane] = make_float4(first_c1[k], __int_as_float(p), first_band[k],
                                        __uint_as_float(first_box[k]));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                int src = half * 32 + (lane >> 1);
                int slot = __shfl(first_slot[k], src);
                float4 val = st[(lane & 1) * 72 + src];
                if (slot >= 0) rec_store(&recs[2 * (long long)slot + (lane & 1)], val);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            first_slot[k] = -1;
        }
#if ASP_SCATTER_PREFETCH >= 2
#pragma unroll
        for (int k = 0; k < kLane; ++k) {
            pu[k] = mu[k], mu[k] = nu[k];
            pv[k] = mv[k], mv[k] = nv[k];
            ph[k] = mh[k], mh[k] = nh[k];
            pa0[k] = ma0[k], ma0[k] = na0[k];
            pa1[k] = ma1[k], ma1[k] = na1[k];
            pU[k] = mU[k], mU[k] = nU[k];
            pV[k] = mV[k], mV[k] = nV[k];
        }
        if constexpr (NX)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < kLane; ++k) px[j][k] = mx_[j][k], mx_[j][k] = nx_[j][k];
        c = cmid;
        cmid = cn;
#else
#pragma unroll
        for (int k = 0; k < kLane; ++k) {
            pu[k] = nu[k];
            pv[k] = nv[k];
            ph[k] = nh[k];
            pa0[k] = na0[k];
            pa1[k] = na1[k];
            pU[k] = nU[k];
            pV[k] = nV[k];
        }
        if constexpr (NX)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < kLane; ++k) px[j][k] = nx_[j][k];
        c = cn;
#endif
    }
    __syncthreads();
    if constexpr (ACC == kAccFix) {
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
                                                      int ntiles, const int* __restrict__ tile_total,
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
            k[o] = scale_exp((long long)tile_total[t] + tile_total[t + ntiles],
                             __uint_as_float(mm));
        }
        tile_k[t] = make_int2(k[0], k[1]);
    }
}

// ----------------------------------------------------------------------------------
// Deposit building blocks.  LDS tile: NOUT maps of 64 rows x kRow words (fp64 or int64),
// pixel (lx, ly) of the tile at word lx * kRow + ly.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ int pix(int lx, int ly) { return lx * kRow + ly; }

template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void accumulate(const Prep& P, float r2, unsigned long long* acc0,
                                           unsigned long long* acc1, int k) {
    float q = __builtin_amdgcn_sqrtf(r2) * P.hinv;  // v_sqrt_f32, 1 ulp
    float w = kernel_shape<KID>(q);
    acc_add<ACC>(&acc0[k], P.s0 * w);
    if constexpr (NOUT == 2) acc_add<ACC>(&acc1[k], P.s1 * w);
}

// One wave sweeps the (clipped) box of one wave-uniform record: lanes along y (the
// contiguous image axis), so the LDS atomics of a wave hit distinct consecutive words.
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void sweep(const Grid& g, const Src64& s, const Prep& P, int X0, int Y0,
                                      const float* xt, const float* yt,
                                      unsigned long long* acc0, unsigned long long* acc1,
                                      int lane) {
    int bh = P.b.y1 - P.b.y0 + 1;
    if (bh <= 64) {
        int rps = 64 / bh;
        int r = lane / bh, c = lane - r * bh;
        if (r < rps) {
            int yi = P.b.y0 + c;
            float Y = yt[c];
            for (int xi = P.b.x0 + r; xi <= P.b.x1; xi += rps) {
                float r2;
                if (decide(g, s, P, xi, yi, xt[xi - P.b.x0], Y, r2))
                    accumulate<KID, NOUT, ACC>(P, r2, acc0, acc1, pix(xi - X0, yi - Y0));
            }
        }
    } else {
        for (int xi = P.b.x0; xi <= P.b.x1; ++xi) {
            float X = xt[xi - P.b.x0];
            for (int c = lane; c < bh; c += 64) {
                int yi = P.b.y0 + c;
                float r2;
                if (decide(g, s, P, xi, yi, X, yt[c], r2))
                    accumulate<KID, NOUT, ACC>(P, r2, acc0, acc1, pix(xi - X0, yi - Y0));
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
    Q.thr = bcast(P.thr, l);
    Q.band = bcast(P.band, l);
    Q.p = bcast(P.p, l);
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

// A prepared record {u, v, h, c0}, {c1, p, band, box} -> the pair loop's state.  Only
// (2h)^2 and 1/h are recomputed (the same fp32 operations as the scatter's), and in
// fixed-point mode the tile's power-of-two scale applied (ldexp: exact).
template <int ACC>
__device__ __forceinline__ void rec_prep(const float4& r0, const float4& r1, int X0, int Y0,
                                         int2 kk, Prep& P) {
    P.u = r0.x;
    P.v = r0.y;
    P.h = r0.z;
    P.p = __float_as_int(r1.y);
    set_band(P, rec_thr(r0.z), r1.z);
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
}

__device__ __forceinline__ void load_rec(const float4* recs, long long i, float4& r0, float4& r1) {
    r0 = recs[2 * i];
    r1 = recs[2 * i + 1];
}

// asp_project2d_props, pass 1 / 2: the record's coefficients of properties (2, 3) / (4, 5)
// replace those of (0, 1) (EXT kernels; the binning, band and box are the record's own).
__device__ __forceinline__ void ext_coef(Prep& P, const float4& e, int pass) {
    P.s0 = pass == 1 ? e.x : e.z;
    P.s1 = pass == 1 ? e.y : e.w;
}

constexpr int kTilePix = kTile * kTile;
constexpr int kFlagAccumulate = 1;
constexpr int kFlagRatio = 2;  // fused ratio: out0 <- map0 / map1

// Corner offset tables: xt[k] = fl32(k * pitch_x), yt[k] = fl32(k * pitch_y) for k < 64 --
// the corner k pixels from a record's box origin, in the frame of the record's (u, v)
// (fl32 of the exact offset from the box origin's corner; the error budget is DESIGN.md
// §3's).  The gathers use them from the tile origin.
__device__ __forceinline__ void corner_tables(const Grid& g, int X0, int Y0, float* xt,
                                              float* yt) {
    (void)X0;
    (void)Y0;
    if (threadIdx.x < kTile)
        xt[threadIdx.x] = (float)((double)threadIdx.x * g.psx);
    else if (threadIdx.x < 2 * kTile)
        yt[threadIdx.x - kTile] = (float)((double)(threadIdx.x - kTile) * g.psy_pix);
}

// Tile prologue: zero accumulators, corner tables.
template <int NOUT, int NT>
__device__ __forceinline__ void tile_prologue(const Grid& g, int X0, int Y0,
                                              unsigned long long* acc, float* xt, float* yt) {
    for (int i = threadIdx.x; i < NOUT * kTileWords; i += NT) acc[i] = 0ull;
    corner_tables(g, X0, Y0, xt, yt);
    __syncthreads();
}

// Convert a pixel's sums and write it (plain store: the tile has one owner).
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

// Lane-per-record deposit of a box of at most S x S pixels: dy^2 per column in
// registers, an unrolled S x S pass decides every pair whose fp32 r2 is outside the error
// band and accumulates it; band pairs (~0.1 %) only set a bit, resolved afterwards in
// fp64 -- keeping the rare slow path out of the unrolled body.
template <int KID, int NOUT, int ACC, int S>
__device__ __forceinline__ void small_box(const Grid& g, const Src64& s, const Prep& P, int bw,
                                          int bh, int X0, int Y0, const float* xt,
                                          const float* yt, unsigned long long* acc0,
                                          unsigned long long* acc1) {
    const int base = pix(P.b.x0 - X0, P.b.y0 - Y0);  // LDS word of pixel (0, 0)
    float dy2[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
        float dy = P.v - yt[min(j, bh - 1)];
        dy2[j] = dy * dy;
    }
    unsigned amb = 0u;
#pragma unroll
    for (int ii = 0; ii < S; ++ii) {
        if (ii < bw) {
            float dx = P.u - xt[ii];
            float dx2 = dx * dx;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                if (j < bh) {
                    float r2 = dx2 + dy2[j];
                    bool a = r2 >= P.lo && r2 <= P.hi;
                    amb |= a ? (1u << (ii * S + j)) : 0u;
                    if (r2 < P.lo)
                        accumulate<KID, NOUT, ACC>(P, r2, acc0, acc1, base + ii * kRow + j);
                }
            }
        }
    }
    while (amb) {
        int bit = __builtin_ctz(amb);
        amb &= amb - 1u;
        int ii = bit / S, j = bit - (bit / S) * S;
        int xi = P.b.x0 + ii, yi = P.b.y0 + j;
        if (exact_pair(g, s, P.p, xi, yi)) {
            float dx = P.u - xt[ii], dy = P.v - yt[j];
            accumulate<KID, NOUT, ACC>(P, dx * dx + dy * dy, acc0, acc1, pix(xi - X0, yi - Y0));
        }
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) {  // v_pk_fma_f32
    return __builtin_elementwise_fma(a, b, c);
}

// Kernel shape on two pairs at once (packed fp32).  Only pairs with fp32 r2 < (2h)^2 use
// the result, so q < 2 up to rounding and the Wendland clamp is not needed there (a q a
// few ulp over 2 gives a term ~1e-28 of the peak).
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
// tile; the caller defers it to the exact path (small_box).  The three corner offsets per
// axis come from registers (Corner3: the corner tables' first entries, the same fp32
// values), not LDS: a table read here made every batch wait (lgkmcnt) for the previous
// batch's LDS atomics, which complete in order ahead of it.
struct Corner3 {
    float x[3], y[3];
};
__device__ __forceinline__ Corner3 corner3(const Grid& g) {  // = xt[0..2], yt[0..2]
    Corner3 c;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        c.x[k] = (float)((double)k * g.psx);
        c.y[k] = (float)((double)k * g.psy_pix);
    }
    return c;
}
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ bool small3_fast(const Prep& P, int bw, int bh, int X0, int Y0,
                                            const Corner3& cc,
                                            unsigned long long* acc0, unsigned long long* acc1) {
    constexpr float kFar = 1e18f;  // outside the box: r2 ~ 1e36, far from any threshold
    float dx2[3];
    f2v dy2;
    float dyc2;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float d = P.u - cc.x[i];
        d = i < bw ? d : kFar;
        dx2[i] = d * d;
    }
    {
        float d0 = P.v - cc.y[0];
        float d1 = P.v - cc.y[1];
        float d2 = P.v - cc.y[2];
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
    const int base = pix(P.b.x0 - X0, P.b.y0 - Y0);
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
        const int k = base + i * kRow;
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

// Per-wave list of records deferred to the exact path (a pair in the error band).
constexpr int kDeferCap = 128;

// Exact body for deferred records: lanes 0 .. cnt-1 take list entries first .. first+cnt-1
// (record indices within the item), reload and re-prepare them and decide every pair
// with the error-band / fp64 logic of small_box.  Wave-level: no block barrier.
template <int KID, int NOUT, int ACC, int EXT>
__device__ __forceinline__ void deferred(const Grid& g, const Src64& s,
                                         const float4* __restrict__ recs,
                                         const float4* __restrict__ ext, int pass, long long start,
                                         const int* dlist, int first, int cnt, int X0, int Y0,
                                         int2 kk, const float* xt, const float* yt,
                                         unsigned long long* acc0, unsigned long long* acc1,
                                         int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int idx = lane < cnt ? dlist[first + lane] : -1;
    __builtin_amdgcn_wave_barrier();
    if (idx < 0) return;
    float4 r0, r1;
    load_rec(recs, start + idx, r0, r1);
    Prep P;
    rec_prep<ACC>(r0, r1, X0, Y0, kk, P);
    if constexpr (EXT) ext_coef(P, ext[start + idx], pass);
    small_box<KID, NOUT, ACC, 4>(g, s, P, P.b.x1 - P.b.x0 + 1, P.b.y1 - P.b.y0 + 1, X0, Y0, xt,
                                 yt, acc0, acc1);
}

// ----------------------------------------------------------------------------------
// Gather form for mid and large boxes (K4g, K6).  A sweep costs an LDS atomic per pair
// and a pass per 64 box pixels; here every thread OWNS 8 pixels of the tile and sums
// their terms in registers.  Wave w owns the 16 x 32 region rows 16 (w / 2) .., columns
// 32 (w % 2) .., as 2 x 4 blocks of 8 x 8 pixels; lane l owns pixel (l / 8, l % 8) of
// each block (block j: block row j / 4, block column j % 4).  Each wave streams the
// item's records itself, 64 at a time (lane i prepares record i into a GEntry held in
// VGPRs), ballots which of them meet its region and walks those: v_readlane puts the
// entry's fields in SGPRs, the blocks the box meets are found with scalar compares, and
// only those blocks' pixels are evaluated -- one pixel per lane per block, so an entry
// costs ~ its box area / 64 wave instructions-per-pixel, whatever its size.  No LDS list,
// no block barrier, no atomics.  Sums: fp32 partials over <= 64 entries folded into fp64
// totals the thread owns in LDS (kAccF64), or exact int64 fixed point in registers
// (kAccFix).
// ----------------------------------------------------------------------------------
constexpr int kGatherThreads = 64;  // one wave per workgroup: one region of the tile
constexpr int kGatherRegions = 8;   // 16 x 32-pixel regions per tile
constexpr int kGatherPix = 8 * kGatherThreads;
static_assert(kGatherRegions * kGatherPix == kTile * kTile, "8 regions x 512 pixels cover the tile");
constexpr int kKernelIndicator = ASP_KERNEL_INDICATOR;
struct GEntry {
    float u, v, lo, hi, hinv, s0, s1;  // tile frame; s0, s1 with the shape's scale folded in
    int p;
    unsigned box;  // tile-local x0 | x1 << 8 | y0 << 16 | y1 << 24 (kNoBox: nothing)
};
constexpr unsigned kNoBox = 0x00ff00ffu;  // x0 = 255 > x1 = 0: meets no region

// One thread's 8 pixels: fp32 partials in registers folded into fp64 totals that the
// thread owns in LDS (kAccF64; word j * 64 + lane: conflict-free), or exact int64
// fixed-point sums in registers (kAccFix).
template <int NOUT, int ACC>
struct GAcc {
    unsigned long long a0[8], a1[8];  // kAccFix sums
    f2 p0[4], p1[4];                  // kAccF64 fp32 partials, pixels (2k, 2k + 1)
    double* t0;
    double* t1;
    __device__ __forceinline__ void init(double* tot) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a0[j] = 0;
            a1[j] = 0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            p0[k] = (f2){0.0f, 0.0f};
            p1[k] = (f2){0.0f, 0.0f};
        }
        t0 = tot + threadIdx.x;
        t1 = tot + kGatherPix + threadIdx.x;
        if constexpr (ACC != kAccFix) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                t0[j * kGatherThreads] = 0.0;
                if (NOUT == 2) t1[j * kGatherThreads] = 0.0;
            }
        }
    }
    // pixel j += w * (s0, s1)
    __device__ __forceinline__ void add(int j, float w, float s0, float s1) {
        if constexpr (ACC == kAccFix) {
            a0[j] += f2fix(s0 * w);
            if (NOUT == 2) a1[j] += f2fix(s1 * w);
        } else {
            p0[j >> 1][j & 1] = fmaf(s0, w, p0[j >> 1][j & 1]);
            if (NOUT == 2) p1[j >> 1][j & 1] = fmaf(s1, w, p1[j >> 1][j & 1]);
        }
    }
    // pixels 2k, 2k + 1 += w.xy * (s0, s1)  (one v_pk_fma_f32 per map)
    __device__ __forceinline__ void add2(int k, f2 w, float s0, float s1) {
        if constexpr (ACC == kAccFix) {
            add(2 * k, w.x, s0, s1);
            add(2 * k + 1, w.y, s0, s1);
        } else {
            p0[k] = __builtin_elementwise_fma(w, (f2){s0, s0}, p0[k]);
            if (NOUT == 2) p1[k] = __builtin_elementwise_fma(w, (f2){s1, s1}, p1[k]);
        }
    }
    __device__ __forceinline__ void fold() {
        if constexpr (ACC != kAccFix) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                t0[j * kGatherThreads] += (double)p0[j >> 1][j & 1];
                if (NOUT == 2) t1[j * kGatherThreads] += (double)p1[j >> 1][j & 1];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                p0[k] = (f2){0.0f, 0.0f};
                p1[k] = (f2){0.0f, 0.0f};
            }
        }
    }
    // the accumulator word of pixel j (as the LDS tile / slabs hold it)
    __device__ __forceinline__ unsigned long long word0(int j) const {
        if constexpr (ACC == kAccFix) return a0[j];
        else return (unsigned long long)__double_as_longlong(t0[j * kGatherThreads]);
    }
    __device__ __forceinline__ unsigned long long word1(int j) const {
        if constexpr (ACC == kAccFix) return a1[j];
        else return (unsigned long long)__double_as_longlong(t1[j * kGatherThreads]);
    }
};

// LDS of K4g / K6: the fp64 totals, one word per pixel and map (none in fixed point).
template <int NOUT, int ACC>
constexpr size_t gather_lds() {
    return ACC == kAccFix ? 8 : (size_t)NOUT * kGatherPix * 8;
}

// This thread's pixels: pixel j at row r0 + 8 (j / 4) + lr, column c0 + 8 (j % 4) + lc.
struct GOwn {
    int r0, c0;  // the wave's region (uniform)
    int lr, lc;  // the lane's place in each 8 x 8 block
    __device__ __forceinline__ int row(int j) const { return r0 + 8 * (j >> 2) + lr; }
    __device__ __forceinline__ int col(int j) const { return c0 + 8 * (j & 3) + lc; }
};
__device__ __forceinline__ GOwn gather_owner(int w) {  // w: the region (uniform)
    const int lane = threadIdx.x;
    GOwn o;
    o.r0 = (w >> 1) * 16;
    o.c0 = (w & 1) * 32;
    o.lr = lane >> 3;
    o.lc = lane & 7;
    return o;
}

// Tile-local corner offsets fl32(k * pitch): the values of the corner tables (K4), here
// computed where they are needed (a gather workgroup has no tables).
__device__ __forceinline__ float corner_off_x(const Grid& g, int k) { return (float)((double)k * g.psx); }
__device__ __forceinline__ float corner_off_y(const Grid& g, int k) { return (float)((double)k * g.psy_pix); }

// The corner coordinates of the thread's pixels: 2 rows, 4 columns; and (wave-uniform) the
// corner span of each of the region's 8 x 16 half block rows: rows xl[r]..xh[r] of block
// row r, columns yl[k]..yh[k] of column half k.
struct GCorner {
    float X[2], Y[4];
    float xl[2], xh[2], yl[2], yh[2];
};
__device__ __forceinline__ GCorner gather_corners(const Grid& g, const GOwn& o) {
    GCorner c;
    c.X[0] = corner_off_x(g, o.row(0));
    c.X[1] = corner_off_x(g, o.row(4));
#pragma unroll
    for (int k = 0; k < 4; ++k) c.Y[k] = corner_off_y(g, o.col(k));
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        c.xl[r] = corner_off_x(g, o.r0 + 8 * r);
        c.xh[r] = corner_off_x(g, o.r0 + 8 * r + 7);
        c.yl[r] = corner_off_y(g, o.c0 + 16 * r);
        c.yh[r] = corner_off_y(g, o.c0 + 16 * r + 15);
    }
    return c;
}

// The region's half block rows the entry's DISC can reach (bit 2 r + k: block row r,
// column half k), from the distance between (u, v) and each half row's corner rectangle
// (closest point by clamping).  Conservative: a skipped half row has every pixel at
// fp32 distance^2 >= lim = (2h)^2 (1 + 2^-8) from the particle -- far outside any rounding
// of the pair distance -- so the edge form (§3) gives each of them exactly 0 and skipping
// them changes no sum.  Computed per lane for its own entry before the walk (vectorised
// over the 64 entries), so the walk tests bits instead of box bounds.
__device__ __forceinline__ unsigned edge_mask(const GCorner& c, float u, float v, float thr) {
    float dx2[2], dy2[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const float dx = u - fminf(fmaxf(u, c.xl[r]), c.xh[r]);
        const float dy = v - fminf(fmaxf(v, c.yl[r]), c.yh[r]);
        dx2[r] = dx * dx;
        dy2[r] = dy * dy;
    }
    const float lim = thr * (1.0f + 0x1p-8f);
    unsigned m = 0u;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 2; ++k) m |= (dx2[r] + dy2[k] < lim) ? 1u << (2 * r + k) : 0u;
    return m;
}

__device__ __forceinline__ GEntry make_gentry(const Prep& P, int X0, int Y0, float scale) {
    GEntry e;
    e.u = P.u; e.v = P.v; e.lo = P.lo; e.hi = P.hi; e.hinv = P.hinv;
    e.s0 = P.s0 * scale; e.s1 = P.s1 * scale; e.p = P.p;
    e.box = (unsigned)(P.b.x0 - X0) | ((unsigned)(P.b.x1 - X0) << 8) |
            ((unsigned)(P.b.y0 - Y0) << 16) | ((unsigned)(P.b.y1 - Y0) << 24);
    return e;
}

__device__ __forceinline__ bool meets_region(unsigned box, const GOwn& o) {
    return (int)(box & 255u) <= o.r0 + 15 && (int)((box >> 8) & 255u) >= o.r0 &&
           (int)((box >> 16) & 255u) <= o.c0 + 31 && (int)(box >> 24) >= o.c0;
}

// Lane l's entry, wave-uniform (SGPRs).
__device__ __forceinline__ GEntry lane_entry(const GEntry& e, int l) {
    GEntry E;
    E.u = bcast(e.u, l); E.v = bcast(e.v, l); E.lo = bcast(e.lo, l); E.hi = bcast(e.hi, l);
    E.hinv = bcast(e.hinv, l); E.s0 = bcast(e.s0, l); E.s1 = bcast(e.s1, l);
    E.p = bcast(e.p, l); E.box = (unsigned)bcast((int)e.box, l);
    return E;
}

// Which of the wave's 8 blocks the box meets (bit j; uniform).
__device__ __forceinline__ unsigned block_hits(unsigned box, const GOwn& o) {
    const int x0 = box & 255u, x1 = (box >> 8) & 255u;
    const int y0 = (box >> 16) & 255u, y1 = box >> 24;
    unsigned m = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int br = o.r0 + 8 * (j >> 2), bc = o.c0 + 8 * (j & 3);
        if (x0 <= br + 7 && x1 >= br && y0 <= bc + 7 && y1 >= bc) m |= 1u << j;
    }
    return m;
}

// Edge-continuous kernels (cubic / Wendland) on a square grid without a mixed cull take no
// decision at all (gather_entry_masked below): W by edge_shape for every pixel of every
// 8 x 16 half block row the entry's disc reaches.  A pixel the reference excludes has
// exact r >= 2h, so its fp32 q is >= 2 (1 - 2^-21) and its term 0 or < 2^-60 W(0); one it
// includes the same way.

// One (uniform) entry, every other case: the box's own rows and columns (non-square grids
// and mixed culls clip the box to the chunk ranges), the error band and the fp64
// decision -- the indicator kernel's neighbour sets are the reference's exactly.
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void gather_entry(const Grid& g, const Src64& s, const GEntry& E,
                                             int X0, int Y0, const GOwn& o, const GCorner& c,
                                             GAcc<NOUT, ACC>& ga) {
    const unsigned m = block_hits(E.box, o);
    const int x0 = E.box & 255u, x1 = (E.box >> 8) & 255u;
    const int y0 = (E.box >> 16) & 255u, y1 = E.box >> 24;
    unsigned in = 0u, amb = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (m & (1u << j)) {
            const float dx = E.u - c.X[j >> 2], dy = E.v - c.Y[j & 3];
            const float r2 = dx * dx + dy * dy;
            const bool inb = (unsigned)(o.row(j) - x0) <= (unsigned)(x1 - x0) &&
                             (unsigned)(o.col(j) - y0) <= (unsigned)(y1 - y0);
            in |= (inb && r2 < E.lo) ? (1u << j) : 0u;
            amb |= (inb && r2 >= E.lo && r2 <= E.hi) ? (1u << j) : 0u;
        }
    }
    for (unsigned a = amb; a; a &= a - 1u) {  // the reference's fp64 decision, one call site
        const int j = __builtin_ctz(a);
        if (exact_pair(g, s, E.p, X0 + o.row(j), Y0 + o.col(j))) in |= 1u << j;
    }
    const float sc = 1.0f / kShapeScale<KID>;  // s0, s1 carry the edge form's scale
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (in & (1u << j)) {  // (the same r2 as above: same operations)
            const float dx = E.u - c.X[j >> 2], dy = E.v - c.Y[j & 3];
            const float r2 = dx * dx + dy * dy;
            const float wk = kernel_shape<KID>(__builtin_amdgcn_sqrtf(r2) * E.hinv) * sc;
            ga.add(j, wk, E.s0, E.s1);
        }
    }
}

// One (uniform) entry of the edge path given its half-row mask bm (edge_mask).
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void gather_entry_masked(float u, float vs, float hinv, float s0,
                                                    float s1, unsigned bm, const GCorner& c,
                                                    GAcc<NOUT, ACC>& ga) {
    const f2 hv = {-hinv, -hinv};
    const f2 vv = {vs, vs};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        if (bm & (3u << (2 * r))) {
            const float dxs = (u - c.X[r]) * hinv;
            const f2 dx2 = {dxs * dxs, dxs * dxs};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (bm & (1u << (2 * r + k))) {
                    const f2 dys = __builtin_elementwise_fma(hv, (f2){c.Y[2 * k], c.Y[2 * k + 1]}, vv);
                    const f2 r2 = __builtin_elementwise_fma(dys, dys, dx2);
                    f2 q;
                    q.x = __builtin_amdgcn_sqrtf(r2.x);
                    q.y = __builtin_amdgcn_sqrtf(r2.y);
                    ga.add2(2 * r + k, edge_shape2<KID>(q), s0, s1);
                }
            }
        }
    }
}

// The wave's walk over its lanes' entries: those whose box meets the wave's region.
template <int KID, int NOUT, int ACC>
__device__ __forceinline__ void gather_walk(const Grid& g, const Src64& s, const GEntry& mine,
                                            int X0, int Y0, const GOwn& o, const GCorner& c,
                                            GAcc<NOUT, ACC>& ga) {
    if (KID != kKernelIndicator && !g.nonsquare && !g.mixed) {  // uniform
        // edge path: each lane finds the half rows its entry's disc reaches, and precomputes
        // v / h; the walk then reads 6 words per entry and tests mask bits
        const unsigned em = mine.box == kNoBox ? 0u : edge_mask(c, mine.u, mine.v, mine.hi);
        const float vs = mine.v * mine.hinv;
        unsigned long long m = __ballot(em != 0u);
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            gather_entry_masked<KID, NOUT, ACC>(bcast(mine.u, l), bcast(vs, l), bcast(mine.hinv, l),
                                                bcast(mine.s0, l), bcast(mine.s1, l),
                                                (unsigned)bcast((int)em, l), c, ga);
        }
    } else {
        unsigned long long m = __ballot(meets_region(mine.box, o));
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            gather_entry<KID, NOUT, ACC>(g, s, lane_entry(mine, l), X0, Y0, o, c, ga);
        }
    }
    ga.fold();
}

// Write the thread's 8 pixels: partial slab (split tiles) or the map.
template <int NOUT, int ACC>
__device__ __forceinline__ void gather_emit(const Grid& g, const GAcc<NOUT, ACC>& ga,
                                            const GOwn& o, int X0, int Y0, int slab,
                                            unsigned long long* slabs, int k0, int k1,
                                            float* out0, float* out1, int flags) {
    if (slab >= 0) {  // unpadded slab layout
        unsigned long long* dst = slabs + (long long)slab * NOUT * kTilePix;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = o.row(j) * kTile + o.col(j);
            dst[k] = ga.word0(j);
            if (NOUT == 2) dst[kTilePix + k] = ga.word1(j);
        }
        return;
    }
    const int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (o.row(j) >= TW || o.col(j) >= TH) continue;
        const long long off = (long long)(X0 + o.row(j)) * g.ny + (Y0 + o.col(j));
        emit_pixel<NOUT, ACC>(off, ga.word0(j), NOUT == 2 ? ga.word1(j) : 0ull, k0, k1, out0,
                              out1, flags);
    }
}

// Which records take which path in K4 (clipped box w x h pixels).
__device__ __forceinline__ bool is_small(int bw, int bh) { return bw <= 4 && bh <= 4; }

// ----------------------------------------------------------------------------------
// K4: deposit one work item (a run of records of one tile) into LDS, then write the
// tile (single-item tiles) or its partial slab (split tiles).
// ----------------------------------------------------------------------------------
template <int NOUT>
constexpr size_t deposit_lds() {
    return (size_t)NOUT * kTileWords * 8 + 2 * kTile * 4;
}

template <int KID, int NOUT, int ACC, int EXT = 0>
__global__ __launch_bounds__(kDepBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_deposit(
    Grid g, Src64 s, const float4* __restrict__ recs, const Item* __restrict__ items,
    const int* __restrict__ order, const int2* __restrict__ tile_k,
    unsigned long long* __restrict__ slabs, float* __restrict__ out0, float* __restrict__ out1,
    int flags, const float4* __restrict__ ext, int pass) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];
    unsigned long long* acc0 = acc;
    unsigned long long* acc1 = acc + kTileWords;
    float* xt = (float*)(acc + NOUT * kTileWords);
    float* yt = xt + kTile;
    __shared__ int defer_lds[kDepBlock / 64][kDeferCap];
#if ASP_SCATTER_ABLATE
    return;
#endif
    const Item it = items[order[blockIdx.x]];  // largest items first (k_tilescan)
    if (it.mode != 0) return;  // the large stream's (K4g)
    int tx = it.tile / g.nty, ty = it.tile - (it.tile / g.nty) * g.nty;
    int X0 = tx * kTile, Y0 = ty * kTile;
    int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    if (it.count == 0) {  // empty tile: the map is 0 there
        if (flags & kFlagAccumulate) return;
        for (int k = threadIdx.x; k < kTilePix; k += kDepBlock) {
            int lx = k >> kTileShift, ly = k & (kTile - 1);
            if (lx >= TW || ly >= TH) continue;
            long long o = (long long)(X0 + lx) * g.ny + (Y0 + ly);
            out0[o] = 0.0f;
            if (NOUT == 2) out1[o] = 0.0f;
        }
        return;
    }
    const int2 kk = ACC == kAccFix ? tile_k[it.tile] : make_int2(0, 0);
    tile_prologue<NOUT, kDepBlock>(g, X0, Y0, acc, xt, yt);
    const int lane = threadIdx.x & 63;
    const Corner3 c3 = corner3(g);
    int* dlist = defer_lds[threadIdx.x >> 6];
    int ndef = 0;  // wave-uniform
    // One batch: record i (index within the item; r0, r1 its halves) of every thread.
    auto batch = [&](int i, const float4& r0, const float4& r1, const float4& e) {
        Prep P;
        P.b = Box{0, -1, 0, -1};
        bool live = i < it.count;
        if (live) {
            rec_prep<ACC>(r0, r1, X0, Y0, kk, P);
            if constexpr (EXT) ext_coef(P, e, pass);
        }
        live = live && P.b.x0 <= P.b.x1;  // (an empty box deposits nothing)
        const int bw = P.b.x1 - P.b.x0 + 1, bh = P.b.y1 - P.b.y0 + 1;
        const bool small = live && is_small(bw, bh);
        bool amb = false;
        if (small) {
            // lane-per-record.  Boxes of <= 3 x 3 corners (pixel-scale h) take the packed
            // body; 4-wide boxes and records with a pair in the error band are deferred to
            // the exact body, a full wave of them at a time
            if (bw <= 3 && bh <= 3)
                amb = !small3_fast<KID, NOUT, ACC>(P, bw, bh, X0, Y0, c3, acc0, acc1);
            else
                amb = true;
        }
        {
            unsigned long long am = __ballot(amb);
            if (am) {
                if (amb) dlist[ndef + __popcll(am & ((1ull << lane) - 1ull))] = i;
                ndef += __popcll(am);
                if (ndef >= 64) {  // a full wave of deferred records
                    ndef -= 64;
                    deferred<KID, NOUT, ACC, EXT>(g, s, recs, ext, pass, it.start, dlist, ndef,
                                                  64, X0, Y0, kk, xt, yt, acc0, acc1, lane);
                }
            }
        }
        unsigned long long mid = __ballot(live && !small);
        while (mid) {
            int l = __builtin_ctzll(mid);
            mid &= mid - 1;
            Prep Q = bcast_prep(P, l);
            sweep<KID, NOUT, ACC>(g, s, Q, X0, Y0, xt, yt, acc0, acc1, lane);
        }
    };
    const int last = it.count - 1;
    // Software pipeline: batch i + 2 is issued before batch i deposits.  The loads are
    // unconditional (index clamped to the item's last record; lanes past the end ignore
    // theirs), so every iteration issues the same two loads and the compiler's wait
    // before batch i leaves the batch just issued in flight (vmcnt(2); the register
    // rotation makes it wait for batch i + 1 too).  Loads under a branch made it
    // vmcnt(0), i.e. one full memory latency per batch: deposit 1.26 -> 1.22 ms (cfg 3).
    float4 r0, r1, q0, q1, re, qe;  // (re, qe, ne: the EXT coefficients, pass > 0)
    auto load_ext = [&](long long i, float4& e) {
        if constexpr (EXT) e = ext[i];
        else e = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    };
    load_rec(recs, it.start + min((int)threadIdx.x, last), r0, r1);
    load_ext(it.start + min((int)threadIdx.x, last), re);
    load_rec(recs, it.start + min((int)threadIdx.x + kDepBlock, last), q0, q1);
    load_ext(it.start + min((int)threadIdx.x + kDepBlock, last), qe);
    for (int base = 0; base < it.count; base += kDepBlock) {
        float4 n0, n1, ne;
        load_rec(recs, it.start + min(base + (int)threadIdx.x + 2 * kDepBlock, last), n0, n1);
        load_ext(it.start + min(base + (int)threadIdx.x + 2 * kDepBlock, last), ne);
        batch(base + threadIdx.x, r0, r1, re);
        r0 = q0;
        r1 = q1;
        re = qe;
        q0 = n0;
        q1 = n1;
        qe = ne;
    }
    if (ndef > 0)
        deferred<KID, NOUT, ACC, EXT>(g, s, recs, ext, pass, it.start, dlist, 0, ndef, X0, Y0, kk,
                                      xt, yt, acc0, acc1, lane);
    __syncthreads();
    if (it.slab >= 0) {  // split tile: partial sums, merged by K5 (slab layout unpadded)
        unsigned long long* dst = slabs + (long long)it.slab * NOUT * kTilePix;
        for (int k = threadIdx.x; k < kTilePix; k += kDepBlock) {
            const int w = pix(k >> kTileShift, k & (kTile - 1));
            dst[k] = acc0[w];
            if (NOUT == 2) dst[kTilePix + k] = acc1[w];
        }
        return;
    }
    for (int k = threadIdx.x; k < kTilePix; k += kDepBlock) {
        int lx2 = k >> kTileShift, ly = k & (kTile - 1);
        if (lx2 >= TW || ly >= TH) continue;
        long long o = (long long)(X0 + lx2) * g.ny + (Y0 + ly);
        const int w = pix(lx2, ly);
        emit_pixel<NOUT, ACC>(o, acc0[w], NOUT == 2 ? acc1[w] : 0ull, kk.x, kk.y, out0, out1,
                              flags);
    }
}

// ----------------------------------------------------------------------------------
// K4g: deposit one work item of the LARGE stream (records whose clipped box is at least
// gather_min pixels on both axes, or gather_area pixels) in the gather form: every wave streams the item's
// records 64 at a time (coalesced 32-B loads, the next 64 in flight) and walks those that
// meet its region (gather_walk).  The tile (or its partial slab) is written straight
// from the registers.
// ----------------------------------------------------------------------------------
template <int KID, int NOUT, int ACC, int EXT = 0>
__global__ __launch_bounds__(kGatherThreads) void k_gather(
    Grid g, Src64 s, const float4* __restrict__ recs, const Item* __restrict__ items,
    const int* __restrict__ order, const int2* __restrict__ tile_k,
    unsigned long long* __restrict__ slabs, float* __restrict__ out0, float* __restrict__ out1,
    int flags, const float4* __restrict__ ext, int pass) {
    extern __shared__ __attribute__((aligned(16))) double tot[];
#if ASP_SCATTER_ABLATE
    return;
#endif
    const Item it = items[order[blockIdx.x / kGatherRegions]];  // largest first
    if (it.mode != 1) return;
    const int tx = it.tile / g.nty, ty = it.tile - (it.tile / g.nty) * g.nty;
    const int X0 = tx * kTile, Y0 = ty * kTile;
    const int2 kk = ACC == kAccFix ? tile_k[it.tile] : make_int2(0, 0);
    const int lane = threadIdx.x;
    // unconditional loads (index clamped to the item's last record), so no wait or copy
    // of the next batch is forced inside the walk
    const int last = it.count - 1;
    float4 r0, r1, e = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    load_rec(recs, it.start + min(lane, last), r0, r1);
    if constexpr (EXT) e = ext[it.start + min(lane, last)];
    const GOwn o = gather_owner(blockIdx.x % kGatherRegions);
    GAcc<NOUT, ACC> ga;
    ga.init(tot);
    const GCorner cc = gather_corners(g, o);
    for (int base = 0; base < it.count; base += 64) {
        GEntry mine;
        mine.box = kNoBox;
        if (base + lane < it.count) {
            Prep P;
            rec_prep<ACC>(r0, r1, X0, Y0, kk, P);
            if constexpr (EXT) ext_coef(P, e, pass);
            P.u += corner_off_x(g, P.b.x0 - X0);  // box-origin frame -> tile frame
            P.v += corner_off_y(g, P.b.y0 - Y0);
            mine = make_gentry(P, X0, Y0, kShapeScale<KID>);
        }
        // the next 64 records load while this batch is walked
        load_rec(recs, it.start + min(base + 64 + lane, last), r0, r1);
        if constexpr (EXT) e = ext[it.start + min(base + 64 + lane, last)];
        gather_walk<KID, NOUT, ACC>(g, s, mine, X0, Y0, o, cc, ga);
    }
    gather_emit<NOUT, ACC>(g, ga, o, X0, Y0, it.slab, slabs, kk.x, kk.y, out0, out1, flags);
}

// ----------------------------------------------------------------------------------
// K5: split tiles -- sum of the item slabs in slab order (deterministic), convert, write.
// Grid (merges, kTilePix / kBlock): each workgroup one 4-row strip of a tile, one pixel
// per thread; the slab loop issues kMergeBatch independent loads per map before summing.
// ----------------------------------------------------------------------------------
constexpr int kMergeBatch = 8;
template <int NOUT, int ACC>
__global__ __launch_bounds__(kBlock) void k_merge(Grid g, const Merge* __restrict__ merges,
                                                  const unsigned long long* __restrict__ slabs,
                                                  const int2* __restrict__ tile_k,
                                                  float* __restrict__ out0,
                                                  float* __restrict__ out1, int flags) {
#if ASP_SCATTER_ABLATE
    return;
#endif
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
// K6: wide particles (footprint over > wide_tiles tiles): they are never binned.  One
// workgroup per tile; every wave streams the wide list 64 particles at a time, prepares
// them (prep_record + clip to the tile) and gathers those meeting its region as K4g does;
// fixed point with the wide particles' own bound.  Adds onto the tile K4/K4g/K5 wrote.
// ----------------------------------------------------------------------------------
template <int KID, int NOUT, int ACC>
__global__ __launch_bounds__(kGatherThreads) void k_wide(
    Grid g, Src64 s, const float* __restrict__ u, const float* __restrict__ v,
    const float* __restrict__ h, const float* __restrict__ a0, const float* __restrict__ a1,
    const int* __restrict__ wide_list, int n_wide, const int* __restrict__ ctr,
    float* __restrict__ out0, float* __restrict__ out1) {
    extern __shared__ __attribute__((aligned(16))) double tot[];
    const int t = blockIdx.x / kGatherRegions;
    const int tx = t / g.nty, ty = t - (t / g.nty) * g.nty;
    const int X0 = tx * kTile, Y0 = ty * kTile;
    const int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    const int k0 = ACC == kAccFix ? scale_exp(n_wide, __uint_as_float((unsigned)ctr[cWideMax0])) : 0;
    const int k1 = (ACC == kAccFix && NOUT == 2)
                       ? scale_exp(n_wide, __uint_as_float((unsigned)ctr[cWideMax1])) : 0;
    const int lane = threadIdx.x;
    const GOwn o = gather_owner(blockIdx.x % kGatherRegions);
    GAcc<NOUT, ACC> ga;
    ga.init(tot);
    const GCorner cc = gather_corners(g, o);
    bool any = false;  // wave-uniform
    for (int c = 0; c < n_wide; c += 64) {
        GEntry mine;
        mine.box = kNoBox;
        const int k = c + lane;
        if (k < n_wide) {
            const int p = wide_list[k];
            Prep P;
            if (prep_record<KID, ACC>(g, s, p, u[p], v[p], h[p], a0[p], NOUT == 2 ? a1[p] : 0.0f,
                                      k0, k1, P) &&
                clip(P.b, X0, Y0, TW, TH)) {
                P.u = (float)(src_u(s, p, P.u) - corner_x(g, X0));  // tile-local frame
                P.v = (float)(src_v(s, p, P.v) - corner_y(g, Y0));
                mine = make_gentry(P, X0, Y0, kShapeScale<KID>);
            }
        }
        any = any || __ballot(mine.box != kNoBox) != 0ull;
        gather_walk<KID, NOUT, ACC>(g, s, mine, X0, Y0, o, cc, ga);
    }
    if (!any) return;
    gather_emit<NOUT, ACC>(g, ga, o, X0, Y0, -1, nullptr, k0, k1, out0, out1, kFlagAccumulate);
}

// ----------------------------------------------------------------------------------
// Diagnostic (bench.py's compute roofline, ASP_COUNT_EVALS=1): the (pixel, particle)
// lane-slots the deposit kernels spend, from the binned records, without evaluating any:
//   K4 small / mid stream: 9 per packed <= 3 x 3 box (every slot of the packed body), the
//      box area for 4 x 4 boxes, 64 per pass of a wave sweep;
//   K4g / K6 gather form: 128 per met 8 x 16 half block row (edge kernels) or 64 per met
//      8 x 8 block (decided path) -- as gather_entry_edge / gather_entry spend them.
// evals[0] += small / mid, evals[1] += gather (records), evals[2] += wide particles.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ long long gather_slots(const Grid& g, int kid, unsigned box, float u,
                                                  float v, float hi) {
    const int x0 = box & 255u, x1 = (box >> 8) & 255u, y0 = (box >> 16) & 255u, y1 = box >> 24;
    const bool edge = kid != kKernelIndicator && !g.nonsquare && !g.mixed;
    long long c = 0;
    for (int w = 0; w < kGatherRegions; ++w) {
        const int r0 = (w >> 1) * 16, c0 = (w & 1) * 32;
        if (edge) {  // the half rows edge_mask lets through (u, v: tile frame)
            GOwn o;
            o.r0 = r0;
            o.c0 = c0;
            o.lr = o.lc = 0;
            c += 128LL * __builtin_popcount(edge_mask(gather_corners(g, o), u, v, hi));
            continue;
        }
        for (int r = 0; r < 2; ++r) {
            const int br = r0 + 8 * r;
            if (!(x0 <= br + 7 && x1 >= br)) continue;
            {
                for (int k = 0; k < 4; ++k) {
                    const int bc = c0 + 8 * k;
                    if (y0 <= bc + 7 && y1 >= bc) c += 64;
                }
            }
        }
    }
    return c;
}

__global__ __launch_bounds__(kBlock) void k_evals(Grid g, int kid, Src64 s,
                                                  const float4* __restrict__ recs,
                                                  const Item* __restrict__ items, int n_items,
                                                  const float* __restrict__ u,
                                                  const float* __restrict__ v,
                                                  const float* __restrict__ h,
                                                  const int* __restrict__ wide_list, int n_wide,
                                                  unsigned long long* __restrict__ evals) {
    long long c0 = 0, c1 = 0, c2 = 0;
    if ((int)blockIdx.x < n_items) {
        const Item it = items[blockIdx.x];
        const int tx = it.tile / g.nty, ty = it.tile - (it.tile / g.nty) * g.nty;
        const int X0 = tx * kTile, Y0 = ty * kTile;
        for (int i = threadIdx.x; i < it.count; i += kBlock) {
            float4 r0, r1;
            load_rec(recs, it.start + i, r0, r1);
            Prep P;
            rec_prep<kAccF64>(r0, r1, X0, Y0, make_int2(0, 0), P);
            const int bw = P.b.x1 - P.b.x0 + 1, bh = P.b.y1 - P.b.y0 + 1;
            if (bw <= 0) continue;  // an empty box
            if (it.mode == 1) {
                c1 += gather_slots(g, kid, __float_as_uint(r1.w),
                                   P.u + corner_off_x(g, P.b.x0 - X0),
                                   P.v + corner_off_y(g, P.b.y0 - Y0), P.hi);
            } else if (bw <= 3 && bh <= 3) {
                c0 += 9;
            } else if (is_small(bw, bh)) {
                c0 += bw * bh;
            } else {
                const int passes = bh <= 64 ? (bw + 64 / bh - 1) / (64 / bh) : bw * ((bh + 63) / 64);
                c0 += 64LL * passes;
            }
        }
    } else {  // one workgroup per tile: the wide particles the tile's K6 gathers
        const int t = blockIdx.x - n_items;
        const int tx = t / g.nty, ty = t - (t / g.nty) * g.nty;
        const int X0 = tx * kTile, Y0 = ty * kTile;
        const int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
        for (int i = threadIdx.x; i < n_wide; i += kBlock) {
            const int p = wide_list[i];
            Prep P;
            if (prep_record<2>(g, s, p, u[p], v[p], h[p], 0.0f, 0.0f, 0, 0, P) &&
                clip(P.b, X0, Y0, TW, TH)) {
                const unsigned box = (unsigned)(P.b.x0 - X0) | ((unsigned)(P.b.x1 - X0) << 8) |
                                     ((unsigned)(P.b.y0 - Y0) << 16) | ((unsigned)(P.b.y1 - Y0) << 24);
                c2 += gather_slots(g, kid, box, (float)(src_u(s, p, P.u) - corner_x(g, X0)),
                                   (float)(src_v(s, p, P.v) - corner_y(g, Y0)), P.hi);
            }
        }
    }
    if (c0) atomicAdd(&evals[0], (unsigned long long)c0);
    if (c1) atomicAdd(&evals[1], (unsigned long long)c1);
    if (c2) atomicAdd(&evals[2], (unsigned long long)c2);
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
// K8 pairs (the kernel_func plugin: _projector.py:26, 86; _pixel_calculations.pyx:30-33),
// one workgroup per GPU tile of a binned window, on the records the session keeps
// resident.  Every included (pixel, particle) pair -- the deposit's exact decision -- is
//   MODE 0: counted per pixel (int32 pixcnt[tile][lx * 64 + ly], int64 tile totals);
//   MODE 1: written as the particle index and the reference's fp64 r^2 = dx^2 + dy^2
//           (dx = U - X, .pyx:13-14, :20-30) at its pixel's slot range, the pixel offsets
//           being the tile base + an exclusive scan of that tile's pixcnt (also written
//           out for the host).  Order within a pixel unspecified.
// The counts come from the same records and decisions as the pairs, so a pixel's slots
// always suffice; a pair that would not fit (a broken invariant) is dropped and counted in
// *overflow, which the host turns into an error.
// ----------------------------------------------------------------------------------
constexpr int kPairsBlock = 256;
template <int MODE>
__global__ __launch_bounds__(kPairsBlock) void k_pairs(
    Grid g, Src64 s, const float4* __restrict__ recs, const long long* __restrict__ tile_start,
    const int* __restrict__ tile_total, const int* __restrict__ wide_list, int n_wide,
    const float* __restrict__ u, const float* __restrict__ v, const float* __restrict__ h,
    int t0, int* __restrict__ pixcnt, long long* __restrict__ tile_pairs,
    const long long* __restrict__ tile_base, long long* __restrict__ offsets,
    int* __restrict__ particle, double* __restrict__ r2out, int* __restrict__ overflow) {
    __shared__ int cur[kTilePix];
    __shared__ float xt[kTile], yt[kTile];
    __shared__ long long wsum[kPairsBlock / 64];
    __shared__ long long soff[MODE == 1 ? kTilePix + 1 : 1];  // MODE 1: the pixel offsets
    const int t = t0 + blockIdx.x;
    const int tx = t / g.nty, ty = t - (t / g.nty) * g.nty;
    const int X0 = tx * kTile, Y0 = ty * kTile;
    const int TW = min(kTile, g.nx - X0), TH = min(kTile, g.ny - Y0);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int kPer = kTilePix / kPairsBlock;  // 16 consecutive pixels per thread
    long long* off = offsets + (long long)blockIdx.x * kTilePix;  // MODE 1
    if constexpr (MODE == 1) {
        // exclusive scan of the tile's pixel counts + the tile's base: the pixel offsets
        const int* c = pixcnt + (long long)t * kTilePix + threadIdx.x * kPer;
        long long loc[kPer], run = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            loc[k] = run;
            run += c[k];
        }
        long long x = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            long long y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        long long base = tile_base[blockIdx.x] + x - run;
        for (int k = 0; k < wv; ++k) base += wsum[k];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            soff[threadIdx.x * kPer + k] = base + loc[k];
            off[threadIdx.x * kPer + k] = base + loc[k];
        }
        if (threadIdx.x == kPairsBlock - 1) {  // = the next tile's base
            soff[kTilePix] = base + run;
            off[kTilePix] = base + run;
        }
    }
    for (int k = threadIdx.x; k < kTilePix; k += kPairsBlock) cur[k] = 0;
    corner_tables(g, X0, Y0, xt, yt);
    __syncthreads();
    auto emit_box = [&](const Prep& P) {  // P in its box-origin frame
        for (int xi = P.b.x0; xi <= P.b.x1; ++xi)
            for (int yi = P.b.y0; yi <= P.b.y1; ++yi) {
                float r2f;
                if (!decide(g, s, P, xi, yi, xt[xi - P.b.x0], yt[yi - P.b.y0], r2f)) continue;
                const int lp = (xi - X0) * kTile + (yi - Y0);
                const int k = atomicAdd(&cur[lp], 1);
                if constexpr (MODE == 1) {
                    const long long slot = soff[lp] + k;
                    if (slot >= soff[lp + 1]) {
                        atomicAdd(overflow, 1);
                        continue;
                    }
                    const Vals x = src_values(g, s, P.p);
                    const double dx = x.U - corner_x(g, xi), dy = x.V - corner_y(g, yi);
                    particle[slot] = P.p;
                    r2out[slot] = dx * dx + dy * dy;
                }
            }
    };
    for (int stream = 0; stream < 2; ++stream) {
        const long long st0 = tile_start[t + stream * g.ntiles];
        const int cnt = tile_total[t + stream * g.ntiles];
        for (int i = threadIdx.x; i < cnt; i += kPairsBlock) {
            float4 r0, r1;
            load_rec(recs, st0 + i, r0, r1);
            Prep P;
            rec_prep<kAccF64>(r0, r1, X0, Y0, make_int2(0, 0), P);
            emit_box(P);
        }
    }
    for (int i = threadIdx.x; i < n_wide; i += kPairsBlock) {
        const int p = wide_list[i];
        Prep P;
        if (!prep_record<2>(g, s, p, u[p], v[p], h[p], 0.0f, 0.0f, 0, 0, P) ||
            !clip(P.b, X0, Y0, TW, TH))
            continue;
        P.u = (float)(src_u(s, p, P.u) - corner_x(g, P.b.x0));  // box-origin frame
        P.v = (float)(src_v(s, p, P.v) - corner_y(g, P.b.y0));
        emit_box(P);
    }
    if constexpr (MODE == 0) {
        __syncthreads();
        long long tot = 0;
        for (int k = threadIdx.x; k < kTilePix; k += kPairsBlock) {
            pixcnt[(long long)t * kTilePix + k] = cur[k];
            tot += cur[k];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0) wsum[wv] = tot;
        __syncthreads();
        if (threadIdx.x == 0) {
            long long a = 0;
            for (int k = 0; k < kPairsBlock / 64; ++k) a += wsum[k];
            tile_pairs[t] = a;
        }
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
__global__ __launch_bounds__(kBlock) void k_neighbours(Grid g, Src64 s, const float* __restrict__ u,
                                                       const float* __restrict__ v,
                                                       const float* __restrict__ h, long long n,
                                                       const long long* __restrict__ pixels,
                                                       long long* __restrict__ counts,
                                                       const long long* __restrict__ offsets,
                                                       int* __restrict__ index, long long cap,
                                                       int pass) {
    __shared__ int wsum[kBlock / 64];
    __shared__ long long run;
    long long px = pixels[blockIdx.x];
    int xi = (int)(px / g.ny), yi = (int)(px - (px / g.ny) * g.ny);
    float X = (float)corner_x(g, xi), Y = (float)corner_y(g, yi);
    if (threadIdx.x == 0) run = pass ? offsets[blockIdx.x] : 0;
    __syncthreads();
    int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (long long base = 0; base < n; base += kBlock) {
        long long p = base + threadIdx.x;
        bool in = false;
        if (p < n) {
            Prep P;
            if (prep_record<2>(g, s, (int)p, u[p], v[p], h[p], 0.0f, 0.0f, 0, 0, P) &&
                xi >= P.b.x0 && xi <= P.b.x1 && yi >= P.b.y0 && yi <= P.b.y1) {
                float r2;
                in = decide(g, s, P, xi, yi, X, Y, r2);
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

bool make_grid(double x_min, double x_max, double y_min, double y_max, int nx, int ny, int cs,
               Grid& g) {
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
    // |corner| over the grid (absolute frame); 2x the tile span (the records' frames)
    const double mgl = 2.0 * kTile * std::max(g.psx, g.psy_pix);
    double mg = std::max({std::fabs(x_min), std::fabs(x_min + nx * g.psx), std::fabs(y_min),
                          std::fabs(y_min + ny * g.psy_pix), mgl});
    g.mg = (float)(mg * (1.0 + 1e-6));
    g.mgl = (float)(mgl * (1.0 + 1e-6));
    g.nx = nx;
    g.gnx = nx;
    g.ox = 0;
    g.ny = ny;
    g.cs = cs;
    g.ncx = (nx + cs - 1) / cs;
    g.ncy = (ny + cs - 1) / cs;
    g.ntx = (nx + kTile - 1) / kTile;
    g.nty = (ny + kTile - 1) / kTile;
    g.ntiles = g.ntx * g.nty;
    g.nonsquare = nx != ny;
    g.mixed = 0;
    g.wide_tiles = kWideTilesDefault;
    g.gather_min = kGatherMinDefault;
    g.gather_area = kGatherAreaDefault;
    return true;
}

constexpr int kMaxBinBlocks = 1024;  // count workgroups (hist rows)
constexpr int kMaxTiles = 4096;  // K1/K3 LDS: cursors + per-tile max (12 B/tile at 2 maps)
static_assert(kMaxTiles <= kScanThreads * 4, "k_tilescan holds <= 4 tiles per thread");

// Images of more than kMaxTiles GPU tiles are projected as WINDOWS of whole tile rows
// (image rows [ox, ox + nx) x all columns; kMaxTiles / nty tile rows each): every window
// is one pass of the pipeline over all particles with the footprints clipped to it, and
// its map is a contiguous part of the (nx, ny) C-order output.  Pixel corners, pitches
// and the chunk cull stay those of the whole image (Grid::gnx, Grid::ox), so every
// decision is the one-window decision.
static inline int window_rows(const Grid& full) {  // tile rows per window
    return std::max(1, std::min(full.ntx, kMaxTiles / full.nty));
}
// Image rows [r0, r1) as a window (any r0: its tile grid starts at row r0).
static inline Grid window_grid_rows(const Grid& full, int r0, int r1) {
    Grid g = full;
    g.ox = r0;
    g.nx = r1 - r0;
    g.ntx = (g.nx + kTile - 1) / kTile;
    g.ntiles = g.ntx * g.nty;
    return g;
}
static inline Grid window_grid(const Grid& full, int tx0, int tx1) {  // whole tile rows
    return window_grid_rows(full, tx0 * kTile, std::min(tx1 * kTile, full.gnx));
}

struct Plan {
    long long n, nblk;  // particles, count workgroups
    long long nblk_s;   // scatter workgroups (grp count workgroups each)
    int grp;
    int n_items, n_merges, n_slabs, n_wide;
    long long n_recs, n_large;  // records; of them in the large stream
};

// items / merges in the work-list buffers
// Deposit items in tilescan order (ASP_ITEM_ORDER=0, an A/B switch) instead of largest first.
// The split tile scan pays when maps run one after another on one stream (the side
// kernel runs beside this map's scatter, a free CU slot away).  With maps on two streams
// (two workspace slots in use) the device is already full of the other map's work: the
// side kernel, and the host's wait for the counters behind it, start late and the
// two-stream overlap loses more than the split saves (1.25e7 share: 0.592 vs 0.540 ms), so
// the one-launch scan is used there.  ASP_SPLIT_SCAN=0 / 1 forces either (read per call).
static bool split_scan_on() {
    if (const char* e = getenv("ASP_SPLIT_SCAN")) return atoi(e) != 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    SlotTable& T = g_slots[dev];
    std::lock_guard<std::mutex> lock(T.mu);
    for (int k = 1; k < kMapSlots; ++k)
        if (T.used[k]) return false;
    return true;
}

static int item_order_identity() {
    static const int identity = [] {
        const char* e = getenv("ASP_ITEM_ORDER");
        return e && atoi(e) == 0 ? 1 : 0;
    }();
    return identity;
}
// deposit work items per map (ASP_ITEMS overrides kTargetItems2d; tuning only)
static inline int item_target() {
    static const int t = getenv("ASP_ITEMS") ? std::max(64, atoi(getenv("ASP_ITEMS"))) : kTargetItems2d;
    return t;
}
static inline size_t item_cap(const Grid& g) { return (size_t)2 * g.ntiles + item_target() + kTargetItems1 + 16; }
static inline size_t merge_cap(const Grid& g) { return (size_t)g.ntiles + 16; }

static inline size_t scatter_lds_base(const Grid& g) {
    return (size_t)2 * g.ntiles * sizeof(int) + (size_t)(kScatterBlock / 64) * kStageF4 * sizeof(float4);
}
static inline size_t scatter_lds(const Grid& g, int nout, bool det) {
    return scatter_lds_base(g) + (det ? (size_t)g.ntiles * nout * sizeof(unsigned) : 0);
}

// K3 on stream st.  rec_cap / wide_cap: the capacities the kernel checks against the
// device counters (speculative launch; see project2d).
template <int KID, int NOUT, int ACC, bool CULL, int SRC, int PROBE, int NX>
static int scatter_variant(const Grid& g, const Src64& s, Workspace& ws, const Plan& pl,
                           const float* u, const float* v, const float* h, const float* a0,
                           const float* a1, long long rec_cap, int wide_cap, hipStream_t st,
                           const XArgs& xa) {
    int* dc = (int*)ws.counters.p;
    const size_t lds = scatter_lds(g, NOUT, ACC == kAccFix);
    hipLaunchKernelGGL((k_scatter<KID, NOUT, ACC, CULL, SRC, PROBE, NX>), dim3((unsigned)pl.nblk_s),
                       dim3(kScatterBlock), lds, st, u, v, h, a0,
                       a1, pl.n, pl.nblk, g, s, (const int*)ws.hist.p,
                       (const long long*)ws.tile_start.p, (const int*)ws.tile_total.p,
                       (float4*)ws.recs.p, (unsigned*)ws.cmx.p, (int*)ws.wide.p, dc, pl.grp,
                       rec_cap, wide_cap, xa);
    ASP_LAUNCHED();
    return ASP_OK;
}

// xa (asp_project2d_props): also write every record's coefficients of properties 2..5
// (two-map fp64 calls only).
template <int KID, int NOUT, int ACC>
static int launch_scatter(const Grid& g, const Src64& s, Workspace& ws, const Plan& pl,
                          const float* u, const float* v, const float* h, const float* a0,
                          const float* a1, long long rec_cap, int wide_cap, hipStream_t st,
                          bool probe = false, const XArgs* xa = nullptr) {
    StageMark m(ws, kSScatter, st);
    const XArgs none{};
    int rc;
#define ASP_SV(C, S, P, X) scatter_variant<KID, NOUT, ACC, C, S, P, X>(g, s, ws, pl, u, v, h, a0, a1, rec_cap, wide_cap, st, X ? *xa : none)
    if constexpr (NOUT == 2 && ACC == kAccF64) {
        if (xa) {
            if (g.nonsquare || g.mixed) rc = ASP_SV(true, 2, 0, 1);
            else if (s.u64) rc = ASP_SV(false, 1, 0, 1);
            else rc = ASP_SV(false, 0, 0, 1);
            ASP_TRY(rc);
            m.done();
            return ASP_OK;
        }
    }
    if (g.nonsquare || g.mixed) rc = probe ? ASP_SV(true, 2, 1, 0) : ASP_SV(true, 2, 0, 0);
    else if (s.u64) rc = probe ? ASP_SV(false, 1, 1, 0) : ASP_SV(false, 1, 0, 0);
    else rc = probe ? ASP_SV(false, 0, 1, 0) : ASP_SV(false, 0, 0, 0);
#undef ASP_SV
    ASP_TRY(rc);
    m.done();
    return ASP_OK;
}

// K3..K7 for one kernel / map count, on the caller's stream.
template <int KID, int NOUT, int ACC>
static int run_tail(const Grid& g, const Src64& s, Workspace& ws, const Plan& pl, const float* u,
                    const float* v, const float* h, const float* a0, const float* a1, float* o0,
                    float* o1, int flags, hipStream_t st, bool pre_scattered,
                    const XArgs* xa = nullptr) {
    int* dc = (int*)ws.counters.p;
    const bool ratio = (flags & ASP_F_RATIO) != 0;
    const bool fuse_ratio = ratio && pl.n_wide == 0;
    const unsigned long long* slabs = (const unsigned long long*)ws.slabs.p;
    const int dflags = ((flags & ASP_F_ACCUMULATE) ? kFlagAccumulate : 0) |
                       (fuse_ratio ? kFlagRatio : 0);
    if (!pre_scattered)
        ASP_TRY((launch_scatter<KID, NOUT, ACC>(g, s, ws, pl, u, v, h, a0, a1, 0x7fffffffLL,
                                                0x7fffffff, st, false, xa)));
    if (ACC == kAccFix) {
        StageMark m(ws, kSScale, st);
        hipLaunchKernelGGL((k_tilescale<NOUT>), dim3((g.ntiles + 63) / 64), dim3(kBlock), 0, st,
                           (const unsigned*)ws.cmx.p, (int)pl.nblk_s, g.ntiles,
                           (const int*)ws.tile_total.p, (int2*)ws.tile_k.p);
        ASP_LAUNCHED();
        m.done();
    }
    {
        StageMark m(ws, kSDeposit, st);
        const size_t lds = deposit_lds<NOUT>();
        ASP_TRY(allow_dyn_lds((const void*)k_deposit<KID, NOUT, ACC>, lds));
        hipLaunchKernelGGL((k_deposit<KID, NOUT, ACC>), dim3(pl.n_items), dim3(kDepBlock), lds, st, g, s, (const float4*)ws.recs.p,
                           (const Item*)ws.items.p, (const int*)ws.iorder.p, (const int2*)ws.tile_k.p,
                           (unsigned long long*)ws.slabs.p, o0, o1, dflags, (const float4*)nullptr, 0);
        ASP_LAUNCHED();
        m.done();
    }
    if (pl.n_large > 0) {
        StageMark m(ws, kSGather, st);
        const size_t lds = gather_lds<NOUT, ACC>();
        hipLaunchKernelGGL((k_gather<KID, NOUT, ACC>), dim3(pl.n_items * kGatherRegions),
                           dim3(kGatherThreads), lds, st, g,
                           s, (const float4*)ws.recs.p, (const Item*)ws.items.p,
                           (const int*)ws.iorder.p, (const int2*)ws.tile_k.p,
                           (unsigned long long*)ws.slabs.p, o0, o1, dflags, (const float4*)nullptr, 0);
        ASP_LAUNCHED();
        m.done();
    }
    if (pl.n_merges > 0) {
        StageMark m(ws, kSMerge, st);
        hipLaunchKernelGGL((k_merge<NOUT, ACC>), dim3(pl.n_merges, kTilePix / kBlock), dim3(kBlock),
                           0, st, g, (const Merge*)ws.merges.p, slabs, (const int2*)ws.tile_k.p,
                           o0, o1, dflags);
        ASP_LAUNCHED();
        m.done();
    }
    if (pl.n_wide > 0) {
        StageMark m(ws, kSWide, st);
        const size_t lds = gather_lds<NOUT, ACC>();
        hipLaunchKernelGGL((k_wide<KID, NOUT, ACC>), dim3(g.ntiles * kGatherRegions),
                           dim3(kGatherThreads), lds, st, g, s,
                           u, v, h, a0, a1, (const int*)ws.wide.p, pl.n_wide, (const int*)dc, o0,
                           o1);
        ASP_LAUNCHED();
        m.done();
    }
    if (ratio && !fuse_ratio) {
        long long npix = (long long)g.nx * g.ny;
        long long blocks = std::min<long long>((npix + kBlock - 1) / kBlock, 8192);
        StageMark m(ws, kSRatio, st);
        hipLaunchKernelGGL(k_ratio, dim3((unsigned)std::max<long long>(1, blocks)), dim3(kBlock),
                           0, st, o0, (const float*)o1, npix);
        ASP_LAUNCHED();
        m.done();
    }
    return ASP_OK;
}

// asp_project2d_props, pass p = 1, 2: properties (2p, 2p + 1) deposited from the records
// the pass-0 map binned and their ext coefficients (K4 / K4g / K5 / K6 as in run_tail, fp64
// accumulation, no ratio) into o0 (, o1; NOUT = 1 for an odd last property).  xa0 / xa1:
// the properties' fp32 arrays (the wide particles read them directly).
template <int KID, int NOUT>
static int run_ext_pass(const Grid& g, const Src64& s, Workspace& ws, const Plan& pl,
                        const float* u, const float* v, const float* h, const float* xa0,
                        const float* xa1, float* o0, float* o1, int flags, hipStream_t st,
                        int pass) {
    int* dc = (int*)ws.counters.p;
    const unsigned long long* slabs = (const unsigned long long*)ws.slabs.p;
    const int dflags = (flags & ASP_F_ACCUMULATE) ? kFlagAccumulate : 0;
    const float4* ext = (const float4*)ws.ext.p;
    {
        StageMark m(ws, kSDeposit, st);
        ASP_TRY(allow_dyn_lds((const void*)k_deposit<KID, NOUT, kAccF64, 1>, deposit_lds<NOUT>()));
        hipLaunchKernelGGL((k_deposit<KID, NOUT, kAccF64, 1>), dim3(pl.n_items), dim3(kDepBlock),
                           deposit_lds<NOUT>(), st, g, s, (const float4*)ws.recs.p,
                           (const Item*)ws.items.p, (const int*)ws.iorder.p,
                           (const int2*)ws.tile_k.p, (unsigned long long*)ws.slabs.p, o0, o1,
                           dflags, ext, pass);
        ASP_LAUNCHED();
        m.done();
    }
    if (pl.n_large > 0) {
        StageMark m(ws, kSGather, st);
        hipLaunchKernelGGL((k_gather<KID, NOUT, kAccF64, 1>), dim3(pl.n_items * kGatherRegions),
                           dim3(kGatherThreads), (gather_lds<NOUT, kAccF64>()), st, g, s,
                           (const float4*)ws.recs.p, (const Item*)ws.items.p,
                           (const int*)ws.iorder.p, (const int2*)ws.tile_k.p,
                           (unsigned long long*)ws.slabs.p, o0, o1, dflags, ext, pass);
        ASP_LAUNCHED();
        m.done();
    }
    if (pl.n_merges > 0) {
        StageMark m(ws, kSMerge, st);
        hipLaunchKernelGGL((k_merge<NOUT, kAccF64>), dim3(pl.n_merges, kTilePix / kBlock),
                           dim3(kBlock), 0, st, g, (const Merge*)ws.merges.p, slabs,
                           (const int2*)ws.tile_k.p, o0, o1, dflags);
        ASP_LAUNCHED();
        m.done();
    }
    if (pl.n_wide > 0) {
        StageMark m(ws, kSWide, st);
        hipLaunchKernelGGL((k_wide<KID, NOUT, kAccF64>), dim3(g.ntiles * kGatherRegions),
                           dim3(kGatherThreads), (gather_lds<NOUT, kAccF64>()), st, g, s, u, v, h,
                           xa0, xa1, (const int*)ws.wide.p, pl.n_wide, (const int*)dc, o0, o1);
        ASP_LAUNCHED();
        m.done();
    }
    return ASP_OK;
}

// Tunables read once per call (experiments; the defaults are the measured choices).
static void grid_tunables(Grid& g) {
    if (const char* e = getenv("ASP_WIDE_TILES")) g.wide_tiles = std::max(1, atoi(e));
    if (const char* e = getenv("ASP_GATHER_MIN")) g.gather_min = std::max(2, atoi(e));
    if (const char* e = getenv("ASP_GATHER_AREA")) g.gather_area = std::max(4, atoi(e));
}

// The projection on DEVICE arrays (fp32 working copies u, v, h, a0, a1; s: the caller's
// fp64 arrays for exact re-decisions, or none) into DEVICE outputs, on stream st.  The
// caller holds the workspace lock and has ordered st behind the previous call.
// bin_only (the kernel_func plug-in session): stop after the scatter -- the records stay in
// ws for k_pairs -- and return the number of wide particles there.
constexpr int kRetSplit = 1;  // internal: >= 2^31 records in one pass, nothing written

// xa / nxp / xo (asp_project2d_props): nxp (1..4) further properties xa->a[0 ..] binned
// with the first two (their coefficients beside each record) and deposited in further
// passes into xo[0 ..] (two-map fp64 calls only).
int project2d_device(Workspace& ws, const Grid& gin, const Src64& s, const float* du,
                     const float* dv, const float* dh, const float* da0, const float* da1,
                     long long n, int kid, int flags, float* d0, float* d1, hipStream_t st,
                     int* bin_only = nullptr, const XArgs* xa = nullptr, int nxp = 0,
                     float* const* xo = nullptr) {
    Grid g = gin;
    const int nout = d1 ? 2 : 1;
    const long long npix = (long long)g.nx * g.ny;
    if (ws.prof) ASP_TRY(prof_next(ws));
    Plan pl{};
    pl.n = n;
    if (n == 0) {  // all-zero map(s) (the ratio map of 0 / 0 is 0 as well)
        if (bin_only) {
            *bin_only = 0;
            return ASP_OK;
        }
        if (!(flags & ASP_F_ACCUMULATE)) {
            StageMark m(ws, kSMemset, st);
            ASP_HIP(hipMemsetAsync(d0, 0, npix * sizeof(float), st));
            if (d1) ASP_HIP(hipMemsetAsync(d1, 0, npix * sizeof(float), st));
            for (int j = 0; j < nxp; ++j) ASP_HIP(hipMemsetAsync(xo[j], 0, npix * sizeof(float), st));
            m.done();
        }
        for (long long& x : ws.stats) x = 0;
        return ASP_OK;
    }
    ASP_TRY(ensure_morton(ws, g.ntx, g.nty, st));
    long long max_blk = kMaxBinBlocks;
    if (const char* e = getenv("ASP_BIN_BLOCKS")) max_blk = std::max(1, atoi(e));
    pl.nblk = std::min<long long>(max_blk, std::max<long long>(1, (n + 8191) / 8192));
    pl.grp = kScatterGroup;
    if (const char* e = getenv("ASP_SCATTER_GROUP")) pl.grp = std::max(1, atoi(e));
    pl.nblk_s = (pl.nblk + pl.grp - 1) / pl.grp;
    const bool det = (flags & ASP_F_DETERMINISTIC) != 0;
    ASP_TRY(ensure(ws.hist, (size_t)pl.nblk * 2 * g.ntiles * sizeof(int)));
    if (det) ASP_TRY(ensure(ws.cmx, (size_t)pl.nblk_s * g.ntiles * nout * sizeof(unsigned)));
    ASP_TRY(ensure(ws.tile_total, (size_t)2 * g.ntiles * sizeof(int)));
    ASP_TRY(ensure(ws.tile_start, (size_t)2 * g.ntiles * sizeof(long long)));
    ASP_TRY(ensure(ws.tile_k, (size_t)g.ntiles * sizeof(int2)));
    ASP_TRY(ensure(ws.items, item_cap(g) * sizeof(Item)));
    ASP_TRY(ensure(ws.iorder, item_cap(g) * sizeof(int)));  // deposit order (k_tilescan)
    ASP_TRY(ensure(ws.merges, merge_cap(g) * sizeof(Merge)));
    ASP_TRY(ensure(ws.counters, (size_t)cNum * sizeof(int)));
    if (!ws.h_counters) ASP_HIP(hipHostMalloc((void**)&ws.h_counters, kMarks * cNum * sizeof(int)));
    int* dc = (int*)ws.counters.p;
    ASP_HIP(hipMemsetAsync(dc, 0, (size_t)cNum * sizeof(int), st));
    {
        StageMark m(ws, kSCount, st);
        hipLaunchKernelGGL(g.nonsquare || g.mixed ? k_count<true> : k_count<false>,
                           dim3((unsigned)pl.nblk), dim3(kCountBlock),
                           (size_t)2 * g.ntiles * sizeof(int), st, du, dv, dh, n, pl.nblk, g, s,
                           (int*)ws.hist.p, dc);
        ASP_LAUNCHED();
        m.done();
    }
    {
        StageMark m(ws, kSColscan, st);
        hipLaunchKernelGGL(k_colscan, dim3((2 * g.ntiles + 63) / 64, 1), dim3(kColscanBlock), 0,
                           st, (int*)ws.hist.p, (int)pl.nblk, 2 * g.ntiles,
                           (int*)ws.tile_total.p, (int)pl.nblk);
        ASP_LAUNCHED();
        m.done();
    }
    // The tile scan in two parts (round 6, ASP_SPLIT_SCAN=0: one launch): the tile starts
    // the scatter needs, on st; the work items, merge list and dispatch order the deposit
    // needs, on the side stream beside the scatter (a one-workgroup kernel off the critical
    // path).
    const bool split = split_scan_on();
    {
        StageMark m(ws, kSTilescan, st);
        if (split)
            hipLaunchKernelGGL((k_tilescan<4, 1>), dim3(1), dim3(kScanThreads), 0, st,
                               (const int*)ws.tile_total.p, (const int*)ws.morton.p, g.ntiles, 2,
                               (long long*)ws.tile_start.p, (Item*)ws.items.p, (Merge*)ws.merges.p,
                               dc, (int*)ws.iorder.p, item_order_identity(), item_target());
        else
            hipLaunchKernelGGL((k_tilescan<4>), dim3(1), dim3(kScanThreads), 0, st,
                               (const int*)ws.tile_total.p, (const int*)ws.morton.p, g.ntiles, 2,
                               (long long*)ws.tile_start.p, (Item*)ws.items.p, (Merge*)ws.merges.p,
                               dc, (int*)ws.iorder.p, item_order_identity(), item_target());
        ASP_LAUNCHED();
        m.done();
    }
    // One small read-back sizes the record / slab buffers.  With buffers
    // left by an earlier call, the scatter is enqueued BEFORE the host waits for it
    // (speculatively: it checks the counters against those capacities itself), so the
    // GPU does not idle across the host round trip.  The copy runs on the side stream, so
    // the scatter behind it on st need not wait for the copy's own latency.
    ASP_TRY(ensure_side(ws));
    ASP_HIP(hipEventRecord(ws.scan_ev, st));
    int gate_dev = -1;  // ASP_SCATTER_GATE: this map's scatter after the last map's deposit
    if (scatter_gate_on() && hipGetDevice(&gate_dev) == hipSuccess) ASP_TRY(gate_wait(gate_dev, st));
    ASP_HIP(hipStreamWaitEvent(ws.side, ws.scan_ev, 0));
    if (split) {
        hipLaunchKernelGGL((k_tilescan<4, 2>), dim3(1), dim3(kScanThreads), 0, ws.side,
                           (const int*)ws.tile_total.p, (const int*)ws.morton.p, g.ntiles, 2,
                           (long long*)ws.tile_start.p, (Item*)ws.items.p, (Merge*)ws.merges.p,
                           dc, (int*)ws.iorder.p, item_order_identity(), item_target());
        ASP_LAUNCHED();
    }
    ASP_HIP(hipMemcpyAsync(ws.h_counters, dc, (size_t)cNum * sizeof(int), hipMemcpyDeviceToHost,
                           ws.side));
    ASP_HIP(hipEventRecord(ws.cnt_ev, ws.side));
    // < 2^31 - 1: the tilescan's clamped record count always exceeds it when it overflows
    const long long rec_cap = (long long)std::min<size_t>(ws.recs.cap / (2 * sizeof(float4)), 0x7ffffffe);
    const int wide_cap = (int)std::min<size_t>(ws.wide.cap / sizeof(int), 0x7fffffff);
    const bool spec = ws.recs.p && ws.wide.p && !xa && getenv("ASP_NO_SPECULATE") == nullptr;
    if (spec) {
#define ASP_SC(K, N, A) \
    launch_scatter<K, N, A>(g, s, ws, pl, du, dv, dh, da0, da1, rec_cap, wide_cap, st)
#define ASP_SC2(K, A) (nout == 1 ? ASP_SC(K, 1, A) : ASP_SC(K, 2, A))
#define ASP_SC3(A) (kid == 0 ? ASP_SC2(0, A) : kid == 1 ? ASP_SC2(1, A) : ASP_SC2(2, A))
        ASP_TRY(det ? ASP_SC3(kAccFix) : ASP_SC3(kAccF64));
#undef ASP_SC3
#undef ASP_SC2
#undef ASP_SC
    }
    ASP_HIP(hipEventSynchronize(ws.cnt_ev));
    if (split) ASP_HIP(hipStreamWaitEvent(st, ws.cnt_ev, 0));  // the deposit reads part 2's output
    const int* hc = ws.h_counters;
    pl.n_recs = hc[cRecs];
    pl.n_items = hc[cItems];
    pl.n_merges = hc[cMerges];
    pl.n_slabs = hc[cSlabs];
    pl.n_wide = hc[cWideCount];
    pl.n_large = hc[cLarge];
    long long rec_limit = 0x7fffffffLL;  // 32-bit record cursors (ASP_MAX_RECORDS: tests)
    if (const char* e = getenv("ASP_MAX_RECORDS")) rec_limit = std::max(1LL, atoll(e));
    if (pl.n_recs >= rec_limit) {  // nothing written yet: the caller splits the batch
        if (spec) ASP_HIP(hipStreamSynchronize(st));  // its (no-op) scatter is done
        return kRetSplit;
    }
    const bool pre = spec && pl.n_recs <= rec_cap && pl.n_wide <= wide_cap;
    if (spec && !pre) ASP_HIP(hipStreamSynchronize(st));  // its (no-op) scatter is done
    const void* recs_before = ws.recs.p;
    ASP_TRY(ensure(ws.recs, (size_t)pl.n_recs * 2 * sizeof(float4)));
    ASP_TRY(ensure(ws.wide, (size_t)pl.n_wide * sizeof(int)));
    ASP_TRY(ensure(ws.slabs, (size_t)pl.n_slabs * nout * kTilePix * sizeof(long long)));
    XArgs xw{};
    if (xa) {  // the extra properties' coefficient array, one float4 per record
        ASP_TRY(ensure(ws.ext, (size_t)std::max(pl.n_recs, 1LL) * sizeof(float4)));
        xw = *xa;
        xw.ext = (float4*)ws.ext.p;
    }
    bool placed = false;  // the records are already scattered (by the placement trials)
    int ntrials = 0;      // scatter runs of the placement trials
    if (!bin_only && !xa && !pre && ws.recs.p != recs_before) {
#define ASP_SC(K, N, A) \
    launch_scatter<K, N, A>(g, s, ws, pl, du, dv, dh, da0, da1, 0x7fffffffLL, 0x7fffffff, st, true)
#define ASP_SC2(K, A) (nout == 1 ? ASP_SC(K, 1, A) : ASP_SC(K, 2, A))
#define ASP_SC3(A) (kid == 0 ? ASP_SC2(0, A) : kid == 1 ? ASP_SC2(1, A) : ASP_SC2(2, A))
        auto scatter = [&]() -> int {
            // the wide-list cursor is the one counter the scatter advances
            ASP_HIP(hipMemsetAsync(dc + cWideCursor, 0, sizeof(int), st));
            return det ? ASP_SC3(kAccFix) : ASP_SC3(kAccF64);
        };
#undef ASP_SC3
#undef ASP_SC2
#undef ASP_SC
        ASP_TRY(place_records(ws, (size_t)pl.n_recs * 2 * sizeof(float4), st, scatter, placed,
                              &ntrials));
    }
    const bool pre_all = pre || placed;
    if (bin_only) {  // the plugin session: the records, for k_pairs
        if (!pre)
            ASP_TRY((launch_scatter<2, 1, kAccF64>(g, s, ws, pl, du, dv, dh, da0, da1, 0x7fffffffLL,
                                                   0x7fffffff, st)));
        *bin_only = pl.n_wide;
        return ASP_OK;
    }
    int rc;
    const XArgs* xp = xa ? &xw : nullptr;
#define ASP_TAIL(K, N, A) \
    run_tail<K, N, A>(g, s, ws, pl, du, dv, dh, da0, da1, d0, d1, flags, st, pre_all, xp)
#define ASP_TAIL2(K, A) (nout == 1 ? ASP_TAIL(K, 1, A) : ASP_TAIL(K, 2, A))
#define ASP_TAIL3(A) (kid == 0 ? ASP_TAIL2(0, A) : kid == 1 ? ASP_TAIL2(1, A) : ASP_TAIL2(2, A))
    rc = det ? ASP_TAIL3(kAccFix) : ASP_TAIL3(kAccF64);
#undef ASP_TAIL3
#undef ASP_TAIL2
#undef ASP_TAIL
    if (rc != ASP_OK) return rc;
    for (int pass = 1; xa && 2 * (pass - 1) < nxp; ++pass) {  // properties 2.. from the records
        const int j = 2 * (pass - 1);
        const bool two = j + 1 < nxp;
        float* o1x = two ? xo[j + 1] : nullptr;
        const int xflags = flags & ASP_F_ACCUMULATE;
#define ASP_XP(K) (two ? run_ext_pass<K, 2>(g, s, ws, pl, du, dv, dh, xw.a[j], xw.a[j + 1], xo[j], o1x, xflags, st, pass) \
                       : run_ext_pass<K, 1>(g, s, ws, pl, du, dv, dh, xw.a[j], xw.a[j], xo[j], o1x, xflags, st, pass))
        rc = kid == 0 ? ASP_XP(0) : kid == 1 ? ASP_XP(1) : ASP_XP(2);
#undef ASP_XP
        if (rc != ASP_OK) return rc;
    }
    if (gate_dev >= 0) ASP_TRY(gate_record(gate_dev, st));
    for (int k = 9; k <= 12; ++k) ws.stats[k] = 0;  // the evals diagnostic of THIS pass only
    if (getenv("ASP_COUNT_EVALS")) {  // diagnostic: the deposit kernels' lane-slots
        ASP_TRY(ensure(ws.aux[5], 3 * sizeof(unsigned long long)));
        ASP_HIP(hipMemsetAsync(ws.aux[5].p, 0, 3 * sizeof(unsigned long long), st));
        hipLaunchKernelGGL(k_evals, dim3((unsigned)(pl.n_items + (pl.n_wide ? g.ntiles : 0))),
                           dim3(kBlock), 0, st, g, kid, s, (const float4*)ws.recs.p,
                           (const Item*)ws.items.p, pl.n_items, du, dv, dh, (const int*)ws.wide.p,
                           pl.n_wide, (unsigned long long*)ws.aux[5].p);
        ASP_LAUNCHED();
        unsigned long long e[3];
        ASP_HIP(hipMemcpyAsync(e, ws.aux[5].p, sizeof(e), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
        ws.stats[9] = (long long)(e[0] + e[1] + e[2]);
        ws.stats[10] = (long long)e[0];
        ws.stats[11] = (long long)e[1];
        ws.stats[12] = (long long)e[2];
    }
    ws.stats[0] = pl.n_recs;
    ws.stats[1] = pl.n_items;
    ws.stats[2] = pl.n_wide;
    ws.stats[3] = kTile;
    ws.stats[4] = g.ntiles;
    ws.stats[5] = hc[cChunk];
    ws.stats[6] = pl.n_merges;
    ws.stats[7] = pl.n_slabs;
    ws.stats[8] = pl.n_large;
    // how this pass's records were scattered: 1 the speculative launch (enqueued before the
    // counter read-back) was kept, 2 placement trials (stats[14] scatter runs), 3 the
    // speculative launch found the buffers too small and the scatter was relaunched after
    // growing them, 0 no earlier buffers (one plain launch)
    ws.stats[13] = pre ? 1 : placed ? 2 : spec ? 3 : 0;
    ws.stats[14] = ntrials;
    return ASP_OK;
}

// Particles per pipeline pass: particle indices and record cursors are 32-bit, so larger
// calls run as batches accumulating into the same maps (ASP_MAX_BATCH lowers it for tests).
static long long max_batch() {
    long long b = 1LL << 30;
    if (const char* e = getenv("ASP_MAX_BATCH")) b = std::max(1LL, atoll(e));
    return b;
}

static Src64 src_from(const Src64& s, long long b) {  // particles b.. of s
    Src64 r = s;
    if (s.u64) {
        r.u64 += b * s.stride;
        r.v64 += b * s.stride;
        r.cu64 += b * s.stride;
        r.cv64 += b * s.stride;
        r.h64 += b;
    }
    r.u32 += b;
    r.v32 += b;
    r.h32 += b;
    return r;
}

// The whole call: every window of the image (window_grid) and, inside it, particle
// batches of < 2^31 particles, each batch split in two while its records reach 2^31.
// Batches after the first accumulate; the ratio of a batched map is formed at the end.
// rows [row_lo, row_hi) of the image only (asp_project2d_rows; default the whole image),
// d0 / d1 pointing at row row_lo: windows of <= window_rows tile rows from row_lo on.
int project2d_full(Workspace& ws, const Grid& full, const Src64& s, const float* du,
                   const float* dv, const float* dh, const float* da0, const float* da1,
                   long long n, int kid, int flags, float* d0, float* d1, hipStream_t st,
                   int row_lo = 0, int row_hi = -1, const XArgs* xa = nullptr, int nxp = 0,
                   float* const* xo = nullptr) {
    const int wr = window_rows(full);
    const long long B = max_batch();
    long long agg[kNStats] = {0};
    if (row_hi < 0) row_hi = full.gnx;
    for (int r0 = row_lo; r0 < row_hi; r0 += wr * kTile) {
        const Grid g = window_grid_rows(full, r0, std::min(r0 + wr * kTile, row_hi));
        const long long off = (long long)(g.ox - row_lo) * full.ny;
        float* w0 = d0 + off;
        float* w1 = d1 ? d1 + off : nullptr;
        float* wx[4] = {nullptr, nullptr, nullptr, nullptr};  // the extra properties' maps
        for (int j = 0; j < nxp; ++j) wx[j] = xo[j] + off;
        std::vector<std::pair<long long, long long>> todo;  // batches, last first
        for (long long a = ((n - 1) / B) * B; a >= 0; a -= B)
            todo.push_back({a, std::min(n, a + B)});
        if (todo.empty()) todo.push_back({0, 0});
        bool batched = todo.size() > 1;
        int passes = 0;
        while (!todo.empty()) {
            const auto [a, b] = todo.back();
            todo.pop_back();
            int f = flags;
            if (batched || b - a < n) f &= ~ASP_F_RATIO;  // ratio after the last batch
            if (passes > 0) f |= ASP_F_ACCUMULATE;
            XArgs xb{};
            if (xa) {
                xb = *xa;
                for (int j = 0; j < 4; ++j) xb.a[j] += a;
            }
            const int rc = project2d_device(ws, g, src_from(s, a), du + a, dv + a, dh + a,
                                            da0 + a, da1 ? da1 + a : nullptr, b - a, kid, f,
                                            w0, w1, st, nullptr, xa ? &xb : nullptr, nxp, wx);
            if (rc == kRetSplit) {
                if (b - a < 2)
                    return fail(ASP_ERR_UNSUPPORTED, "one particle makes >= 2^31 records");
                const long long m = a + (b - a) / 2;
                todo.push_back({m, b});
                todo.push_back({a, m});
                batched = true;
                continue;
            }
            ASP_TRY(rc);
            ++passes;
            for (int k : {0, 1, 2, 6, 7, 8, 9, 10, 11, 12, 14}) agg[k] += ws.stats[k];
            agg[13] = std::max(agg[13], ws.stats[13]);
        }
        if (passes > 1 && (flags & ASP_F_RATIO)) {
            const long long npix = (long long)g.nx * g.ny;
            const long long blocks = std::min<long long>((npix + kBlock - 1) / kBlock, 8192);
            StageMark m(ws, kSRatio, st);
            hipLaunchKernelGGL(k_ratio, dim3((unsigned)std::max<long long>(1, blocks)), dim3(kBlock),
                               0, st, w0, (const float*)w1, npix);
            ASP_LAUNCHED();
            m.done();
        }
    }
    for (int k : {0, 1, 2, 6, 7, 8, 9, 10, 11, 12, 13, 14}) ws.stats[k] = agg[k];
    ws.stats[4] = (long long)((row_hi - row_lo + kTile - 1) / kTile) * full.nty;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && &ws != &g_ws[dev]) {  // asp_last_stats reads slot 0
        // under slot 0's lock: a slot-0 call on another thread writes the same words (no
        // cycle: slot-0 calls never take another slot's lock)
        std::lock_guard<std::mutex> lk(g_ws[dev].mu);
        std::copy(ws.stats, ws.stats + kNStats, g_ws[dev].stats);
    }
    return ASP_OK;
}

static int check_args(const void* a1, const float* out0, const float* out1, long long n, int kid,
                      int flags) {
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (kid < 0 || kid > 2) return fail(ASP_ERR_INVALID, "unknown kernel_id");
    if (!out0) return fail(ASP_ERR_INVALID, "out0 is NULL");
    if ((a1 == nullptr) != (out1 == nullptr))
        return fail(ASP_ERR_INVALID, "a1 and out1 must both be given or both be NULL");
    if ((flags & ASP_F_RATIO) && !out1) return fail(ASP_ERR_INVALID, "ASP_F_RATIO needs out1");
    if ((flags & ASP_F_RATIO) && (flags & ASP_F_ACCUMULATE))
        return fail(ASP_ERR_INVALID, "ASP_F_RATIO cannot be combined with ASP_F_ACCUMULATE");
    // The int64 fixed point quantises each map on its own per-tile scale: pixels covered
    // only by kernel tails keep a few units of weight, so their quotient has no precision
    // (DESIGN.md §4, round 4).  Ratio maps are fp64-accumulated only.
    if ((flags & ASP_F_RATIO) && (flags & ASP_F_DETERMINISTIC))
        return fail(ASP_ERR_INVALID, "ASP_F_RATIO cannot be combined with ASP_F_DETERMINISTIC "
                                     "(fixed-point components carry no relative precision in "
                                     "kernel-tail pixels; form ratios from fp64 maps)");
    return ASP_OK;
}

static int setup_grid(double x_min, double x_max, double y_min, double y_max, int nx, int ny,
                      int cs, Grid& g) {
    if (!make_grid(x_min, x_max, y_min, y_max, nx, ny, cs, g))
        return fail(ASP_ERR_INVALID,
                    "invalid grid: need nx, ny, chunk_size >= 1, finite x_max > x_min, "
                    "y_max > y_min");
    grid_tunables(g);
    if (g.nty > kMaxTiles)
        return fail(ASP_ERR_UNSUPPORTED, "image too wide (ny > 4096 * 64 pixels)");
    return ASP_OK;
}

// Host outputs: device maps in the workspace (pre-loaded for ASP_F_ACCUMULATE).
static int host_outputs(Workspace& ws, float* out0, float* out1, long long npix, int flags,
                        hipStream_t st, float*& d0, float*& d1) {
    const int nout = out1 ? 2 : 1;
    for (int k = 0; k < nout; ++k) ASP_TRY(ensure(ws.out[k], (size_t)npix * sizeof(float)));
    d0 = (float*)ws.out[0].p;
    d1 = nout == 2 ? (float*)ws.out[1].p : nullptr;
    if (flags & ASP_F_ACCUMULATE) {
        ASP_HIP(hipMemcpyAsync(d0, out0, npix * sizeof(float), hipMemcpyHostToDevice, st));
        if (d1) ASP_HIP(hipMemcpyAsync(d1, out1, npix * sizeof(float), hipMemcpyHostToDevice, st));
    }
    return ASP_OK;
}

static int host_results(float* out0, float* out1, const float* d0, const float* d1,
                        long long npix, hipStream_t st) {
    ASP_HIP(hipMemcpyAsync(out0, d0, npix * sizeof(float), hipMemcpyDeviceToHost, st));
    if (out1) ASP_HIP(hipMemcpyAsync(out1, d1, npix * sizeof(float), hipMemcpyDeviceToHost, st));
    ASP_HIP(hipStreamSynchronize(st));
    return ASP_OK;
}

// xprops / nxp / xouts: asp_project2d_props' properties 2.. (device pointers).
static int check_props(int nxp, const void* const* xprops, float* const* xouts, int flags) {
    if (nxp == 0) return ASP_OK;
    if (nxp < 0 || nxp > 4) return fail(ASP_ERR_INVALID, "nprops must be 1 .. 6");
    if (!xprops || !xouts) return fail(ASP_ERR_INVALID, "NULL props / outs");
    for (int j = 0; j < nxp; ++j)
        if (!xprops[j] || !xouts[j]) return fail(ASP_ERR_INVALID, "NULL property or output");
    if (!(flags & ASP_F_DEVICE_PTRS))
        return fail(ASP_ERR_UNSUPPORTED, "more than two properties: device pointers only "
                                         "(ASP_F_DEVICE_PTRS)");
    if (flags & (ASP_F_RATIO | ASP_F_DETERMINISTIC))
        return fail(ASP_ERR_UNSUPPORTED, "more than two properties: no ASP_F_RATIO / "
                                         "ASP_F_DETERMINISTIC (fp64 sums; ratios with asp_ratio)");
    return ASP_OK;
}

// SPH weights (asp_project2d_sph, north_star's "mass/rho-weighted scatter"): the fp32
// working copy of a property A is fl32(A * (m / rho)) -- evaluated in fp64 from the
// caller's values, rounded once (rho NULL: fl32(A * m)).  The SPH estimate of a field is
// sum_j (m_j / rho_j) A_j W(r_ij, h_j) (get_densities: _SnapshotBase.py:833); the scatter
// then bins and deposits these coefficients as any property's.
template <class T>
__global__ __launch_bounds__(kBlock) void k_weigh(const T* __restrict__ a, const T* __restrict__ m,
                                                  const T* __restrict__ rho,
                                                  float* __restrict__ out, long long n) {
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (long long)gridDim.x * kBlock) {
        const double w = rho ? (double)m[i] / (double)rho[i] : (double)m[i];
        out[i] = (float)((double)a[i] * w);
    }
}

// The weighted fp32 copies of a0 (, a1) and properties 2.. into ws.wts (slot k = property
// k), on st; the pointers are redirected to them.
template <class T>
static int weigh_props(Workspace& ws, const T* a0, const T* a1, const T* const* xprops, int nxp,
                       const T* m, const T* rho, long long n, hipStream_t st, const float** da0,
                       const float** da1, const float** xw) {
    const T* src[6] = {a0, a1, nullptr, nullptr, nullptr, nullptr};
    for (int j = 0; j < nxp; ++j) src[2 + j] = xprops[j];
    const long long blocks = std::min<long long>((n + kBlock - 1) / kBlock, 8192);
    for (int k = 0; k < 6; ++k) {
        if (!src[k]) continue;
        ASP_TRY(ensure(ws.wts[k], (size_t)std::max(n, 1LL) * sizeof(float)));
        if (n > 0) {
            hipLaunchKernelGGL(k_weigh<T>, dim3((unsigned)blocks), dim3(kBlock), 0, st, src[k], m,
                               rho, (float*)ws.wts[k].p, n);
            ASP_LAUNCHED();
        }
    }
    *da0 = (const float*)ws.wts[0].p;
    if (a1) *da1 = (const float*)ws.wts[1].p;
    for (int j = 0; j < nxp; ++j) xw[j] = (const float*)ws.wts[2 + j].p;
    return ASP_OK;
}

static int project2d(const float* u, const float* v, const float* h, const float* a0,
                     const float* a1, long long n, double x_min, double x_max, double y_min,
                     double y_max, int nx, int ny, int cs, int kid, int flags, float* out0,
                     float* out1, int device, void* stream, int row_lo = 0, int row_hi = -1,
                     const float* const* xprops = nullptr, int nxp = 0,
                     float* const* xouts = nullptr, const float* wm = nullptr,
                     const float* wr = nullptr) {
    ASP_TRY(check_args(a1, out0, out1, n, kid, flags));
    ASP_TRY(check_props(nxp, (const void* const*)xprops, xouts, flags));
    if (nxp > 0 && !a1) return fail(ASP_ERR_INVALID, "properties 2.. need a1 / out1");
    if (n > 0 && (!u || !v || !h || !a0)) return fail(ASP_ERR_INVALID, "NULL particle array");
    Grid g;
    ASP_TRY(setup_grid(x_min, x_max, y_min, y_max, nx, ny, cs, g));
    if (row_hi < 0) row_hi = nx;
    if (row_lo < 0 || row_lo >= row_hi || row_hi > nx)
        return fail(ASP_ERR_INVALID, "rows: need 0 <= row_lo < row_hi <= nx");
    nx = row_hi - row_lo;  // the rows this call writes (the grid keeps the whole image's)
    ASP_TRY(set_device(device));
    Workspace& ws = slot_ws(device, map_slot(device, (hipStream_t)stream));
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
    const int nout = out1 ? 2 : 1;
    const bool dev = flags & ASP_F_DEVICE_PTRS;
    const long long npix = (long long)nx * ny;
    const float *du = u, *dv = v, *dh = h, *da0 = a0, *da1 = a1;
    float *d0 = out0, *d1 = out1;
    if (!dev) {
        const float* src[5] = {u, v, h, a0, a1};
        for (int k = 0; k < 4 + (nout == 2); ++k) {
            ASP_TRY(ensure(ws.in[k], (size_t)n * sizeof(float)));
            ASP_TRY(h2d_staged(ws, ws.in[k].p, src[k], (size_t)n * sizeof(float), st));
        }
        du = (const float*)ws.in[0].p;
        dv = (const float*)ws.in[1].p;
        dh = (const float*)ws.in[2].p;
        da0 = (const float*)ws.in[3].p;
        da1 = nout == 2 ? (const float*)ws.in[4].p : nullptr;
        ASP_TRY(host_outputs(ws, out0, out1, npix, flags, st, d0, d1));
    }
    const float* xw[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int j = 0; j < nxp; ++j) xw[j] = xprops[j];
    if (wm) {  // asp_project2d_sph: the properties times m / rho
        const float *dm = wm, *dr = wr;
        if (!dev) {
            const float* src[2] = {wm, wr};
            for (int k = 0; k < 2; ++k) {
                if (!src[k]) continue;
                ASP_TRY(ensure(ws.inw[k], (size_t)n * sizeof(float)));
                ASP_TRY(h2d_staged(ws, ws.inw[k].p, src[k], (size_t)n * sizeof(float), st));
            }
            dm = (const float*)ws.inw[0].p;
            dr = wr ? (const float*)ws.inw[1].p : nullptr;
        }
        ASP_TRY(weigh_props<float>(ws, da0, da1, xprops, nxp, dm, dr, n, st, &da0, &da1, xw));
    }
    const Src64 s{nullptr, nullptr, nullptr, nullptr, nullptr, 0, du, dv, dh};
    XArgs xa{};
    for (int j = 0; j < 4; ++j) xa.a[j] = j < nxp ? xw[j] : (nxp ? xw[0] : nullptr);
    ASP_TRY(project2d_full(ws, g, s, du, dv, dh, da0, da1, n, kid, flags, d0, d1, st, row_lo,
                           row_hi, nxp ? &xa : nullptr, nxp, xouts));
    if (!dev) ASP_TRY(host_results(out0, out1, d0, d1, npix, st));
    return ws_end_.finish();
}

// create_image on the reader's fp64 arrays: stage (axis selection, fp32 working copies in
// HBM) and project with the fp64 values kept for the exact re-decisions.
__global__ __launch_bounds__(kBlock) void k_to_f32(const double* __restrict__ a,
                                                   float* __restrict__ b, long long n) {
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (long long)gridDim.x * kBlock)
        b[i] = (float)a[i];  // round to nearest, as NumPy's astype(float32)
}

static int project2d_f64(const double* pos, const double* h, const double* a0,
                         const double* a1, long long n, int axis, double x_min, double x_max,
                         double y_min, double y_max, int nx, int ny, int cs, int kid, int flags,
                         float* out0, float* out1, int device, void* stream,
                         const double* const* xprops = nullptr, int nxp = 0,
                         float* const* xouts = nullptr, const double* wm = nullptr,
                         const double* wr = nullptr) {
    ASP_TRY(check_args(a1, out0, out1, n, kid, flags));
    ASP_TRY(check_props(nxp, (const void* const*)xprops, xouts, flags));
    if (nxp > 0 && !a1) return fail(ASP_ERR_INVALID, "properties 2.. need a1 / out1");
    if (n > 0 && (!pos || !h || !a0)) return fail(ASP_ERR_INVALID, "NULL particle array");
    // axis: the pixel test's axis, | ASP_AXIS_CULL(c) to cull on axis c's columns
    const int cull_axis = (axis >> 4) ? (axis >> 4) - 1 : (axis & 15);
    axis &= 15;
    if (axis < 0 || axis > 2 || cull_axis < 0 || cull_axis > 2)
        return fail(ASP_ERR_INVALID, "projection axis must be 0 (X), 1 (Y) or 2 (Z)");
    Grid g;
    ASP_TRY(setup_grid(x_min, x_max, y_min, y_max, nx, ny, cs, g));
    g.mixed = cull_axis != axis;
    ASP_TRY(set_device(device));
    Workspace& ws = slot_ws(device, map_slot(device, (hipStream_t)stream));
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
    const int nout = out1 ? 2 : 1;
    const bool dev = flags & ASP_F_DEVICE_PTRS;
    const bool dev_out = dev || (flags & ASP_F_DEVICE_OUTPUTS);  // maps stay on the device
    const long long npix = (long long)nx * ny;
    const double *dpos = pos, *dh64 = h, *da0 = a0, *da1 = a1;
    float *d0 = out0, *d1 = out1;
    if (!dev) {
        // the fp64 arrays stay resident: the exact re-decisions read positions and h
        const double* src[4] = {pos, h, a0, a1};
        const size_t words[4] = {3, 1, 1, 1};
        for (int k = 0; k < 3 + (nout == 2); ++k) {
            ASP_TRY(ensure(ws.in64[k], (size_t)n * words[k] * sizeof(double)));
            ASP_TRY(h2d_staged(ws, ws.in64[k].p, src[k], (size_t)n * words[k] * sizeof(double), st));
        }
        dpos = (const double*)ws.in64[0].p;
        dh64 = (const double*)ws.in64[1].p;
        da0 = (const double*)ws.in64[2].p;
        da1 = nout == 2 ? (const double*)ws.in64[3].p : nullptr;
        if (!dev_out) ASP_TRY(host_outputs(ws, out0, out1, npix, flags, st, d0, d1));
    }
    for (int k = 0; k < 4 + (nout == 2); ++k) ASP_TRY(ensure(ws.in[k], (size_t)n * sizeof(float)));
    float* f[5] = {(float*)ws.in[0].p, (float*)ws.in[1].p, (float*)ws.in[2].p, (float*)ws.in[3].p,
                   nout == 2 ? (float*)ws.in[4].p : nullptr};
    // asp_project2d_sph_f64: the properties' fp32 copies are m / rho * A (weigh_props), so
    // the staging converts positions and h only
    ASP_TRY(stage_device(dpos, dh64, wm ? nullptr : da0, wm ? nullptr : da1, n, axis, f[0], f[1],
                         f[2], wm ? nullptr : f[3], wm ? nullptr : f[4], st));
    const float* fa0 = f[3];
    const float* fa1 = f[4];
    const float* xw[4] = {nullptr, nullptr, nullptr, nullptr};
    if (wm) {
        const double *dm = wm, *dr = wr;
        if (!dev) {
            const double* src[2] = {wm, wr};
            for (int k = 0; k < 2; ++k) {
                if (!src[k]) continue;
                ASP_TRY(ensure(ws.inw[k], (size_t)n * sizeof(double)));
                ASP_TRY(h2d_staged(ws, ws.inw[k].p, src[k], (size_t)n * sizeof(double), st));
            }
            dm = (const double*)ws.inw[0].p;
            dr = wr ? (const double*)ws.inw[1].p : nullptr;
        }
        ASP_TRY(weigh_props<double>(ws, da0, da1, xprops, nxp, dm, dr, n, st, &fa0, &fa1, xw));
    }
    static const int cols[3][2] = {{1, 2}, {0, 2}, {0, 1}};  // _projector.py:38-46
    const Src64 s{dpos + cols[axis][0], dpos + cols[axis][1], dpos + cols[cull_axis][0],
                  dpos + cols[cull_axis][1], dh64, 3, f[0], f[1], f[2]};
    XArgs xa{};
    for (int j = 0; j < nxp && !wm; ++j) {  // fp32 working copies of properties 2..
        ASP_TRY(ensure(ws.inx[j], (size_t)std::max(n, 1LL) * sizeof(float)));
        if (n > 0) {
            const long long blocks = std::min<long long>((n + kBlock - 1) / kBlock, 8192);
            hipLaunchKernelGGL(k_to_f32, dim3((unsigned)blocks), dim3(kBlock), 0, st, xprops[j],
                               (float*)ws.inx[j].p, n);
            ASP_LAUNCHED();
        }
        xw[j] = (const float*)ws.inx[j].p;
    }
    for (int j = 0; j < 4; ++j) xa.a[j] = nxp ? xw[j < nxp ? j : 0] : nullptr;
    ASP_TRY(project2d_full(ws, g, s, f[0], f[1], f[2], fa0, fa1, n, kid,
                           (flags & ~ASP_F_DEVICE_OUTPUTS) | ASP_F_DEVICE_PTRS, d0, d1, st, 0, -1,
                           nxp ? &xa : nullptr, nxp, xouts));
    if (!dev_out) ASP_TRY(host_results(out0, out1, d0, d1, npix, st));
    return ws_end_.finish();
}

// The kernel_func plug-in session (asp_pairs_begin / _emit / _end): the particles are
// staged and binned ONCE per create_image call, window by window (window_grid); the
// records of the current window stay resident in the session's own workspace between the
// emits, so a map needing many host batches costs one binning per window, not one per
// batch.
struct PairsSession {
    Workspace ws;  // the session's own buffers (a call on the device cannot evict them)
    Grid full;
    Src64 s{};
    const float* f[3] = {nullptr, nullptr, nullptr};  // fp32 working copies u, v, h
    long long n = 0;
    int device = 0;
    int flags = 0;
    hipStream_t st = nullptr;
    int wtx0 = -1, wtx1 = -1;  // tile rows binned now
    int n_wide = 0;
    std::vector<long long> tile_pairs;  // per GPU tile of the whole image
};

static inline int pairs_window_of(const PairsSession& S, int t) {  // first tile row of t's window
    const int tx = t / S.full.nty, wr = window_rows(S.full);
    return (tx / wr) * wr;
}

// Bin the window holding tile rows [tx0, ..) and count its pixels' pairs (MODE 0).
static int pairs_bin(PairsSession& S, int tx0) {
    Workspace& ws = S.ws;
    const int wr = window_rows(S.full);
    const int tx1 = std::min(tx0 + wr, S.full.ntx);
    if (S.wtx0 == tx0) return ASP_OK;
    const Grid g = window_grid(S.full, tx0, tx1);
    S.wtx0 = -1;
    ASP_TRY(ensure(ws.pairs[0], (size_t)g.ntiles * kTilePix * sizeof(int)));  // pixcnt
    ASP_TRY(ensure(ws.pairs[3], (size_t)g.ntiles * sizeof(long long)));       // tile totals
    if (S.n == 0) {  // nothing binned: zero pixel counts and tile totals
        ASP_HIP(hipMemsetAsync(ws.pairs[0].p, 0, (size_t)g.ntiles * kTilePix * sizeof(int), S.st));
        ASP_HIP(hipMemsetAsync(ws.pairs[3].p, 0, (size_t)g.ntiles * sizeof(long long), S.st));
        S.n_wide = 0;
    } else {
        int nw = 0;
        const int rc = project2d_device(ws, g, S.s, S.f[0], S.f[1], S.f[2], S.f[2], nullptr, S.n,
                                        ASP_KERNEL_INDICATOR, 0, nullptr, nullptr, S.st, &nw);
        if (rc == kRetSplit)
            return fail(ASP_ERR_UNSUPPORTED, "kernel_func plug-in: >= 2^31 records in one window");
        ASP_TRY(rc);
        S.n_wide = nw;
        hipLaunchKernelGGL(k_pairs<0>, dim3((unsigned)g.ntiles), dim3(kPairsBlock), 0, S.st, g,
                           S.s, (const float4*)ws.recs.p, (const long long*)ws.tile_start.p,
                           (const int*)ws.tile_total.p, (const int*)ws.wide.p, nw, S.f[0], S.f[1],
                           S.f[2], 0, (int*)ws.pairs[0].p, (long long*)ws.pairs[3].p,
                           (const long long*)nullptr, (long long*)nullptr, (int*)nullptr,
                           (double*)nullptr, (int*)nullptr);
        ASP_LAUNCHED();
    }
    S.wtx0 = tx0;
    S.wtx1 = tx1;
    return ASP_OK;
}

static int pairs_begin(const double* pos, const double* h, long long n, int axis, double x_min,
                       double x_max, double y_min, double y_max, int nx, int ny, int cs,
                       int flags, int device, void* stream, long long* tile_pairs,
                       PairsSession** out) {
    *out = nullptr;
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (n > 0x7fffffffLL)
        return fail(ASP_ERR_UNSUPPORTED, "kernel_func plug-in: n >= 2^31 particles per call");
    if (n > 0 && (!pos || !h)) return fail(ASP_ERR_INVALID, "NULL particle array");
    if (!tile_pairs) return fail(ASP_ERR_INVALID, "NULL tile_pairs");
    const int cull_axis = (axis >> 4) ? (axis >> 4) - 1 : (axis & 15);
    axis &= 15;
    if (axis < 0 || axis > 2 || cull_axis < 0 || cull_axis > 2)
        return fail(ASP_ERR_INVALID, "projection axis must be 0 (X), 1 (Y) or 2 (Z)");
    Grid g;
    ASP_TRY(setup_grid(x_min, x_max, y_min, y_max, nx, ny, cs, g));
    g.mixed = cull_axis != axis;
    ASP_TRY(set_device(device));
    PairsSession* S = new (std::nothrow) PairsSession();
    if (!S) return fail(ASP_ERR_NOMEM, "session");
    S->full = g;
    S->n = n;
    S->device = device;
    S->flags = flags;
    S->st = (hipStream_t)stream;
    Workspace& ws = S->ws;
    auto bail = [&](int rc) {
        (void)hipStreamSynchronize(S->st);
        ws_teardown(ws);
        delete S;
        return rc;
    };
    const bool dev = flags & ASP_F_DEVICE_PTRS;
    const double *dpos = pos, *dh64 = h;
    if (!dev && n > 0) {
        int rc = ensure(ws.in64[0], (size_t)n * 3 * sizeof(double));
        if (rc == ASP_OK) rc = ensure(ws.in64[1], (size_t)n * sizeof(double));
        if (rc == ASP_OK) rc = h2d_staged(ws, ws.in64[0].p, pos, (size_t)n * 3 * sizeof(double), S->st);
        if (rc == ASP_OK) rc = h2d_staged(ws, ws.in64[1].p, h, (size_t)n * sizeof(double), S->st);
        if (rc != ASP_OK) return bail(rc);
        dpos = (const double*)ws.in64[0].p;
        dh64 = (const double*)ws.in64[1].p;
    }
    for (int k = 0; k < 3; ++k) {
        const int rc = ensure(ws.in[k], (size_t)n * sizeof(float));
        if (rc != ASP_OK) return bail(rc);
    }
    float* f[3] = {(float*)ws.in[0].p, (float*)ws.in[1].p, (float*)ws.in[2].p};
    if (n > 0) {
        const int rc = stage_device(dpos, dh64, nullptr, nullptr, n, axis, f[0], f[1], f[2],
                                    nullptr, nullptr, S->st);
        if (rc != ASP_OK) return bail(rc);
    }
    static const int cols[3][2] = {{1, 2}, {0, 2}, {0, 1}};  // _projector.py:38-46
    S->s = Src64{dpos + cols[axis][0], dpos + cols[axis][1], dpos + cols[cull_axis][0],
                 dpos + cols[cull_axis][1], dh64, 3, f[0], f[1], f[2]};
    for (int k = 0; k < 3; ++k) S->f[k] = f[k];
    // every window once: its per-tile pair totals (the last window stays binned)
    S->tile_pairs.assign((size_t)g.ntiles, 0);
    const int wr = window_rows(g);
    for (int tx0 = 0; tx0 < g.ntx; tx0 += wr) {
        int rc = pairs_bin(*S, tx0);
        const Grid w = window_grid(g, tx0, std::min(tx0 + wr, g.ntx));
        if (rc == ASP_OK)
            rc = hipMemcpyAsync(S->tile_pairs.data() + (size_t)tx0 * g.nty, ws.pairs[3].p,
                                (size_t)w.ntiles * sizeof(long long), hipMemcpyDeviceToHost,
                                S->st) == hipSuccess ? ASP_OK : fail(ASP_ERR_HIP, "tile totals");
        if (rc == ASP_OK)
            rc = hipStreamSynchronize(S->st) == hipSuccess ? ASP_OK : fail(ASP_ERR_HIP, "sync");
        if (rc != ASP_OK) return bail(rc);
    }
    std::copy(S->tile_pairs.begin(), S->tile_pairs.end(), tile_pairs);
    *out = S;
    return ASP_OK;
}

// Pairs of the GPU tiles [t0, t1) (global row-major tile ids), pixels tile by tile and
// lx * 64 + ly inside a tile: offsets ((t1 - t0) * 4096 + 1, from 0), particle, r2.
static int pairs_emit(PairsSession& S, int t0, int t1, long long* offsets, int* particle,
                      double* r2) {
    if (t0 < 0 || t1 > S.full.ntiles || t0 > t1) return fail(ASP_ERR_INVALID, "bad tile range");
    if (!offsets) return fail(ASP_ERR_INVALID, "NULL offsets");
    Workspace& ws = S.ws;
    ASP_HIP(hipSetDevice(S.device));
    const bool dev = S.flags & ASP_F_DEVICE_PTRS;
    const long long npx = (long long)(t1 - t0) * kTilePix;
    long long total = 0;
    for (int t = t0; t < t1; ++t) total += S.tile_pairs[t];
    if (total > 0 && (!particle || !r2)) return fail(ASP_ERR_INVALID, "NULL pair outputs");
    long long* doff = offsets;
    int* dpart = particle;
    double* dr2 = r2;
    if (!dev) {
        ASP_TRY(ensure(ws.aux[0], (size_t)(npx + 1) * sizeof(long long)));
        ASP_TRY(ensure(ws.aux[1], (size_t)std::max(total, 1LL) * sizeof(int)));
        ASP_TRY(ensure(ws.aux[2], (size_t)std::max(total, 1LL) * sizeof(double)));
        doff = (long long*)ws.aux[0].p;
        dpart = (int*)ws.aux[1].p;
        dr2 = (double*)ws.aux[2].p;
    }
    ASP_TRY(ensure(ws.aux[3], (size_t)(t1 - t0 + 1) * sizeof(long long)));
    ASP_TRY(ensure(ws.aux[4], sizeof(int)));
    int* dovf = (int*)ws.aux[4].p;
    ASP_HIP(hipMemsetAsync(dovf, 0, sizeof(int), S.st));
    if (npx == 0 || S.n == 0) {
        // no tiles, or no particles (nothing was binned: no records for k_pairs to read):
        // every pixel's range is empty
        if (!dev) std::fill(offsets, offsets + npx + 1, 0LL);
        else ASP_HIP(hipMemsetAsync(offsets, 0, (size_t)(npx + 1) * sizeof(long long), S.st));
        ASP_HIP(hipStreamSynchronize(S.st));
        return ASP_OK;
    }
    // window by window (the session re-bins only when the range moves to another window)
    long long done = 0;
    for (int a = t0; a < t1;) {
        const int tx0 = pairs_window_of(S, a);
        ASP_TRY(pairs_bin(S, tx0));
        const int wt0 = tx0 * S.full.nty;                          // window's first tile
        const int b = std::min(t1, S.wtx1 * S.full.nty);
        std::vector<long long> base((size_t)(b - a));
        for (int t = a; t < b; ++t) {
            base[t - a] = done;
            done += S.tile_pairs[t];
        }
        long long* dbase = (long long*)ws.aux[3].p;
        ASP_HIP(hipMemcpyAsync(dbase, base.data(), base.size() * sizeof(long long),
                               hipMemcpyHostToDevice, S.st));
        const Grid g = window_grid(S.full, S.wtx0, S.wtx1);
        hipLaunchKernelGGL(k_pairs<1>, dim3((unsigned)(b - a)), dim3(kPairsBlock), 0, S.st, g,
                           S.s, (const float4*)ws.recs.p, (const long long*)ws.tile_start.p,
                           (const int*)ws.tile_total.p, (const int*)ws.wide.p, S.n_wide, S.f[0],
                           S.f[1], S.f[2], a - wt0, (int*)ws.pairs[0].p, (long long*)nullptr,
                           (const long long*)dbase, doff + (long long)(a - t0) * kTilePix, dpart,
                           dr2, dovf);
        ASP_LAUNCHED();
        ASP_HIP(hipStreamSynchronize(S.st));  // dbase is reused by the next window's launch
        a = b;
    }
    int ovf = 0;
    ASP_HIP(hipMemcpyAsync(&ovf, dovf, sizeof(int), hipMemcpyDeviceToHost, S.st));
    if (!dev) {
        ASP_HIP(hipMemcpyAsync(offsets, doff, (size_t)(npx + 1) * sizeof(long long),
                               hipMemcpyDeviceToHost, S.st));
        if (total > 0) {
            ASP_HIP(hipMemcpyAsync(particle, dpart, (size_t)total * sizeof(int),
                                   hipMemcpyDeviceToHost, S.st));
            ASP_HIP(hipMemcpyAsync(r2, dr2, (size_t)total * sizeof(double), hipMemcpyDeviceToHost,
                                   S.st));
        }
    }
    ASP_HIP(hipStreamSynchronize(S.st));
    if (ovf) return fail(ASP_ERR_INVALID, "pair slots overflowed (counts and pairs disagree)");
    return ASP_OK;
}

static int pairs_end(PairsSession* S) {
    if (!S) return ASP_OK;
    (void)hipSetDevice(S->device);
    (void)hipStreamSynchronize(S->st);
    ws_teardown(S->ws);  // buffers, pinned memory, the side stream and its events
    delete S;
    return ASP_OK;
}

}  // namespace asp

// ==================================================================================
// C-ABI
// ==================================================================================
using namespace asp;

extern "C" {

int asp_version(void) { return ASP_API_VERSION * 10000 + 2; }

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

int asp_project2d_rows(const float* u, const float* v, const float* h, const float* a0,
                       const float* a1, int64_t n, double u_min, double u_max, double v_min,
                       double v_max, int32_t nx, int32_t ny, int32_t chunk_size, int32_t row_lo,
                       int32_t row_hi, int32_t kernel_id, int32_t flags, float* out0,
                       float* out1, int32_t device, void* stream) {
    t_err.clear();
    return project2d(u, v, h, a0, a1, n, u_min, u_max, v_min, v_max, nx, ny, chunk_size,
                     kernel_id, flags, out0, out1, device, stream, row_lo, row_hi);
}

int asp_project2d_props(const float* u, const float* v, const float* h, const float* const* props,
                        int32_t nprops, int64_t n, double u_min, double u_max, double v_min,
                        double v_max, int32_t nx, int32_t ny, int32_t chunk_size,
                        int32_t kernel_id, int32_t flags, float* const* outs, int32_t device,
                        void* stream) {
    t_err.clear();
    if (nprops < 1 || nprops > 6 || !props || !outs)
        return fail(ASP_ERR_INVALID, "nprops must be 1 .. 6 with props / outs given");
    return project2d(u, v, h, props[0], nprops > 1 ? props[1] : nullptr, n, u_min, u_max, v_min,
                     v_max, nx, ny, chunk_size, kernel_id, flags, outs[0],
                     nprops > 1 ? outs[1] : nullptr, device, stream, 0, -1,
                     nprops > 2 ? props + 2 : nullptr, std::max(0, nprops - 2),
                     nprops > 2 ? outs + 2 : nullptr);
}

int asp_project2d_props_f64(const double* positions, const double* h,
                            const double* const* props, int32_t nprops, int64_t n, int32_t axis,
                            double u_min, double u_max, double v_min, double v_max, int32_t nx,
                            int32_t ny, int32_t chunk_size, int32_t kernel_id, int32_t flags,
                            float* const* outs, int32_t device, void* stream) {
    t_err.clear();
    if (nprops < 1 || nprops > 6 || !props || !outs)
        return fail(ASP_ERR_INVALID, "nprops must be 1 .. 6 with props / outs given");
    return project2d_f64(positions, h, props[0], nprops > 1 ? props[1] : nullptr, n, axis, u_min,
                         u_max, v_min, v_max, nx, ny, chunk_size, kernel_id, flags, outs[0],
                         nprops > 1 ? outs[1] : nullptr, device, stream,
                         nprops > 2 ? props + 2 : nullptr, std::max(0, nprops - 2),
                         nprops > 2 ? outs + 2 : nullptr);
}

int asp_project2d_sph(const float* u, const float* v, const float* h, const float* mass,
                      const float* rho, const float* const* props, int32_t nprops, int64_t n,
                      double u_min, double u_max, double v_min, double v_max, int32_t nx,
                      int32_t ny, int32_t chunk_size, int32_t kernel_id, int32_t flags,
                      float* const* outs, int32_t device, void* stream) {
    t_err.clear();
    if (nprops < 1 || nprops > 6 || !props || !outs)
        return fail(ASP_ERR_INVALID, "nprops must be 1 .. 6 with props / outs given");
    if (n > 0 && !mass) return fail(ASP_ERR_INVALID, "NULL mass array");
    return project2d(u, v, h, props[0], nprops > 1 ? props[1] : nullptr, n, u_min, u_max, v_min,
                     v_max, nx, ny, chunk_size, kernel_id, flags, outs[0],
                     nprops > 1 ? outs[1] : nullptr, device, stream, 0, -1,
                     nprops > 2 ? props + 2 : nullptr, std::max(0, nprops - 2),
                     nprops > 2 ? outs + 2 : nullptr, mass, rho);
}

int asp_project2d_sph_f64(const double* positions, const double* h, const double* mass,
                          const double* rho, const double* const* props, int32_t nprops,
                          int64_t n, int32_t axis, double u_min, double u_max, double v_min,
                          double v_max, int32_t nx, int32_t ny, int32_t chunk_size,
                          int32_t kernel_id, int32_t flags, float* const* outs, int32_t device,
                          void* stream) {
    t_err.clear();
    if (nprops < 1 || nprops > 6 || !props || !outs)
        return fail(ASP_ERR_INVALID, "nprops must be 1 .. 6 with props / outs given");
    if (n > 0 && !mass) return fail(ASP_ERR_INVALID, "NULL mass array");
    return project2d_f64(positions, h, props[0], nprops > 1 ? props[1] : nullptr, n, axis, u_min,
                         u_max, v_min, v_max, nx, ny, chunk_size, kernel_id, flags, outs[0],
                         nprops > 1 ? outs[1] : nullptr, device, stream,
                         nprops > 2 ? props + 2 : nullptr, std::max(0, nprops - 2),
                         nprops > 2 ? outs + 2 : nullptr, mass, rho);
}

int asp_project2d_f64(const double* positions, const double* h, const double* a0,
                      const double* a1, int64_t n, int32_t axis, double u_min, double u_max,
                      double v_min, double v_max, int32_t nx, int32_t ny, int32_t chunk_size,
                      int32_t kernel_id, int32_t flags, float* out0, float* out1, int32_t device,
                      void* stream) {
    t_err.clear();
    return project2d_f64(positions, h, a0, a1, n, axis, u_min, u_max, v_min, v_max, nx, ny,
                         chunk_size, kernel_id, flags, out0, out1, device, stream);
}

int asp_pairs_begin(const double* positions, const double* h, int64_t n, int32_t axis,
                    double u_min, double u_max, double v_min, double v_max, int32_t nx,
                    int32_t ny, int32_t chunk_size, int32_t flags, int32_t device, void* stream,
                    int64_t* tile_pairs, void** session) {
    t_err.clear();
    if (!session) return fail(ASP_ERR_INVALID, "NULL session");
    PairsSession* S = nullptr;
    const int rc = pairs_begin(positions, h, n, axis, u_min, u_max, v_min, v_max, nx, ny,
                               chunk_size, flags, device, stream, (long long*)tile_pairs, &S);
    *session = S;
    return rc;
}

int asp_pairs_emit(void* session, int32_t tile_lo, int32_t tile_hi, int64_t* offsets,
                   int32_t* particle, double* r2) {
    t_err.clear();
    if (!session) return fail(ASP_ERR_INVALID, "NULL session");
    return pairs_emit(*(PairsSession*)session, tile_lo, tile_hi, (long long*)offsets, particle, r2);
}

int asp_pairs_end(void* session) {
    t_err.clear();
    return pairs_end((PairsSession*)session);
}

int asp_kernel_eval(int32_t kernel_id, const double* r, const double* h, double* w, int64_t n,
                    int32_t flags, int32_t device, void* stream) {
    t_err.clear();
    if (kernel_id < 0 || kernel_id > 2) return fail(ASP_ERR_INVALID, "unknown kernel_id");
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (n == 0) return ASP_OK;
    ASP_TRY(set_device(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
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
    return ws_end_.finish();
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
    ASP_TRY(set_device(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = (hipStream_t)stream;
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
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
    return ws_end_.finish();
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
    ASP_TRY(set_device(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = nullptr;
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
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
    const Src64 s{nullptr, nullptr, nullptr, nullptr, nullptr, 0, (const float*)ws.in[0].p,
                  (const float*)ws.in[1].p, (const float*)ws.in[2].p};
    hipLaunchKernelGGL(k_neighbours, dim3((unsigned)npix), dim3(kBlock), 0, st, g, s,
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
        hipLaunchKernelGGL(k_neighbours, dim3((unsigned)npix), dim3(kBlock), 0, st, g, s,
                           (const float*)ws.in[0].p, (const float*)ws.in[1].p,
                           (const float*)ws.in[2].p, (long long)n, (const long long*)ws.aux[0].p,
                           (long long*)ws.aux[1].p, (const long long*)ws.aux[2].p,
                           (int*)ws.aux[3].p, wcap, 1);
        ASP_HIP(hipGetLastError());
        ASP_HIP(hipMemcpyAsync(index, ws.aux[3].p, wcap * sizeof(int), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    return ws_end_.finish();
}

int asp_ratio(float* out0, const float* out1, int64_t n, int32_t device, void* stream) {
    t_err.clear();
    if (n < 0 || !out0 || !out1) return fail(ASP_ERR_INVALID, "bad argument");
    if (n == 0) return ASP_OK;
    ASP_TRY(set_device(device));
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
    for (int sl = 0; sl < kMapSlots; ++sl) {  // every map slot's workspace
        Workspace& ws = slot_ws(device, sl);
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
    }
    return ASP_OK;
}

int asp_profile(int32_t device, int32_t enable) {
    return asp_profile_stages(device, enable ? 0xffffffffu : 0u);
}

int asp_profile_read(int32_t device, double* ms_sum, int64_t* launches, int32_t nstages) {
    t_err.clear();
    if (device < 0 || device >= 64 || !ms_sum || !launches)
        return fail(ASP_ERR_INVALID, "bad argument");
    for (int k = 0; k < nstages; ++k) {
        ms_sum[k] = 0.0;
        launches[k] = 0;
    }
    for (int sl = 0; sl < kMapSlots; ++sl) {  // summed over the map slots
        Workspace& ws = slot_ws(device, sl);
        std::lock_guard<std::mutex> lock(ws.mu);
        if (ws.prof) {
            ASP_HIP(hipSetDevice(device));
            ASP_TRY(prof_fold(ws));
        }
        for (int k = 0; k < nstages && k < kStages; ++k) {
            ms_sum[k] += ws.stage_ms[k];
            launches[k] += ws.stage_n[k];
        }
    }
    return ASP_OK;
}

int asp_last_stats(int32_t device, int64_t* stats, int32_t nstats) {
    if (device < 0 || device >= 64 || !stats) return fail(ASP_ERR_INVALID, "bad argument");
    std::lock_guard<std::mutex> lk(g_ws[device].mu);  // a call in flight writes them
    for (int k = 0; k < nstats && k < kNStats; ++k) stats[k] = g_ws[device].stats[k];
    return ASP_OK;
}

int asp_release(int32_t device) {
    int lo = device < 0 ? 0 : device, hi = device < 0 ? 63 : device;
    int ndev = asp_device_count();
    for (int d = lo; d <= hi && d < ndev; ++d)
      for (int sl = 0; sl < kMapSlots; ++sl) {
        Workspace& ws = slot_ws(d, sl);
        std::lock_guard<std::mutex> lock(ws.mu);
        if (hipSetDevice(d) != hipSuccess) continue;
        if (ws.last_ev) (void)hipEventSynchronize(ws.last_ev);
        for (Buf* b : ws.all_bufs()) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
        if (ws.h_counters) (void)hipHostFree(ws.h_counters);
        ws.h_counters = nullptr;
        release_pinned(ws);
        ws.morton_ntx = ws.morton_nty = -1;
        ws.morton3_key[0] = ws.morton3_key[1] = ws.morton3_key[2] = -1;
    }
    return ASP_OK;
}

}  // extern "C"
