// asp_project3d.hip -- MI355X (gfx950) SPH particle -> voxel-cube deposit (512^3 cube,
// SURVEY.md §8(a) last row; BASELINE.json configs[4]).
//
// The reference has no volumetric path; the cube's semantics are the build's own,
// restated on the CPU by oracle/asp_oracle.c (oracle_project3d): voxel-corner sampling
// with each axis' own pitch, 3-D distance, the same kernels and the same strict
// r2 < (2h)^2 neighbour test as the 2-D map (_pixel_calculations.pyx:11-14, :30-34).
//
// Same pipeline shape as the 2-D projector, on 16 x 16 x 32 voxel bricks (z fastest,
// matching the (nx, ny, nz) C-order output, so one brick row is a 128-byte run):
//   C1 count     streaming pass over (x, y, z, h): LDS histogram of (particle, brick)
//                insertions per workgroup -> hist[block][brick]
//   C2 colscan / tilescan   shared with the 2-D path (asp_binning.hpp), bricks in 3-D
//                Morton order
//   C3 scatter   second pass: 32-byte records {x, y, z, h}, {a, box, lx, ly} (the box
//                clipped to the brick and the column offsets, formed here) into their
//                bricks' runs; a wave's (particle, brick) pairs dealt one per lane, paired
//                stores through an LDS stage
//   C4 deposit   one workgroup per work item, largest first: fp64 LDS brick accumulator
//                (64 KiB + a spare plane); records classified by their box's column count,
//                boxes of <= 48 columns lane-per-record, wider ones a wave per record with
//                lanes over the columns; each column walks only its sphere's planes (packed
//                fp32 pairs for the edge kernels; the indicator kernel keeps the oracle's
//                fp64 test: bit-exact neighbour sets); the term A*W is fp32, summed in fp64
//   C5 merge     bricks split over several items: fp64 slab sum in slab order
// A call may produce a slab of planes [k_lo, k_hi) only (Z-slab ownership across GPUs,
// asp_amd.distributed.project3d_sharded).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/asp.h"
#include "asp_binning.hpp"
#include "asp_device.hpp"
#include "asp_host.hpp"

namespace asp {

// Brick edge (voxels); z fastest.  16 x 16 x 32: two 512-thread deposit workgroups per
// CU.  32 x 16 x 32 (build switch ASP_CUBE_BX=32; one 1024-thread workgroup per CU, the
// 128-KiB brick) cuts the records to 1.28 per particle (1.39) and halves the scatter's
// open brick runs -- scatter 3.76 -> 3.21 ms -- but the deposit ran 9.94 -> 11.15 ms and
// the merge 0.07 -> 0.25 ms (round 5)
#ifndef ASP_CUBE_BX
#define ASP_CUBE_BX 16
#endif
constexpr int kBX = ASP_CUBE_BX, kBY = 16, kBZ = 32;
constexpr int kBXs = kBX == 32 ? 5 : 4, kBYs = 4, kBZs = 5;
static_assert(kBX == 1 << kBXs, "brick edge in x: 16 or 32");
constexpr int kBrickVox = kBX * kBY * kBZ;   // 8192 -> 64 KiB of fp64 accumulators
#ifndef ASP_CUBE_PAD
#define ASP_CUBE_PAD 1
#endif
#ifndef ASP_CUBE_PLANES
#define ASP_CUBE_PLANES 1
#endif
#ifndef ASP_CUBE_ODD_MASK
#define ASP_CUBE_ODD_MASK 0  // 1: mask the odd column's extra plane-pair add (A/B switch)
#endif
// LDS accumulator layout.  Plane-major (ASP_CUBE_PLANES, default): voxel (i, j, k) at
// k * 256 + i * 16 + j, so a plane is 256 doubles = 8 x 64 banks and a voxel's bank pair
// depends on its column only -- the lanes of a wave walking adjacent columns from
// different first planes never share a bank pair.  Column-major (0): rows of a column
// padded to kBZP doubles (a 32-double row stride put the same k of adjacent columns in
// one bank), the bank then shifting with each lane's first plane.
constexpr int kBZP = kBZ + ASP_CUBE_PAD;
static_assert(ASP_CUBE_PLANES || ASP_CUBE_PAD >= 1, "column-major: the pad word takes plane kBZ");
constexpr int kPlane = kBX * kBY;
constexpr int kKStride = ASP_CUBE_PLANES ? kPlane : 1;  // LDS step from plane k to k + 1
// (plane-major: one spare plane kBZ after the brick, the odd-length columns' last pair)
constexpr int kBrickLds = ASP_CUBE_PLANES ? (kBZ + 1) * kPlane : kBX * kBY * kBZP;
__device__ __forceinline__ int lds_at(int li, int lj, int lk) {
    return ASP_CUBE_PLANES ? lk * kPlane + li * kBY + lj : (li * kBY + lj) * kBZP + lk;
}
__device__ __forceinline__ int lds_vox(int v) {  // dense brick index -> padded LDS index
    return lds_at(v >> (kBYs + kBZs), (v >> kBZs) & (kBY - 1), v & (kBZ - 1));
}
constexpr int kMaxBricks = 16384;            // C1/C3 LDS: one int per brick (64 KiB)
static_assert(kMaxBricks <= kScanThreads * kScanPer, "k_tilescan holds <= kScanPer bricks per thread");
constexpr int k3Block = 512;                 // count / scatter / merge workgroup
constexpr int kStage3 = 136;                 // scatter: float4 staging per wave (paired stores)
constexpr int kDBlock = 2 * kBX * kBY;       // deposit workgroup: two threads per brick column
#ifndef ASP_CUBE_LANE_COLS
#define ASP_CUBE_LANE_COLS 48
#endif
constexpr int kLaneCols = ASP_CUBE_LANE_COLS;  // boxes up to this many (i, j) columns:
                                               // lane-per-record, wider: a wave per record

// Deposit rounds: records classified per round (LDS list of 2-byte indices) and the
// classes (0: boxes of more than lane_cols columns, 1..kNCCls + 1: lane-per-record boxes by
// column count, large to small)
#ifndef ASP_CUBE_ROUND
#define ASP_CUBE_ROUND 4096
#endif
constexpr int kRound = ASP_CUBE_ROUND;
// Lane classes by the box's column count (round 5): a lane-per-record wave runs
// max-over-lanes column steps, so records of similar column counts go together.  The box
// volume classes before (80 / 32 / 12) mixed column counts within a class (CPU model:
// tools/sim/cube_classes.py): deposit 11.84 -> 11.07 ms (same process; thresholds 36 / 25 / 16 / 9 / 4 against 10 or 13 finer ones
// and 40 / 30 / 20 / 12 / 6: 11.07-11.30 ms).
#ifndef ASP_CUBE_CCLS
#define ASP_CUBE_CCLS 36, 25, 16, 9, 4
#endif
constexpr int kCCls[] = {ASP_CUBE_CCLS};  // descending: class 1 + #{t : cols <= t}
constexpr int kNCCls = sizeof(kCCls) / sizeof(int);
constexpr int kQCls = 2 + kNCCls;  // the wave class, then the lane classes large to small
#ifndef ASP_CUBE_WAVE_TAKE
#define ASP_CUBE_WAVE_TAKE 32
#endif
constexpr int kWaveTake = ASP_CUBE_WAVE_TAKE;  // wave-class records claimed at a time
static_assert(kRound % kDBlock == 0 && kRound <= 65536, "round of whole blocks, 16-bit index");

struct Grid3 {
    double x_min, y_min, z_min;
    double px, py, pz;       // (max - min) / n per axis
    double ipx, ipy, ipz;    // reciprocals (candidate boxes only)
    int nx, ny, nz;
    int k_lo, nzl;           // output planes [k_lo, k_lo + nzl)
    int i_lo, nxl;           // this pass's window of x planes [i_lo, i_lo + nxl) (i_lo a
                             // multiple of kBX; the whole slab unless it has > kMaxBricks)
    int nbx, nby, nbz, nb;   // bricks over the output slab
    int lane_cols;           // deposit: boxes up to this many columns lane-per-record
    int diag;                // timing diagnostic (ASP_CUBE_DIAG): 1 skip the wave class, 2 the lane classes
};

struct Box3 {
    int i0, i1, j0, j1, k0, k1;  // inclusive voxel ranges (absolute indices)
};

// A particle's voxel box in fp32: a superset of the voxels its sphere can reach, with a
// margin (2^-20 relative to the operand magnitudes in cells, plus 2^-10 cell) far above
// the fp32 roundings of the operands and products (< 2^-21 relative).  The box only
// bounds what is walked -- every voxel in it is still tested (fp64 for the indicator
// kernel, the edge form for the others) -- so any superset is exact, for the deposit's
// walk and for the bricks count and scatter bin a particle to (round 4: an fp64 form
// before, count 0.52 -> 0.44 ms).
struct Grid3f {
    float x_min, y_min, z_min, ipx, ipy, ipz;
};
__device__ __forceinline__ bool axis_cells_f(float w, float rad, float w_min, float ip, int lo,
                                             int hi, int& a, int& b) {
    const float t0 = (w - rad - w_min) * ip, t1 = (w + rad - w_min) * ip;
    const float d = (fabsf(w) + rad + fabsf(w_min)) * ip * 0x1p-20f + 0x1p-10f;
    const float f0 = fmaxf(ceilf(t0 - d), (float)lo);
    const float f1 = fminf(floorf(t1 + d), (float)hi);
    if (!(f0 <= f1)) return false;
    a = (int)f0;
    b = (int)f1;
    return true;
}
__device__ __forceinline__ bool footprint3f(const Grid3& g, const Grid3f& f, float x, float y,
                                            float z, float h, Box3& b) {
    const float rad = fabsf(2.0f * h);
    if (!(rad > 0.0f) || !__builtin_isfinite(rad)) return false;
    if (!__builtin_isfinite(x) || !__builtin_isfinite(y) || !__builtin_isfinite(z)) return false;
    return axis_cells_f(x, rad, f.x_min, f.ipx, g.i_lo, g.i_lo + g.nxl - 1, b.i0, b.i1) &&
           axis_cells_f(y, rad, f.y_min, f.ipy, 0, g.ny - 1, b.j0, b.j1) &&
           axis_cells_f(z, rad, f.z_min, f.ipz, g.k_lo, g.k_lo + g.nzl - 1, b.k0, b.k1);
}

__device__ __forceinline__ void load3(const float* __restrict__ x, const float* __restrict__ y,
                                      const float* __restrict__ z, const float* __restrict__ h,
                                      long long p, long long p1, float& px, float& py, float& pz,
                                      float& ph) {
    // unconditional loads, index clamped to the range (p1 >= 1): loads under a branch made
    // the compiler wait (vmcnt(0)) for every load and store in flight at the top of each
    // batch, the prefetched batch included
    const long long q = p < p1 ? p : p1 - 1;
    px = x[q];
    py = y[q];
    pz = z[q];
    const float hq = h[q];
    ph = p < p1 ? hq : 0.0f;  // h = 0: no footprint
}

// ----------------------------------------------------------------------------------
// C1: count insertions per (block, brick)
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(k3Block) void k3_count(const float* __restrict__ x,
                                                    const float* __restrict__ y,
                                                    const float* __restrict__ z,
                                                    const float* __restrict__ h, long long n,
                                                    long long per_block, Grid3 g,
                                                    int* __restrict__ hist, int inter) {
    extern __shared__ __attribute__((aligned(16))) int lh[];
    for (int t = threadIdx.x; t < g.nb; t += k3Block) lh[t] = 0;
    __syncthreads();
    // inter: block b takes the k3Block-particle batches b, b + nblk, ... (the whole grid
    // streams one window of the arrays at a time, as the 2-D count does); else one
    // contiguous range per block
    const long long stride = inter ? (long long)gridDim.x * k3Block : k3Block;
    const long long p0 = inter ? (long long)blockIdx.x * k3Block : (long long)blockIdx.x * per_block;
    const long long p1 = inter ? n : min(n, p0 + per_block);
    const Grid3f gf = {(float)g.x_min, (float)g.y_min, (float)g.z_min,
                       (float)g.ipx, (float)g.ipy, (float)g.ipz};
    auto bin = [&](float cx, float cy, float cz, float ch) {
        Box3 b;
        if (footprint3f(g, gf, cx, cy, cz, ch, b)) {
            int bi0 = (b.i0 - g.i_lo) >> kBXs, bi1 = (b.i1 - g.i_lo) >> kBXs;
            int bj0 = b.j0 >> kBYs, bj1 = b.j1 >> kBYs;
            int bk0 = (b.k0 - g.k_lo) >> kBZs, bk1 = (b.k1 - g.k_lo) >> kBZs;
            for (int bi = bi0; bi <= bi1; ++bi)
                for (int bj = bj0; bj <= bj1; ++bj)
                    for (int bk = bk0; bk <= bk1; ++bk)
                        atomicAdd(&lh[(bi * g.nby + bj) * g.nbz + bk], 1);
        }
    };
    // three particle buffers in rotation, two batches ahead: a copy of the next batch into
    // the current one at the loop's back edge made the compiler wait for its loads there,
    // so one batch was in flight at a time (round 5)
    float ax, ay, az, ah, bx, by, bz, bh, cx, cy, cz, ch;
    load3(x, y, z, h, p0 + threadIdx.x, p1, ax, ay, az, ah);
    load3(x, y, z, h, p0 + stride + threadIdx.x, p1, bx, by, bz, bh);
    for (long long base = p0; base < p1; base += 3 * stride) {
        load3(x, y, z, h, base + 2 * stride + threadIdx.x, p1, cx, cy, cz, ch);
        bin(ax, ay, az, ah);
        if (base + stride >= p1) break;  // block-uniform
        load3(x, y, z, h, base + 3 * stride + threadIdx.x, p1, ax, ay, az, ah);
        bin(bx, by, bz, bh);
        if (base + 2 * stride >= p1) break;
        load3(x, y, z, h, base + 4 * stride + threadIdx.x, p1, bx, by, bz, bh);
        bin(cx, cy, cz, ch);
    }
    __syncthreads();
    int* row = hist + (long long)blockIdx.x * g.nb;
    for (int t = threadIdx.x; t < g.nb; t += k3Block) row[t] = lh[t];
}

// ----------------------------------------------------------------------------------
// C3: scatter 32-byte records {x, y, z, h}, {a, box, lx, ly} into the bricks' runs
// ----------------------------------------------------------------------------------
// The record's second half: a, the particle's box clipped to brick (bi, bj, bk) in
// brick-local voxels (5 bits per bound: i0 i1 j0 j1 k0 k1), and the fp32 offsets of the
// particle from the box's first column, fl32(x - X[I0 + i0]), fl32(y - Y[J0 + j0]) -- formed
// here, where the brick is known, by the expressions the deposit used to evaluate from the
// particle (same fp64 operations, so identical bits): the deposit's classification and
// record set-up no longer recompute the footprint (round 5).  The box's
// clip to the cube (TW / TH / TD) is implied: footprint3f already clips to the slab.
__device__ __forceinline__ float4 rec_half1(const Grid3& g, int bi0, int bi1, int bj0, int bj1,
                                            int bk0, int bk1, int bi, int bj, int bk, float x,
                                            float y, float a) {
    const int I0 = g.i_lo + bi * kBX, J0 = bj * kBY, K0 = g.k_lo + bk * kBZ;
    const int i0 = max(bi0 - I0, 0), i1 = min(bi1 - I0, kBX - 1);
    const int j0 = max(bj0 - J0, 0), j1 = min(bj1 - J0, kBY - 1);
    const int k0 = max(bk0 - K0, 0), k1 = min(bk1 - K0, kBZ - 1);
    const unsigned bits = (unsigned)i0 | (unsigned)i1 << 5 | (unsigned)j0 << 10 |
                          (unsigned)j1 << 15 | (unsigned)k0 << 20 | (unsigned)k1 << 25;
    const float lx = (float)((double)x - (g.x_min + (double)(I0 + i0) * g.px));
    const float ly = (float)((double)y - (g.y_min + (double)(J0 + j0) * g.py));
    return make_float4(a, __uint_as_float(bits), lx, ly);
}
__device__ __forceinline__ Box3 rec_box(float bits_f) {
    const unsigned v = __float_as_uint(bits_f);
    return Box3{(int)(v & 31), (int)(v >> 5 & 31), (int)(v >> 10 & 31),
                (int)(v >> 15 & 31), (int)(v >> 20 & 31), (int)(v >> 25 & 31)};
}
// TB = GRP x k3Block threads: scatter workgroup b takes the batches of count workgroups
// GRP b .. GRP b + GRP - 1 (interleaved: batch r nblk + GRP b + g, g < GRP, is one
// contiguous range of TB particles; contiguous: their adjacent ranges), so its runs are
// the union of theirs -- GRP x fewer (workgroup, brick) runs open at once (the scatter's
// record stores cost with the number of open runs; 512 workgroups of 512
// -> 256 of 1024: scatter 3.91 -> 3.62 ms at 10^8 / 512^3, count unchanged).
template <int PROBE, int TB>  // PROBE 1: the placement trials' launches (asp_project2d.hip k_scatter)
__global__ __launch_bounds__(TB) void k3_scatter(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
    const float* __restrict__ h, const float* __restrict__ a, long long n, long long per_block,
    Grid3 g, const int* __restrict__ hist, const long long* __restrict__ brick_start,
    float4* __restrict__ recs, int inter, const int* __restrict__ ctr, long long rec_cap) {
    // speculative launch (enqueued before the host has read the record count): a no-op
    // when the records would not fit the buffer it was given
    if ((long long)ctr[cRecs] > rec_cap) return;
    extern __shared__ __attribute__((aligned(16))) int cur[];
    float4* stage = (float4*)(cur + ((g.nb + 3) & ~3)) + (threadIdx.x >> 6) * kStage3;
    constexpr int GRP = TB / k3Block;
    const int* row = hist + (long long)blockIdx.x * GRP * g.nb;
    for (int t = threadIdx.x; t < g.nb; t += TB) cur[t] = (int)brick_start[t] + row[t];
    __syncthreads();
    // the count's batch assignment (k3_count), GRP count workgroups at a time
    const long long stride = inter ? (long long)gridDim.x * TB : TB;
    const long long p0 = inter ? (long long)blockIdx.x * TB : (long long)blockIdx.x * GRP * per_block;
    const long long p1 = inter ? n : min(n, p0 + GRP * per_block);
    const Grid3f gf = {(float)g.x_min, (float)g.y_min, (float)g.z_min,
                       (float)g.ipx, (float)g.ipy, (float)g.ipz};
    // A wave's (particle, brick) pairs are dealt 64 per round, one per lane, so every
    // store instruction is full.  Nested brick loops per lane ran max-over-lanes
    // iterations with few lanes active (1.39 records per particle, ~6 iterations per wave
    // at 10^8 / 512^3: 23 % of the store lanes busy).  Round 5: scatter 3.96 -> 3.91 ms,
    // 3.83 -> 3.62 with the grouped workgroups.
    const int lane = threadIdx.x & 63;
    // Paired store (as the 2-D scatter): the wave's records staged in LDS (first halves at
    // [lane], second halves at [72 + lane]: no bank conflicts either way), then lanes 2j and
    // 2j + 1 write the two 16-B halves of record j, so one store instruction covers 32
    // whole 32-B records instead of 64 half records.  slot < 0: no record.  Called by the
    // whole wave.
    auto pstore = [&](int slot, const float4& r0, const float4& r1) {
        stage[lane] = r0;
        stage[72 + lane] = r1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int src = half * 32 + (lane >> 1);
            const int sl = __shfl(slot, src);
            const float4 v = stage[(lane & 1) * 72 + src];
            if (sl >= 0) {
                recs[2 * (long long)sl + (lane & 1)] = v;
                asm volatile("" ::: "memory");  // one dwordx4 store per half record
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    auto bin = [&](float cx, float cy, float cz, float ch, float ca) {
        Box3 b = {};
        int nbr = 0, bi0 = 0, bj0 = 0, bk0 = 0, nj = 1, nk = 1;
        if (footprint3f(g, gf, cx, cy, cz, ch, b)) {
            bi0 = (b.i0 - g.i_lo) >> kBXs;
            bj0 = b.j0 >> kBYs;
            bk0 = (b.k0 - g.k_lo) >> kBZs;
            nj = (b.j1 >> kBYs) - bj0 + 1;
            nk = ((b.k1 - g.k_lo) >> kBZs) - bk0 + 1;
            nbr = (((b.i1 - g.i_lo) >> kBXs) - bi0 + 1) * nj * nk;
        }
        if (__ballot(nbr > 1) == 0) {  // one brick at most per lane: one record each
            const int slot = nbr ? atomicAdd(&cur[(bi0 * g.nby + bj0) * g.nbz + bk0], 1) : -1;
            pstore(slot, make_float4(cx, cy, cz, ch),
                   rec_half1(g, b.i0, b.i1, b.j0, b.j1, b.k0, b.k1, bi0, bj0, bk0, cx, cy, ca));
            return;
        }
        // the box's six absolute bounds are dealt unpacked (any cube edge: a 16-bit packing
        // overflowed the sign bit from voxel 32768 on)
        int incl = nbr;  // inclusive scan of the pair counts over the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d) incl += v;
        }
        const int total = __shfl(incl, 63), excl = incl - nbr;
        for (int r = 0; r < total; r += 64) {
            const int p = r + lane;
            int s = 0;  // the pair's source lane: the number of lanes with incl <= p
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1)
                if (__shfl(incl, s + st - 1) <= p) s += st;
            const float fx = __shfl(cx, s), fy = __shfl(cy, s), fz = __shfl(cz, s);
            const float fh = __shfl(ch, s), fa = __shfl(ca, s);
            const int sj = __shfl(nj, s), sk = __shfl(nk, s);
            const int q = p - __shfl(excl, s);
            const int t = q / sk, dk = q - t * sk, di = t / sj, dj = t - di * sj;
            const int bi = __shfl(bi0, s) + di, bj = __shfl(bj0, s) + dj, bk = __shfl(bk0, s) + dk;
            const int i0 = __shfl(b.i0, s), i1 = __shfl(b.i1, s), j0 = __shfl(b.j0, s);
            const int j1 = __shfl(b.j1, s), k0 = __shfl(b.k0, s), k1 = __shfl(b.k1, s);
            const int slot = p < total ? atomicAdd(&cur[(bi * g.nby + bj) * g.nbz + bk], 1) : -1;
            pstore(slot, make_float4(fx, fy, fz, fh),
                   rec_half1(g, i0, i1, j0, j1, k0, k1, bi, bj, bk, fx, fy, fa));
        }
    };
    // Two particle buffers in ping-pong (no register copies at the loop's back edge, which
    // made the compiler wait for every load and store in flight before it could issue the
    // next batch's loads): batch j + 1 is loaded while batch j is binned.
    float ax, ay, az, ah, aa, bx, by, bz, bh, ba;
    load3(x, y, z, h, p0 + threadIdx.x, p1, ax, ay, az, ah);
    aa = a[min(p0 + (long long)threadIdx.x, p1 - 1)];  // (unused where h = 0)
    for (long long base = p0; base < p1; base += 2 * stride) {
        long long q = base + stride + threadIdx.x;
        load3(x, y, z, h, q, p1, bx, by, bz, bh);
        ba = a[min(q, p1 - 1)];
        bin(ax, ay, az, ah, aa);
        if (base + stride >= p1) break;  // block-uniform
        q = base + 2 * stride + threadIdx.x;
        load3(x, y, z, h, q, p1, ax, ay, az, ah);
        aa = a[min(q, p1 - 1)];
        bin(bx, by, bz, bh, ba);
    }
}

// ----------------------------------------------------------------------------------
// C4: deposit one work item (a run of records of one brick) into the LDS brick
// ----------------------------------------------------------------------------------
struct Rec3 {
    double x, y, z, thr;  // fp64 copies of the fp32 inputs; thr = (2h)^2 in fp64
    float hinv, s;        // 1 / h, a * norm(h)
    float kc;             // brick-local plane coordinate of z, (z - z_min) / pz - K0
    float lx, ly;         // fl32(x - X[i0]), fl32(y - Y[j0]): offsets from the box's first column
    float zr, thrf;       // fl32(z - Z[0]) (from the brick's first plane), fl32(thr)
    Box3 b;               // clipped to the brick, brick-local indices
};

// Edge-continuous kernels (cubic, Wendland) take no per-voxel decision (as the 2-D gather,
// DESIGN.md §3): edge_shape2 (asp_device.hpp) gives exactly 0 for q >= 2, evaluated in fp32
// from fp32 plane offsets, two planes per packed instruction, so a voxel whose exact test
// differs contributes < 2^-60 W(0).  The indicator kernel keeps the fp64 test (bit-exact
// voxel counts).

// One (i, j) column of a record's box.  The oracle's test is
//   r2 = dx * dx + dy * dy + dz * dz  <  (2h)^2      (voxel_pass, left to right in fp64)
// so s = dx * dx + dy * dy is the same intermediate for every k of the column, and only
// the k with |dz| <= sqrt(thr - s) can pass.  That range is widened to a superset (the
// rounding of s + dz^2 allows |dz|^2 up to thr - s + ~2 eps thr; 8 eps thr is added, and
// axis_cells adds its 2^-40 relative + 2^-20 cell margin) and each k in it gets the exact
// test, so neighbour sets stay bit-exact while the box corners outside the sphere
// (about half of a box at physical h) are never visited.
// the candidate planes [a, b] (brick-local) of column (li, lj); s = its dx^2 + dy^2.
// The half-width sqrt(thr - s + 2^-49 thr) / pz is formed in fp32: its relative error
// (< 2^-21) and that of kc (< 2^-24 of 512 planes) stay far inside the margin of
// 2^-10 plane + 2^-18 relative, so [a, b] remains a superset of the passing planes.
__device__ __forceinline__ bool column_range(const Grid3& g, const Rec3& R, int li, int lj,
                                             const double* xt, const double* yt, double& s,
                                             int& a, int& b) {
    double dx = R.x - xt[li];
    double dy = R.y - yt[lj];
    s = dx * dx + dy * dy;
    if (!(s < R.thr)) return false;  // s + dz * dz >= s >= thr for every k
    float rz = __builtin_amdgcn_sqrtf((float)((R.thr - s) + R.thr * 0x1p-49)) * (float)g.ipz;
    rz = rz * (1.0f + 0x1p-18f) + 0x1p-10f;
    float fa = fmaxf(ceilf(R.kc - rz), (float)R.b.k0);
    float fb = fminf(floorf(R.kc + rz), (float)R.b.k1);
    if (!(fa <= fb)) return false;
    a = (int)fa;
    b = (int)fb;
    return true;
}

template <int KID>
__device__ __forceinline__ void voxel3(const Rec3& R, double s, int li, int lj, int lk,
                                       const double* zt, double* acc) {
    double dz = R.z - zt[lk];
    double r2 = s + dz * dz;
    if (r2 < R.thr) {
        float q = __builtin_amdgcn_sqrtf((float)r2) * R.hinv;
        float w = kernel_shape<KID>(q);
        atomicAdd(&acc[lds_at(li, lj, lk)], (double)(R.s * w));
    }
}

// The plane walk of one column, planes [a, b] (brick-local), edge-continuous kernels: in
// units of h, q = sqrt(dz'^2 + s') with dz' = (zr - k pz) / h and s' = s / h^2 formed once
// per column, and the term's coefficient folded into the shape's last factor (Wendland:
// t^4 (c + 2c q)) -- two packed operations fewer per plane pair than q = sqrt(r2) / h and
// f(q) * c.  col: the column's plane-0 word; sfh = s'; zh = (z - Z[0]) / h; pzh = -pz / h;
// sc = the term coefficient x kShapeScale.
template <int KID>
__device__ __forceinline__ void plane_walk(double* col, float fa, float fb, float sfh, float zh,
                                           float pzh, float sc) {
    const f2 zr2 = {zh, zh}, npz = {pzh, pzh}, sf2 = {sfh, sfh};
    const f2 sc2 = {sc, sc}, sc22 = {2.0f * sc, 2.0f * sc};
    auto planes2 = [&](f2 pl) {
        const f2 dz = __builtin_elementwise_fma(pl, npz, zr2);
        const f2 r2 = __builtin_elementwise_fma(dz, dz, sf2);
        const f2 q = f2{__builtin_amdgcn_sqrtf(r2.x), __builtin_amdgcn_sqrtf(r2.y)};
        if constexpr (KID == 1) {  // Wendland C2: c t^4 (1 + 2q) = t^4 (c + 2c q)
            const f2 t = pk_one_minus_half_clamp(q);
            const f2 t2 = t * t;
            return (t2 * t2) * __builtin_elementwise_fma(sc22, q, sc2);
        } else {
            return edge_shape2<KID>(q) * sc2;
        }
    };
    // whole plane pairs, no odd last plane: a column of odd length also adds plane fb + 1,
    // where the term is 0 (beyond the sphere: the range is a superset of its planes and the
    // box's last plane is the sphere's, the brick's or the slab's) or lands in the brick's
    // spare plane kBZ / a plane past the slab, neither ever read out.  The plane numbers are
    // small integers in fp32 (exact), so the packed pair doubles as the loop counter.
    f2 lk2 = {fa, fa + 1.0f};
    double* p = col + (int)fa * kKStride;
    for (; lk2.x <= fb; lk2 += (f2){2.0f, 2.0f}, p += 2 * kKStride) {
        const f2 w = planes2(lk2);
        atomicAdd(p, (double)w.x);
#if ASP_CUBE_ODD_MASK
        if (lk2.y <= fb)  // the odd column's extra plane: no LDS add (the LDS pipe is shared)
#endif
            atomicAdd(p + kKStride, (double)w.y);
    }
}

// Per-record constants of the edge-continuous column walk, formed once per record (the
// walk's loops then hold them in registers).
struct ColE {
    float tin;       // fl32(thr) (1 + 2^-20): columns with s below can meet the sphere
    float tpe;       // fl32(thr) (1 + 2^-19)
    float rzs;       // 1 / pz (1 + 2^-18)
    float kc, k0f, k1f;
    float h2, zh, pzh, sc;
};
template <int KID>
__device__ __forceinline__ ColE col_consts(const Grid3& g, const Rec3& R) {
    ColE K;
    K.tin = R.thrf * (1.0f + 0x1p-20f);
    K.tpe = R.thrf * (1.0f + 0x1p-19f);
    K.rzs = (float)g.ipz * (1.0f + 0x1p-18f);
    K.kc = R.kc;
    K.k0f = (float)R.b.k0;
    K.k1f = (float)R.b.k1;
    K.h2 = R.hinv * R.hinv;
    K.zh = R.zr * R.hinv;
    K.pzh = -(float)g.pz * R.hinv;
    K.sc = R.s * kShapeScale<KID>;
    return K;
}

// One column of an edge-continuous kernel: s = dx^2 + dy^2 in fp32 (offsets from the box's
// first column, column3), its plane range, the walk.  column3's half-width argument
// max(thr - s, 0) + thr 2^-20 is replaced by thr (1 + 2^-19) - s, never smaller for the
// columns that pass (s < thr (1 + 2^-20)), so the range stays a superset; the scale and the
// margin are one fma.
template <int KID>
__device__ __forceinline__ void column_e(const ColE& K, double* col, float sf) {
    if (!(sf < K.tin)) return;  // the column misses the sphere
    const float rz = fmaf(__builtin_amdgcn_sqrtf(K.tpe - sf), K.rzs, 0x1p-10f);
    // clamps by v_med3 (an fmaxf / fminf re-canonicalised the per-record bound in every
    // column: one instruction each)
    const float fa = __builtin_amdgcn_fmed3f(ceilf(K.kc - rz), K.k0f, 0x1p30f);
    const float fb = __builtin_amdgcn_fmed3f(floorf(K.kc + rz), -0x1p30f, K.k1f);
    if (!(fa <= fb)) return;
    plane_walk<KID>(col, fa, fb, sf * K.h2, K.zh, K.pzh, K.sc);
}

template <int KID>
__device__ __forceinline__ void column3(const Grid3& g, const Rec3& R, int li, int lj, int K0,
                                        const double* xt, const double* yt, const double* zt,
                                        double* acc) {
    if constexpr (KID == 2) {
        double s;
        int a, b;
        if (!column_range(g, R, li, lj, xt, yt, s, a, b)) return;
        for (int lk = a; lk <= b; ++lk) voxel3<KID>(R, s, li, lj, lk, zt, acc);
    } else {  // fp32 throughout: the column's plane range and dz, no decision
        // offsets from the box's first column in fp32 (no LDS corner reads per column):
        // within 2^-24 (|lx| + 16 pitches) of the exact ones, ~2^-20 of h for these boxes
        const float dx = fmaf(-(float)(li - R.b.i0), (float)g.px, R.lx);
        const float dy = fmaf(-(float)(lj - R.b.j0), (float)g.py, R.ly);
        column_e<KID>(col_consts<KID>(g, R), acc + lds_at(li, lj, 0), fmaf(dx, dx, dy * dy));
    }
}

template <int KID>
__global__ __launch_bounds__(kDBlock) void k3_deposit(Grid3 g, const float4* __restrict__ recs,
                                                      const Item* __restrict__ items,
                                                      const int* __restrict__ order,
                                                      double* __restrict__ slabs,
                                                      float* __restrict__ out, int accumulate) {
    extern __shared__ __attribute__((aligned(16))) double acc[];
    double* xt = acc + kBrickLds;
    double* yt = xt + kBX;
    double* zt = yt + kBY;
    __shared__ unsigned short qlist[kRound];  // the round's record indices, by class
    __shared__ int qmeta[3 * kQCls];
    // largest items first (the tilescan's dispatch order, as the 2-D deposit): the split
    // central bricks' items, ~16x the average work, no longer start late and finish last
    const Item it = items[order ? order[blockIdx.x] : blockIdx.x];
    int bi = it.tile / (g.nby * g.nbz);
    int rem = it.tile - bi * (g.nby * g.nbz);
    int bj = rem / g.nbz, bk = rem - (rem / g.nbz) * g.nbz;
    int I0 = g.i_lo + bi * kBX, J0 = bj * kBY, K0 = g.k_lo + bk * kBZ;
    int TW = min(kBX, g.i_lo + g.nxl - I0), TH = min(kBY, g.ny - J0), TD = min(kBZ, g.k_lo + g.nzl - K0);
    auto out_index = [&](int v) -> long long {
        int li = v >> (kBYs + kBZs), lj = (v >> kBZs) & (kBY - 1), lk = v & (kBZ - 1);
        if (li >= TW || lj >= TH || lk >= TD) return -1;
        return ((long long)(I0 - g.i_lo + li) * g.ny + (J0 + lj)) * g.nzl + (K0 - g.k_lo + lk);
    };
    if (it.count == 0) {  // empty brick
        if (accumulate) return;
        for (int v = threadIdx.x; v < kBrickVox; v += kDBlock) {
            long long o = out_index(v);
            if (o >= 0) out[o] = 0.0f;
        }
        return;
    }
    for (int v = threadIdx.x; v < kBrickLds; v += kDBlock) acc[v] = 0.0;
    if (threadIdx.x < kBX) xt[threadIdx.x] = g.x_min + (double)(I0 + (int)threadIdx.x) * g.px;
    else if (threadIdx.x < kBX + kBY)
        yt[threadIdx.x - kBX] = g.y_min + (double)(J0 + (int)threadIdx.x - kBX) * g.py;
    else if (threadIdx.x < kBX + kBY + kBZ)
        zt[threadIdx.x - kBX - kBY] = g.z_min + (double)(K0 + (int)threadIdx.x - kBX - kBY) * g.pz;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // A record's state for the walk: its box clipped to the brick (brick-local), the fp64
    // centre and threshold, 1/h, the term coefficient and the brick-local plane of z.
    auto prep = [&](const float4& q0, const float4& q1, Rec3& R) -> bool {
        R.b = rec_box(q1.y);  // clipped to the brick by the scatter (rec_half1)
        R.x = q0.x;
        R.y = q0.y;
        R.z = q0.z;
        double t = 2.0 * (double)q0.w;
        R.thr = t * t;
        R.hinv = 1.0f / q0.w;
        R.s = (float)term_coef<KID>(q1.x, q0.w);
        R.kc = (float)((R.z - g.z_min) * g.ipz - (double)K0);
        R.lx = q1.z;
        R.ly = q1.w;
        R.zr = (float)(R.z - (g.z_min + (double)K0 * g.pz));
        R.thrf = (float)R.thr;
        return true;
    };
    // The item's records are taken in rounds of kRound.  Each round is first CLASSIFIED:
    // boxes of more than lane_cols columns (a wave walks each) and kNCCls + 1 classes of
    // the lane-per-record boxes by column count; the record indices are counting-sorted by class
    // into an LDS list.  Then every wave repeatedly claims a chunk of one class (the wave
    // class first, then the lane classes from large to small boxes) until the round is
    // exhausted: a wave's 64 lanes walk boxes of similar size, where records in arrival
    // order put a wave at the pace of its largest box (modelled lane utilisation of the
    // lane path 0.21 -> 0.5, tools/sim/cube_lanes.py).  No barrier inside a round.
    int* qcnt = qmeta;             // records per class
    int* qhead = qmeta + kQCls;    // claimed so far
    int* qoff = qmeta + 2 * kQCls; // class start in qlist
    for (int r0i = 0; r0i < it.count; r0i += kRound) {
        const int nr = min(kRound, it.count - r0i);
        if (threadIdx.x < kQCls) {
            qcnt[threadIdx.x] = 0;
            qhead[threadIdx.x] = 0;
        }
        __syncthreads();
        unsigned cr[kRound / kDBlock];  // class << 16 | rank, per record of this thread
        // all of this thread's records of the round loaded first: loads interleaved with
        // the class counters' LDS atomics were issued one at a time, each waiting a full
        // memory latency (vmcnt(0)) before the next (round 5)
        // the class from the box the scatter stored in the record's second half
        float qv[kRound / kDBlock];
#pragma unroll
        for (int q = 0; q < kRound / kDBlock; ++q)
            qv[q] = recs[2 * (it.start + r0i + min(q * kDBlock + (int)threadIdx.x, nr - 1)) + 1].y;
#pragma unroll
        for (int q = 0; q < kRound / kDBlock; ++q) {
            const int i = q * kDBlock + (int)threadIdx.x;
            int c = -1;
            if (i < nr) {
                const Box3 b = rec_box(qv[q]);
                const int cols = (b.i1 - b.i0 + 1) * (b.j1 - b.j0 + 1);
                c = 1;
#pragma unroll
                for (int t = 0; t < kNCCls; ++t) c += cols <= kCCls[t];
                if (cols > g.lane_cols) c = 0;
                if ((g.diag == 1 && c == 0) || (g.diag == 2 && c > 0)) c = -1;
            }
            cr[q] = c < 0 ? 0xffffffffu : ((unsigned)c << 16) | (unsigned)atomicAdd(&qcnt[c], 1);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int o = 0;
            for (int c = 0; c < kQCls; ++c) {
                qoff[c] = o;
                o += qcnt[c];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kRound / kDBlock; ++q)
            if (cr[q] != 0xffffffffu)
                qlist[qoff[cr[q] >> 16] + (cr[q] & 0xffffu)] =
                    (unsigned short)(q * kDBlock + (int)threadIdx.x);
        __syncthreads();
        // claim chunks: the wave class kWaveTake records at a time (each is walked by the
        // whole wave), the lane classes 64 at a time (one per lane).  The next chunk is
        // claimed and its records loaded before the current one is walked.
        int ccls = 0;  // claim cursor: the class being claimed from (wave-uniform)
        // records claimed at a time: the wave class kWaveTake (each walked by the whole
        // wave), the lane classes 64 (one per lane)
        auto take = [](int c) { return c == 0 ? kWaveTake : 64; };
        auto claim = [&](int& cls, int& base) {
            while (ccls < kQCls) {
                int b0 = 0;
                if (lane == 0) b0 = atomicAdd(&qhead[ccls], take(ccls));
                b0 = __shfl(b0, 0);
                if (b0 < qcnt[ccls]) {
                    cls = ccls;
                    base = b0;
                    return;
                }
                ++ccls;
            }
            cls = kQCls;  // exhausted
            base = 0;
        };
        auto fetch = [&](int cls, int base, int& i, float4& q0, float4& q1) {
            const bool have = cls < kQCls && lane < take(cls) &&
                              base + lane < qcnt[min(cls, kQCls - 1)];
            i = have ? (int)qlist[qoff[cls] + base + lane] : -1;
            const long long ri = it.start + r0i + max(i, 0);  // unconditional load
            q0 = recs[2 * ri];
            q1 = recs[2 * ri + 1];
        };
        int cls, base, i;
        float4 q0, q1;
        claim(cls, base);
        fetch(cls, base, i, q0, q1);
        while (cls < kQCls) {
            int ncls, nbase, ni;
            float4 n0, n1;
            claim(ncls, nbase);
            fetch(ncls, nbase, ni, n0, n1);
            Rec3 R = {};
            const bool live = i >= 0 && prep(q0, q1, R);
            const int bw = R.b.i1 - R.b.i0 + 1, bh = R.b.j1 - R.b.j0 + 1;
            if (cls > 0) {  // lane classes: lane-per-record
                // one flat loop over the box's columns: a wave runs max(bw * bh) column
                // steps, where nested i / j loops ran about max(bw) * max(bh) over its lanes
                if (live) {
                    const int nc = bw * bh;
                    int li = R.b.i0, lj = R.b.j0;
                    if constexpr (KID == 2) {
                        for (int c = 0; c < nc; ++c) {
                            column3<KID>(g, R, li, lj, K0, xt, yt, zt, acc);
                            if (++lj > R.b.j1) {
                                lj = R.b.j0;
                                ++li;
                            }
                        }
                    } else {
                        // the record's constants once; the column offsets stepped (one
                        // subtraction per column instead of two conversions and two fma:
                        // <= 16 roundings of ~2^-24 |d|, a value effect only)
                        const ColE K = col_consts<KID>(g, R);
                        const float px = (float)g.px, py = (float)g.py;
                        float dx = R.lx, dy = R.ly;
                        for (int c = 0; c < nc; ++c) {
                            column_e<KID>(K, acc + lds_at(li, lj, 0), fmaf(dx, dx, dy * dy));
                            if (++lj > R.b.j1) {
                                lj = R.b.j0;
                                ++li;
                                dy = R.ly;
                                dx -= px;
                            } else {
                                dy -= py;
                            }
                        }
                    }
                }
            } else {
                unsigned long long big = __ballot(live);
                if constexpr (KID != 2) {
                    // each record's column constants formed by its own lane (all 64 at
                    // once), then broadcast: the whole wave forming them per record cost
                    // ~10 VALU per wave-class record, as did the first column's division
                    const ColE Kl = col_consts<KID>(g, R);
                    const float px = (float)g.px, py = (float)g.py;
                    while (big) {
                        const int l = __builtin_ctzll(big);
                        big &= big - 1;
                        ColE K;
                        K.tin = bcast(Kl.tin, l);
                        K.tpe = bcast(Kl.tpe, l);
                        K.rzs = Kl.rzs;  // (the same for every record)
                        K.kc = bcast(Kl.kc, l);
                        K.k0f = bcast(Kl.k0f, l);
                        K.k1f = bcast(Kl.k1f, l);
                        K.h2 = bcast(Kl.h2, l);
                        K.zh = bcast(Kl.zh, l);
                        K.pzh = bcast(Kl.pzh, l);
                        K.sc = bcast(Kl.sc, l);
                        const float lx = bcast(R.lx, l), ly = bcast(R.ly, l);
                        const int i0 = bcast(R.b.i0, l), j0 = bcast(R.b.j0, l);
                        const int qw = bcast(bw, l), qh = bcast(bh, l);
                        // column cc = ci * qh + cj; a lane's first (ci, cj) by fp32 (exact:
                        // (lane + 1/2) / qh is never within 1/32 of an integer), its next 64
                        // columns on by increments
                        const int di = 64 / qh, dj = 64 - di * qh;
                        int ci = (int)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)qh));
                        int cj = lane - ci * qh;
                        for (int cc = lane; cc < qw * qh; cc += 64) {
                            const float dx = fmaf(-(float)ci, px, lx), dy = fmaf(-(float)cj, py, ly);
                            column_e<KID>(K, acc + lds_at(i0 + ci, j0 + cj, 0), fmaf(dx, dx, dy * dy));
                            ci += di;
                            cj += dj;
                            if (cj >= qh) {
                                cj -= qh;
                                ++ci;
                            }
                        }
                    }
                }
                while (KID == 2 && big) {
                    int l = __builtin_ctzll(big);
                    big &= big - 1;
                    Rec3 Q = {};
                    Q.x = __shfl(R.x, l);
                    Q.y = __shfl(R.y, l);
                    Q.z = __shfl(R.z, l);
                    Q.thr = __shfl(R.thr, l);
                    Q.hinv = bcast(R.hinv, l);
                    Q.s = bcast(R.s, l);
                    Q.kc = bcast(R.kc, l);
                    Q.lx = bcast(R.lx, l);
                    Q.ly = bcast(R.ly, l);
                    Q.zr = bcast(R.zr, l);
                    Q.thrf = bcast(R.thrf, l);
                    Q.b.i0 = bcast(R.b.i0, l);
                    Q.b.j0 = bcast(R.b.j0, l);
                    Q.b.k0 = bcast(R.b.k0, l);
                    Q.b.k1 = bcast(R.b.k1, l);
                    int qw = bcast(bw, l), qh = bcast(bh, l);
                    // lanes take the box's (i, j) columns: column cc = ci * qh + cj, the
                    // next one of a lane 64 further on (one division per record, not per column)
                    const int di = 64 / qh, dj = 64 - di * qh;
                    int ci = lane / qh, cj = lane - ci * qh;
                    for (int cc = lane; cc < qw * qh; cc += 64) {
                        column3<KID>(g, Q, Q.b.i0 + ci, Q.b.j0 + cj, K0, xt, yt, zt, acc);
                        ci += di;
                        cj += dj;
                        if (cj >= qh) {
                            cj -= qh;
                            ++ci;
                        }
                    }
                }
            }
            cls = ncls;
            base = nbase;
            i = ni;
            q0 = n0;
            q1 = n1;
        }
        __syncthreads();  // the round's list is reused by the next round
    }
    if constexpr (ASP_CUBE_PLANES) {
        // thread t: column c = t mod 256, planes [kh, kh + 16) -- conflict-free LDS reads
        // (adjacent lanes, adjacent columns), 16 consecutive outputs per thread
        static_assert(kDBlock == 2 * kPlane && kBZ == 32, "two half-columns per thread pair");
        const int c = (int)threadIdx.x & (kPlane - 1), kh = ((int)threadIdx.x / kPlane) * (kBZ / 2);
        if (it.slab >= 0) {  // dense brick order (c * kBZ + k), as k3_merge reads it
            double* dst = slabs + (long long)it.slab * kBrickVox + c * kBZ + kh;
#pragma unroll
            for (int q = 0; q < kBZ / 2; ++q) dst[q] = acc[(kh + q) * kPlane + c];
            return;
        }
        const int li = c >> kBYs, lj = c & (kBY - 1);
        if (li >= TW || lj >= TH) return;
        float* o = out + ((long long)(I0 - g.i_lo + li) * g.ny + (J0 + lj)) * g.nzl + (K0 - g.k_lo) + kh;
        const int nq = min(kBZ / 2, TD - kh);
        for (int q = 0; q < nq; ++q) {
            const float val = (float)acc[(kh + q) * kPlane + c];
            o[q] = accumulate ? o[q] + val : val;
        }
        return;
    }
    if (it.slab >= 0) {
        double* dst = slabs + (long long)it.slab * kBrickVox;
        for (int v = threadIdx.x; v < kBrickVox; v += kDBlock) dst[v] = acc[lds_vox(v)];
        return;
    }
    for (int v = threadIdx.x; v < kBrickVox; v += kDBlock) {
        long long o = out_index(v);
        if (o < 0) continue;
        float val = (float)acc[lds_vox(v)];
        out[o] = accumulate ? out[o] + val : val;
    }
}

// C5: bricks split over several items -- fp64 sum of their slabs in slab order.
__global__ __launch_bounds__(k3Block) void k3_merge(Grid3 g, const Merge* __restrict__ merges,
                                                    const double* __restrict__ slabs,
                                                    float* __restrict__ out, int accumulate) {
    const Merge m = merges[blockIdx.x];
    int bi = m.tile / (g.nby * g.nbz);
    int rem = m.tile - bi * (g.nby * g.nbz);
    int bj = rem / g.nbz, bk = rem - (rem / g.nbz) * g.nbz;
    int I0 = g.i_lo + bi * kBX, J0 = bj * kBY, K0 = g.k_lo + bk * kBZ;
    int TW = min(kBX, g.i_lo + g.nxl - I0), TH = min(kBY, g.ny - J0), TD = min(kBZ, g.k_lo + g.nzl - K0);
    for (int v = threadIdx.x; v < kBrickVox; v += k3Block) {
        int li = v >> (kBYs + kBZs), lj = (v >> kBZs) & (kBY - 1), lk = v & (kBZ - 1);
        if (li >= TW || lj >= TH || lk >= TD) continue;
        double s = 0.0;
        for (int j = 0; j < m.nslab; ++j) s += slabs[(long long)(m.slab0 + j) * kBrickVox + v];
        long long o = ((long long)(I0 - g.i_lo + li) * g.ny + (J0 + lj)) * g.nzl + (K0 - g.k_lo + lk);
        float val = (float)s;
        out[o] = accumulate ? out[o] + val : val;
    }
}

// ----------------------------------------------------------------------------------
// Host side
// ----------------------------------------------------------------------------------
static uint32_t spread3(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3ff;
    v = (v | (v << 16)) & 0x030000ff;
    v = (v | (v << 8)) & 0x0300f00f;
    v = (v | (v << 4)) & 0x030c30c3;
    v = (v | (v << 2)) & 0x09249249;
    return v;
}

static int ensure_morton3(Workspace& ws, const Grid3& g, hipStream_t st) {
    if (ws.morton3_key[0] == g.nbx && ws.morton3_key[1] == g.nby && ws.morton3_key[2] == g.nbz)
        return ASP_OK;
    std::vector<std::pair<uint32_t, int>> key((size_t)g.nb);
    for (int bi = 0; bi < g.nbx; ++bi)
        for (int bj = 0; bj < g.nby; ++bj)
            for (int bk = 0; bk < g.nbz; ++bk) {
                int t = (bi * g.nby + bj) * g.nbz + bk;
                key[t] = {spread3(bi) << 2 | spread3(bj) << 1 | spread3(bk), t};
            }
    std::sort(key.begin(), key.end());
    std::vector<int> order(key.size());
    for (size_t i = 0; i < key.size(); ++i) order[i] = key[i].second;
    ASP_TRY(ensure(ws.morton3, order.size() * sizeof(int)));
    ASP_HIP(hipMemcpyAsync(ws.morton3.p, order.data(), order.size() * sizeof(int),
                           hipMemcpyHostToDevice, st));
    ASP_HIP(hipStreamSynchronize(st));
    ws.morton3_key[0] = g.nbx;
    ws.morton3_key[1] = g.nby;
    ws.morton3_key[2] = g.nbz;
    return ASP_OK;
}

static bool make_grid3(const double* ext, int nx, int ny, int nz, int k_lo, int k_hi,
                       Grid3& g) {
    if (!(nx > 0 && ny > 0 && nz > 0) || k_lo < 0 || k_hi > nz || k_lo >= k_hi) return false;
    for (int a = 0; a < 3; ++a)
        if (!std::isfinite(ext[2 * a]) || !std::isfinite(ext[2 * a + 1]) ||
            !(ext[2 * a + 1] > ext[2 * a]))
            return false;
    g.x_min = ext[0];
    g.y_min = ext[2];
    g.z_min = ext[4];
    g.px = (ext[1] - ext[0]) / nx;
    g.py = (ext[3] - ext[2]) / ny;
    g.pz = (ext[5] - ext[4]) / nz;
    if (!(g.px > 0.0 && g.py > 0.0 && g.pz > 0.0)) return false;
    g.ipx = 1.0 / g.px;
    g.ipy = 1.0 / g.py;
    g.ipz = 1.0 / g.pz;
    if (!std::isfinite(g.ipx) || !std::isfinite(g.ipy) || !std::isfinite(g.ipz)) return false;
    g.nx = nx;
    g.ny = ny;
    g.nz = nz;
    g.k_lo = k_lo;
    g.nzl = k_hi - k_lo;
    g.i_lo = 0;
    g.nxl = nx;
    g.nbx = (nx + kBX - 1) / kBX;
    g.nby = (ny + kBY - 1) / kBY;
    g.nbz = (g.nzl + kBZ - 1) / kBZ;
    long long nb = (long long)g.nbx * g.nby * g.nbz;
    // more bricks than one pass holds: windows of whole brick columns in x (window3); -1:
    // not even one brick column fits
    g.nb = (long long)g.nby * g.nbz > kMaxBricks ? -1 : (int)std::min<long long>(nb, 0x7fffffff);
    g.lane_cols = kLaneCols;
    if (const char* e = getenv("ASP_CUBE_LANE_COLS")) g.lane_cols = std::max(0, atoi(e));
    g.diag = getenv("ASP_CUBE_DIAG") ? atoi(getenv("ASP_CUBE_DIAG")) : 0;
    return true;
}

// internal: >= 2^31 records in one pass.  The speculative scatter (enqueued before the
// counters are read) may already have written records into the spare capacity of the
// existing buffer; the caller's split discards them.
constexpr int kRetSplit3 = 1;

// One window (w.i_lo, w.nxl; <= kMaxBricks bricks) of the cube on stream st: count,
// scans, scatter (placement trials on a fresh record buffer), deposit, merge.
static int cube_pass(Workspace& ws, const Grid3& g, const float* dx, const float* dy,
                     const float* dz, const float* dh, const float* da, long long n, int kid,
                     int acc, float* dout, hipStream_t st, long long* agg) {
    long long n_recs = 0;
    int n_items = 0, n_merges = 0, n_slabs = 0;
    ASP_TRY(ensure_morton3(ws, g, st));
    // count workgroups (scatter workgroups: half as many), at most 384 (round 6, same process
    // at 10^8: 512 / 384 / 256 / 128 -> cube 13.92-13.96 / 13.86-13.87 / 14.46-14.48 / 17.9 ms:
    // fewer scatter workgroups keep fewer (workgroup, brick) runs open, scatter 3.61 -> 3.44,
    // count 0.41 -> 0.54); ASP_CUBE_BLOCKS overrides (read per call)
    const long long max_blk = getenv("ASP_CUBE_BLOCKS") ? std::max(2, atoi(getenv("ASP_CUBE_BLOCKS"))) : 384;
    long long nblk = std::min<long long>(max_blk, std::max<long long>(1, (n + 8191) / 8192));
    // batch-interleaved count / scatter (ASP_CUBE_INTERLEAVE=0: contiguous ranges per block)
    static const int inter = getenv("ASP_CUBE_INTERLEAVE") ? atoi(getenv("ASP_CUBE_INTERLEAVE")) : 1;
    long long per_block = (n + nblk - 1) / nblk;
    nblk = (n + per_block - 1) / per_block;
    ASP_TRY(ensure(ws.hist, (size_t)nblk * g.nb * sizeof(int)));
    ASP_TRY(ensure(ws.tile_total, (size_t)g.nb * sizeof(int)));
    ASP_TRY(ensure(ws.tile_start, (size_t)g.nb * sizeof(long long)));
    // target item count: 1024 (round 5; 512 / 1024 / 2048 / 4096: deposit + merge 10.45 /
    // 9.99-10.04 / 10.06 / 10.15 ms, same process -- fewer split bricks, fewer fp64 slabs
    // to write and merge); ASP_CUBE_ITEMS overrides (read per call)
    int target = 1024;
    if (const char* e = getenv("ASP_CUBE_ITEMS")) target = std::max(64, atoi(e));
    ASP_TRY(ensure(ws.items, (size_t)(g.nb + target + 16) * sizeof(Item)));
    ASP_TRY(ensure(ws.iorder, (size_t)(g.nb + target + 16) * sizeof(int)));
    const bool morton_order = getenv("ASP_CUBE_ITEM_ORDER") && atoi(getenv("ASP_CUBE_ITEM_ORDER")) == 0;  // A/B
    int* iord = morton_order ? nullptr : (int*)ws.iorder.p;
    ASP_TRY(ensure(ws.merges, (size_t)(g.nb + 16) * sizeof(Merge)));
    ASP_TRY(ensure(ws.counters, cNum * sizeof(int)));
    if (!ws.h_counters) ASP_HIP(hipHostMalloc((void**)&ws.h_counters, kMarks * cNum * sizeof(int)));
    int* dc = (int*)ws.counters.p;
    ASP_HIP(hipMemsetAsync(dc, 0, cNum * sizeof(int), st));
    const size_t lds_bins = (size_t)g.nb * sizeof(int);
    {
        StageMark m(ws, kS3Count, st);
        hipLaunchKernelGGL(k3_count, dim3((unsigned)nblk), dim3(k3Block), lds_bins, st, dx, dy,
                           dz, dh, n, per_block, g, (int*)ws.hist.p, inter);
        ASP_LAUNCHED();
        m.done();
    }
    {
        StageMark m(ws, kS3Colscan, st);
        hipLaunchKernelGGL(k_colscan, dim3((g.nb + 63) / 64), dim3(kColscanBlock), 0, st,
                           (int*)ws.hist.p, (int)nblk, g.nb, (int*)ws.tile_total.p, (int)nblk);
        ASP_LAUNCHED();
        m.done();
    }
    {
        StageMark m(ws, kS3Tilescan, st);
        if (g.nb <= 4 * kScanThreads)
            hipLaunchKernelGGL(k_tilescan<4>, dim3(1), dim3(kScanThreads), 0, st,
                           (const int*)ws.tile_total.p, (const int*)ws.morton3.p, g.nb, 1,
                           (long long*)ws.tile_start.p, (Item*)ws.items.p,
                           (Merge*)ws.merges.p, dc, iord, 0, target);
        else
            hipLaunchKernelGGL(k_tilescan<kScanPer>, dim3(1), dim3(kScanThreads), 0, st,
                           (const int*)ws.tile_total.p, (const int*)ws.morton3.p, g.nb, 1,
                           (long long*)ws.tile_start.p, (Item*)ws.items.p,
                           (Merge*)ws.merges.p, dc, iord, 0, target);
        ASP_LAUNCHED();
        m.done();
    }
    auto scatter_launch = [&](bool probe, long long cap) -> int {
        StageMark m(ws, kS3Scatter, st);
        // grouped workgroups (GRP 2) need an even count grid; ASP_CUBE_SGRP=1: one count
        // workgroup per scatter workgroup (A/B switch, read per call)
        const char* ge = getenv("ASP_CUBE_SGRP");
        const bool g2 = (ge ? atoi(ge) != 1 : true) && nblk % 2 == 0;
        auto kern = g2 ? (probe ? k3_scatter<1, 2 * k3Block> : k3_scatter<0, 2 * k3Block>)
                       : (probe ? k3_scatter<1, k3Block> : k3_scatter<0, k3Block>);
        const int tb = g2 ? 2 * k3Block : k3Block;
        const size_t lds_sc = (size_t)((g.nb + 3) & ~3) * sizeof(int) +
                              (size_t)(tb / 64) * kStage3 * sizeof(float4);
        // (the largest: 16384 bricks + 16 waves' staging, so the attribute is set once)
        ASP_TRY(allow_dyn_lds((const void*)kern, (size_t)kMaxBricks * sizeof(int) +
                                                     (size_t)(tb / 64) * kStage3 * sizeof(float4)));
        hipLaunchKernelGGL(kern, dim3((unsigned)(g2 ? nblk / 2 : nblk)), dim3(tb), lds_sc, st, dx,
                           dy, dz, dh, da, n, per_block, g, (const int*)ws.hist.p,
                           (const long long*)ws.tile_start.p, (float4*)ws.recs.p, inter,
                           (const int*)dc, cap);
        ASP_LAUNCHED();
        m.done();
        return ASP_OK;
    };
    auto scatter = [&](bool probe) { return scatter_launch(probe, 0x7ffffffeLL); };
    // One small read-back sizes the buffers.  With a record buffer left by an earlier call,
    // the scatter is enqueued BEFORE the host waits for the counters (it checks them against
    // that buffer's capacity itself), so the GPU does not idle across the host round trip
    // (as the 2-D path, asp_project2d.hip).
    ASP_TRY(ensure_side(ws));  // (its events)
    ASP_HIP(hipMemcpyAsync(ws.h_counters, dc, cNum * sizeof(int), hipMemcpyDeviceToHost, st));
    ASP_HIP(hipEventRecord(ws.cnt_ev, st));
    const long long rec_cap =
        (long long)std::min<size_t>(ws.recs.cap / (2 * sizeof(float4)), 0x7ffffffe);
    const bool spec = ws.recs.p != nullptr && getenv("ASP_NO_SPECULATE") == nullptr;
    if (spec) ASP_TRY(scatter_launch(false, rec_cap));
    ASP_HIP(hipEventSynchronize(ws.cnt_ev));
    n_items = ws.h_counters[cItems];
    n_recs = ws.h_counters[cRecs];
    n_slabs = ws.h_counters[cSlabs];
    n_merges = ws.h_counters[cMerges];
    long long rec_limit = 0x7fffffffLL;  // 32-bit record cursors (ASP_MAX_RECORDS: tests)
    if (const char* e = getenv("ASP_MAX_RECORDS")) rec_limit = std::max(1LL, atoll(e));
    if (n_recs >= rec_limit) {  // the caller splits (a speculative scatter wrote into spare room)
        if (spec) ASP_HIP(hipStreamSynchronize(st));
        return kRetSplit3;
    }
    const bool pre = spec && n_recs <= rec_cap;  // the speculative scatter did the work
    if (spec && !pre) ASP_HIP(hipStreamSynchronize(st));  // its no-op is done: buffer free
    const void* recs_before = ws.recs.p;
    ASP_TRY(ensure(ws.recs, (size_t)n_recs * 2 * sizeof(float4)));
    ASP_TRY(ensure(ws.slabs, (size_t)n_slabs * kBrickVox * sizeof(double)));
    bool placed = pre;  // a fresh record buffer: placement trials (asp_host.hpp)
    if (!pre && ws.recs.p != recs_before)
        ASP_TRY(place_records(ws, (size_t)n_recs * 2 * sizeof(float4), st,
                              [&]() { return scatter(true); }, placed));
    if (!placed) ASP_TRY(scatter(false));
    {
        StageMark m(ws, kS3Deposit, st);
        size_t lds = (size_t)kBrickLds * sizeof(double) + (kBX + kBY + kBZ) * sizeof(double);
        auto kern = kid == 0 ? k3_deposit<0> : kid == 1 ? k3_deposit<1> : k3_deposit<2>;
        ASP_TRY(allow_dyn_lds((const void*)kern, lds));
        hipLaunchKernelGGL(kern, dim3(n_items), dim3(kDBlock), lds, st, g,
                           (const float4*)ws.recs.p, (const Item*)ws.items.p, (const int*)iord,
                           (double*)ws.slabs.p, dout, acc);
        ASP_LAUNCHED();
        m.done();
    }
    if (n_merges > 0) {
        StageMark m(ws, kS3Merge, st);
        hipLaunchKernelGGL(k3_merge, dim3(n_merges), dim3(k3Block), 0, st, g,
                           (const Merge*)ws.merges.p, (const double*)ws.slabs.p, dout, acc);
        ASP_LAUNCHED();
        m.done();
    }
    agg[0] += n_recs;
    agg[1] += n_items;
    agg[2] += n_merges;
    agg[3] += n_slabs;
    return ASP_OK;
}

static int project3d(const float* x, const float* y, const float* z, const float* h,
                     const float* a, long long n, const double* ext, int nx, int ny, int nz,
                     int k_lo, int k_hi, int kid, int flags, float* out, int device,
                     void* stream) {
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (kid < 0 || kid > 2) return fail(ASP_ERR_INVALID, "unknown kernel_id");
    if (!out) return fail(ASP_ERR_INVALID, "out is NULL");
    if (flags & ~(ASP_F_DEVICE_PTRS | ASP_F_ACCUMULATE))
        return fail(ASP_ERR_UNSUPPORTED, "asp_project3d supports ASP_F_DEVICE_PTRS and "
                                         "ASP_F_ACCUMULATE only");
    if (n > 0 && (!x || !y || !z || !h || !a)) return fail(ASP_ERR_INVALID, "NULL particle array");
    Grid3 g;
    if (!make_grid3(ext, nx, ny, nz, k_lo, k_hi, g))
        return fail(ASP_ERR_INVALID,
                    "invalid cube: need nx, ny, nz >= 1, 0 <= k_lo < k_hi <= nz and finite "
                    "max > min on every axis");
    if (g.nb < 0)
        return fail(ASP_ERR_UNSUPPORTED, "cube slab too wide: ny x (k_hi - k_lo) spans more than "
                                         "16384 16x32 brick columns; split the planes [k_lo, k_hi)");
    if (device < 0 || device >= 64) return fail(ASP_ERR_INVALID, "bad device");
    int ndev = 0;
    ASP_HIP(hipGetDeviceCount(&ndev));
    if (device >= ndev) return fail(ASP_ERR_INVALID, "device index out of range");
    ASP_HIP(hipSetDevice(device));
    hipStream_t st = (hipStream_t)stream;
    // a workspace slot per stream, as the 2-D maps have (asp_host.hpp map_slot): cubes on
    // two streams overlap -- one cube's store-bound scatter beside the other's VALU-bound
    // deposit (round 5)
    Workspace& ws = slot_ws(device, map_slot(device, st));
    std::lock_guard<std::mutex> lock(ws.mu);
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
    const bool dev = flags & ASP_F_DEVICE_PTRS;
    const int acc = (flags & ASP_F_ACCUMULATE) ? 1 : 0;
    const long long nvox = (long long)nx * ny * g.nzl;
    const float *dx = x, *dy = y, *dz = z, *dh = h, *da = a;
    float* dout = out;
    if (!dev) {
        const float* src[5] = {x, y, z, h, a};
        for (int k = 0; k < 5; ++k) {
            ASP_TRY(ensure(ws.in[k], (size_t)n * sizeof(float)));
            if (n > 0)
                ASP_HIP(hipMemcpyAsync(ws.in[k].p, src[k], (size_t)n * sizeof(float),
                                       hipMemcpyHostToDevice, st));
        }
        dx = (const float*)ws.in[0].p;
        dy = (const float*)ws.in[1].p;
        dz = (const float*)ws.in[2].p;
        dh = (const float*)ws.in[3].p;
        da = (const float*)ws.in[4].p;
        ASP_TRY(ensure(ws.out[0], (size_t)nvox * sizeof(float)));
        dout = (float*)ws.out[0].p;
        if (acc)
            ASP_HIP(hipMemcpyAsync(dout, out, nvox * sizeof(float), hipMemcpyHostToDevice, st));
    }
    if (ws.prof) ASP_TRY(prof_next(ws));
    long long agg[4] = {0, 0, 0, 0};  // records, items, merges, slabs over the windows
    if (n == 0) {
        if (!acc) {
            StageMark m(ws, kSMemset, st);
            ASP_HIP(hipMemsetAsync(dout, 0, nvox * sizeof(float), st));
            m.done();
        }
    } else {
        // windows of whole brick columns in x, each <= kMaxBricks bricks: every window one
        // pass over all particles with the footprints clipped to it; its slab of the output
        // is contiguous ((nx, ny, nzl) C-order, x slowest)
        const int wb = std::max(1, kMaxBricks / (g.nby * g.nbz));
        for (int bx0 = 0; bx0 < g.nbx; bx0 += wb) {
            Grid3 w = g;
            w.i_lo = bx0 * kBX;
            w.nxl = std::min((bx0 + wb) * kBX, nx) - w.i_lo;
            w.nbx = std::min(wb, g.nbx - bx0);
            w.nb = w.nbx * g.nby * g.nbz;
            // particle batches of < 2^31 (ASP_MAX_BATCH), halved while a pass would reach
            // 2^31 records; batches after the first accumulate
            long long B = 1LL << 30;
            if (const char* e = getenv("ASP_MAX_BATCH")) B = std::max(1LL, atoll(e));
            std::vector<std::pair<long long, long long>> todo;
            for (long long a = ((n - 1) / B) * B; a >= 0; a -= B) todo.push_back({a, std::min(n, a + B)});
            int passes = 0;
            while (!todo.empty()) {
                const auto [a, b] = todo.back();
                todo.pop_back();
                const int rc = cube_pass(ws, w, dx + a, dy + a, dz + a, dh + a, da + a, b - a,
                                         kid, passes ? 1 : acc,
                                         dout + (long long)w.i_lo * ny * g.nzl, st, agg);
                if (rc == kRetSplit3) {
                    if (b - a < 2)
                        return fail(ASP_ERR_UNSUPPORTED, "one particle makes >= 2^31 records");
                    todo.push_back({a + (b - a) / 2, b});
                    todo.push_back({a, a + (b - a) / 2});
                    continue;
                }
                ASP_TRY(rc);
                ++passes;
            }
        }
    }
    if (!dev) {
        ASP_HIP(hipMemcpyAsync(out, dout, nvox * sizeof(float), hipMemcpyDeviceToHost, st));
        ASP_HIP(hipStreamSynchronize(st));
    }
    ws.stats[0] = agg[0];
    ws.stats[1] = agg[1];
    ws.stats[2] = 0;
    ws.stats[3] = kBrickVox;
    ws.stats[4] = (long long)g.nbx * g.nby * g.nbz;
    ws.stats[5] = n > 0 ? ws.h_counters[cChunk] : 0;
    ws.stats[6] = agg[2];
    ws.stats[7] = agg[3];
    ws.stats[8] = n > 0 ? 1 : 0;
    for (int k = 9; k < kNStats; ++k) ws.stats[k] = 0;  // 2-D-only counters
    if (&ws != &g_ws[device]) {  // asp_last_stats reads slot 0 (under its lock, as in 2-D)
        std::lock_guard<std::mutex> lk(g_ws[device].mu);
        std::copy(ws.stats, ws.stats + kNStats, g_ws[device].stats);
    }
    return ws_end_.finish();
}

}  // namespace asp

using namespace asp;

extern "C" int asp_project3d(const float* x, const float* y, const float* z, const float* h,
                             const float* a, int64_t n, double x_min, double x_max, double y_min,
                             double y_max, double z_min, double z_max, int32_t nx, int32_t ny,
                             int32_t nz, int32_t k_lo, int32_t k_hi, int32_t kernel_id,
                             int32_t flags, float* out, int32_t device, void* stream) {
    t_err.clear();
    const double ext[6] = {x_min, x_max, y_min, y_max, z_min, z_max};
    return project3d(x, y, z, h, a, n, ext, nx, ny, nz, k_lo, k_hi, kernel_id, flags, out, device,
                     stream);
}
