// asp_device.hpp -- device-side building blocks of the projector (gfx950 / CDNA4).
//
// Reference semantics restated here (paths under /root/reference/src/astro_sph_tools/):
//   pixel corner        tools/projections/_pixel_calculations.pyx:11-14
//   neighbour test      tools/projections/_pixel_calculations.pyx:30-31  (r2 < (2h)^2)
//   chunk (tile) cull   tools/projections/_projector.py:34-48
//   kernel              tools/projections/_kernels.pyx:9-20
//
// Neighbour membership is decided EXACTLY as the reference decides it in fp64, at fp32
// cost: the fp32 test r2_32 < thr_32 is trusted whenever |r2_32 - thr_32| exceeds a
// rigorous per-record error band; pairs inside the band (~0.1 % near the 2h edge) are
// re-decided by the reference's own fp64 arithmetic, including the chunk cull.  See
// DESIGN.md §3 for the bound.
//
// Accumulation.  LDS fp32 atomics run ~8x slower than fp64 or integer
// ones on gfx950 (tools/microbench_lds.hip), so tiles accumulate either
//  * kAccF64 (default): fp32 terms A*W added in fp64 with ds_add_f64 -- more precise than
//    the fp32 map it produces; or
//  * kAccFix (ASP_F_DETERMINISTIC): terms scaled by a per-tile power of two, rounded to
//    int64 and added with ds_add_u64.  Integer sums are associative, so maps are bitwise
//    reproducible regardless of scheduling and input order.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace asp {

constexpr int kBlock = 256;        // threads per workgroup for streaming kernels
constexpr int kDepBlock = 512;     // deposit workgroup (8 waves; 2 per CU at 64 KiB LDS)
constexpr int kTile = 64;          // GPU tile edge in pixels
constexpr int kTileShift = 6;
#ifndef ASP_WIDE_TILES
#define ASP_WIDE_TILES 256
#endif
constexpr int kWideTiles = ASP_WIDE_TILES;  // particles overlapping more tiles take the wide path
constexpr int kScaleBits = 61;     // per-tile bound n_t * max|c| maps to <= 2^61
constexpr int kAccF64 = 0;         // LDS fp64 accumulation
constexpr int kAccFix = 1;         // LDS int64 fixed point (deterministic)

struct Grid {
    double x_min, y_min;
    double psx;       // (x_max - x_min) / nx                        _projector.py:34
    double psy_pix;   // (y_max - y_min) / nx  (S2 quirk)            .pyx:12
    double psy_cull;  // (y_max - y_min) / ny                        _projector.py:35
    float xminf, yminf;   // fp32 copies for the candidate-box estimate
    float ipsx, ipsy;     // fp32 reciprocal pitches (pixel pitches)
    float mg;         // bound on |corner coordinate| over the grid (error band)
    int nx, ny, cs;
    int ncx, ncy;     // reference chunks per axis
    int ntx, nty, ntiles;  // GPU tiles
    int nonsquare;    // nx != ny: the y chunk cull is not implied by the r2 test
    int band_cols;    // records spanning >= this many tile columns: row-band deposit
    int nstream;      // 2: second record run per tile for them (histogram columns x 2)
    int wide_tiles;   // particles over more tiles than this take the wide path (K6)
};

struct Box {
    int x0, x1, y0, y1;  // inclusive pixel ranges
};

// Per-record state for the pair loop.
struct Prep {
    float u, v, h;
    float lo;    // fp32 r2 < lo: inside for sure;  lo <= r2 <= hi: decide in fp64;
    float hi;    // r2 > hi: outside  (lo, hi = (2h)^2 -/+ error band; +-inf: always fp64)
    float hinv;  // 1/h
    float s0, s1;  // a * norm(h) (kAccF64) or a * norm(h) * 2^k_tile (kAccFix)
    float thr;   // (2h)^2 in fp32
    float band;  // |r2 - thr| <= band: the fp32 decision is not trusted (inf: never)
    Box b;
};

struct Item {       // one deposit work item: a run of records of one GPU tile
    long long start;
    int tile;
    int count;      // 0: empty tile (write zeros)
    int slab;       // -1: the tile's only item (writes the map); >= 0: int64 partial slab
    int mode;       // 0: regular records; 1: large records (2-D map, gathered)
};

struct Merge {      // a tile split over several items: sum their slabs
    int tile;
    int slab0;
    int nslab;
    int pad;
};

__device__ __forceinline__ double corner_x(const Grid& g, int xi) {
    return g.x_min + (double)xi * g.psx;            // .pyx:13
}
__device__ __forceinline__ double corner_y(const Grid& g, int yi) {
    return g.y_min + (double)yi * g.psy_pix;        // .pyx:14
}

// _projector.py:38-48 for the chunk holding pixel (xi, yi).  fp64, reference order:
// (w_min + chunk_start * pitch) - 2*h  <=  w  <  (w_min + chunk_end * pitch) + 2*h.
__device__ __forceinline__ bool cull_pass(const Grid& g, double u, double v, double h,
                                          int xi, int yi) {
    int xi0 = (xi / g.cs) * g.cs, yi0 = (yi / g.cs) * g.cs;
    int xe = min(xi0 + g.cs, g.nx), ye = min(yi0 + g.cs, g.ny);
    double h2 = 2.0 * h;
    double xlo = g.x_min + (double)xi0 * g.psx, xhi = g.x_min + (double)xe * g.psx;
    double ylo = g.y_min + (double)yi0 * g.psy_cull, yhi = g.y_min + (double)ye * g.psy_cull;
    return (u >= xlo - h2) && (u < xhi + h2) && (v >= ylo - h2) && (v < yhi + h2);
}

// Inclusive range of chunk indices whose cull accepts coordinate w (one axis).  Both
// bounds are monotone in the chunk index, so the set is an interval: estimate, then walk
// to the exact edges with the reference formula.
__device__ __forceinline__ void chunk_range(double w, double h, double w_min, double ps,
                                            int npx, int cs, int& c_lo, int& c_hi) {
    int nc = (npx + cs - 1) / cs;
    double h2 = 2.0 * h;
    c_lo = 0;
    c_hi = -1;
    if (!__builtin_isfinite(w) || !__builtin_isfinite(h)) return;
    auto lo_ok = [&](int c) { return w >= (w_min + (double)(c * cs) * ps) - h2; };
    auto hi_ok = [&](int c) {
        int e = min((c + 1) * cs, npx);
        return w < (w_min + (double)e * ps) + h2;
    };
    double est = floor((w + h2 - w_min) / ((double)cs * ps));
    int cmax = est < -1.0 ? -1 : (est > nc - 1.0 ? nc - 1 : (int)est);
    while (cmax >= 0 && !lo_ok(cmax)) --cmax;
    while (cmax + 1 <= nc - 1 && lo_ok(cmax + 1)) ++cmax;
    double est2 = ceil((w - h2 - w_min) / ((double)cs * ps)) - 1.0;
    int cmin = est2 < 0.0 ? 0 : (est2 > (double)nc ? nc : (int)est2);
    while (cmin <= nc - 1 && !hi_ok(cmin)) ++cmin;
    while (cmin - 1 >= 0 && hi_ok(cmin - 1)) --cmin;
    c_lo = cmin;
    c_hi = cmax;
}

// Candidate pixel box of a particle: a superset of the pixels that can pass the exact
// test.  fp32 estimate of (w - 2|h| - w_min) / pitch with a margin delta that bounds its
// rounding error: at most ~6 roundings of 2^-24 relative to (|w| + |w_min| + 2|h|) / pitch
// (w_min and 1/pitch to fp32, the difference, the product, the two offsets), so 2^-20
// leaves a 2.7x margin; plus 2^-12 px so that a corner at exactly 2h stays a candidate.
// (A wider margin makes more pixel-scale boxes 4 corners wide, which leave the fast 3 x 3
// deposit.)  False when nothing can pass.
__device__ __forceinline__ bool footprint(const Grid& g, float u, float v, float h, Box& b) {
    float hd = fabsf(2.0f * h);
    if (!(hd > 0.0f) || !__builtin_isfinite(hd)) {
        // h == 0: r2 < 0 never holds (S12).  Non-finite: excluded.
        // |2h| overflowing fp32 only happens for non-finite h (|h| < 1.7e38).
        return false;
    }
    if (!__builtin_isfinite(u) || !__builtin_isfinite(v)) return false;
    float cx = (u - g.xminf) * g.ipsx, rx = hd * g.ipsx;
    float cy = (v - g.yminf) * g.ipsy, ry = hd * g.ipsy;
    float dx = (fabsf(u) + fabsf(g.xminf) + hd) * g.ipsx * 0x1p-20f + 0x1p-12f;
    float dy = (fabsf(v) + fabsf(g.yminf) + hd) * g.ipsy * 0x1p-20f + 0x1p-12f;
    float fx0 = fmaxf(ceilf(cx - rx - dx), 0.0f);
    float fx1 = fminf(floorf(cx + rx + dx), (float)(g.nx - 1));
    float fy0 = fmaxf(ceilf(cy - ry - dy), 0.0f);
    float fy1 = fminf(floorf(cy + ry + dy), (float)(g.ny - 1));
    if (!(fx0 <= fx1) || !(fy0 <= fy1)) return false;
    b.x0 = (int)fx0;
    b.x1 = (int)fx1;
    b.y0 = (int)fy0;
    b.y1 = (int)fy1;
    if (g.nonsquare) {  // S2: the y cull pitch differs from the pixel pitch
        int c0, c1;
        chunk_range((double)v, (double)h, g.y_min, g.psy_cull, g.ny, g.cs, c0, c1);
        b.y0 = max(b.y0, c0 * g.cs);
        b.y1 = min(b.y1, min((c1 + 1) * g.cs, g.ny) - 1);
        if (b.y0 > b.y1) return false;
    }
    return true;
}

// Kernel normalisation K / h^3 (fp64 for exponent range).
template <int KID>
__device__ __forceinline__ double kernel_norm64(float h) {
    double hd = (double)h;
    double h3 = hd * hd * hd;
    // 1/h^3: hardware reciprocal + one Newton step (a few ulp; the value path is held to
    // the fp32 tolerance).  Deterministic, so the fixed-point bound of K3 stays exact.
    double r = __builtin_amdgcn_rcp(h3);
    r = r * (2.0 - h3 * r);
    if constexpr (KID == 0) return (1.0 / M_PI) * r;                     // _kernels.pyx:16,18
    else if constexpr (KID == 1) return (21.0 / (16.0 * M_PI)) * r;
    else return 1.0;
}

// Per-record term coefficient c = a * norm(h).  The SAME function feeds the per-tile
// bound (scatter) and the terms (deposit), so |c| <= max|c| holds bit-for-bit.
template <int KID>
__device__ __forceinline__ double term_coef(float a, float h) {
    return (double)a * kernel_norm64<KID>(h);
}

// Kernel shape f(q), W = norm(h) * f(q); max f = f(0) = 1 for all three kernels.
// Explicit FMAs: the value path is held to the fp32 tolerance, not to bit-exactness
// (only the neighbour decision is, and it never reaches here).
template <int KID>
__device__ __forceinline__ float kernel_shape(float q) {
    if constexpr (KID == 0) {  // M4 cubic spline (_kernels.pyx:14-19)
        float q2 = q * q;
        float a = fmaf(q2, fmaf(0.75f, q, -1.5f), 1.0f);  // 1 - 1.5 q^2 + 0.75 q^3
        float t = 2.0f - q;
        float b = 0.25f * (t * t * t);
        return q < 1.0f ? a : (q < 2.0f ? b : 0.0f);
    } else if constexpr (KID == 1) {  // Wendland C2, support 2h
        float t = fmaxf(fmaf(-0.5f, q, 1.0f), 0.0f);
        float t2 = t * t;
        return (t2 * t2) * fmaf(2.0f, q, 1.0f);
    } else {
        return 1.0f;
    }
}

// Error band of a record: thr = (2h)^2 in fp32 and the band around it
// inside which the fp32 decision is not trusted (+inf: every pair goes to fp64).
__device__ __forceinline__ void rec_band(const Grid& g, float h, float& thr, float& band) {
    float D = 2.0f * h;
    float Da = fabsf(D);
    thr = D * D;
    float eps = 0x1p-22f * (g.mg + Da);
    band = 4.0f * Da * eps + 2.0f * eps * eps + 0x1p-20f * Da * Da;
    // Negative h narrows the chunk cull below the disc: decide every pair in fp64.
    if (h < 0.0f || !__builtin_isfinite(band)) band = __builtin_inff();
}

// thr -/+ band rounded: the band bounds the decision error with a >= 2x margin and its
// 2^-20 D^2 term alone exceeds these two roundings (2^-24 thr each).
__device__ __forceinline__ void set_band(Prep& P, float thr, float band) {
    P.lo = thr - band;
    P.hi = thr + band;
    P.thr = thr;
    P.band = band;
}

template <int KID, int ACC = kAccF64>
__device__ __forceinline__ bool prep_record(const Grid& g, float u, float v, float h, float a0,
                                            float a1, int k0, int k1, Prep& P) {
    if (!footprint(g, u, v, h, P.b)) return false;
    P.u = u;
    P.v = v;
    P.h = h;
    float thr, band;
    rec_band(g, h, thr, band);
    set_band(P, thr, band);
    P.hinv = __builtin_amdgcn_rcpf(h);  // value path only (fp32 tolerance)
    if constexpr (ACC == kAccFix) {
        P.s0 = (float)ldexp(term_coef<KID>(a0, h), k0);
        P.s1 = (float)ldexp(term_coef<KID>(a1, h), k1);
    } else {
        P.s0 = (float)term_coef<KID>(a0, h);
        P.s1 = (float)term_coef<KID>(a1, h);
    }
    return true;
}

// Reference decision in fp64 (.pyx:13-14, :20-31 and the chunk cull): the slow path.
__device__ __forceinline__ bool exact_pair(const Grid& g, float u, float v, float h,
                                                      int xi, int yi) {
    double ud = u, vd = v, hd = h;
    double dx = ud - corner_x(g, xi);
    double dy = vd - corner_y(g, yi);
    double r2 = dx * dx + dy * dy;
    double t = 2.0 * hd;
    return (r2 < t * t) && cull_pass(g, ud, vd, hd, xi, yi);
}

// The full decision for one (record, pixel) pair given the fp32 corner coordinates.
// Returns inclusion and the fp32 r2 used for the kernel value.
__device__ __forceinline__ bool decide(const Grid& g, const Prep& P, int xi, int yi, float X,
                                       float Y, float& r2) {
    float dx = P.u - X;
    float dy = P.v - Y;
    r2 = dx * dx + dy * dy;
    bool in = r2 < P.lo;
    if (r2 >= P.lo && r2 <= P.hi) in = exact_pair(g, P.u, P.v, P.h, xi, yi);
    return in;
}

// Round a scaled term (|f| < 2^62) to int64, toward zero: for a = |f|, hi = floor(a/2^32)
// and lo = a - hi*2^32 in [0, 2^32) are both exact in fp32 (lo is a multiple of ulp(a)
// below 2^32, so it needs <= 23 significant bits); the sign is applied in two's
// complement.  A pure function of f, so the fixed-point sums are reproducible.
__device__ __forceinline__ unsigned long long f2fix(float f) {
    float a = fabsf(f);
    float hi = floorf(a * 0x1p-32f);
    float lo = fmaf(-hi, 0x1p32f, a);
    unsigned long long m =
        ((unsigned long long)(unsigned int)hi << 32) | (unsigned long long)(unsigned int)lo;
    return f < 0.0f ? 0ull - m : m;
}

// Add one term to an LDS tile accumulator word.
#ifndef ASP_ABLATE_ACC
#define ASP_ABLATE_ACC 0  // diagnostic builds only (wrong maps): 1 = no LDS add, 2 = the fp64
                          // term's bits added with ds_add_u64, 3 = fp32 term, ds_add_u32
#endif
template <int ACC>
__device__ __forceinline__ void acc_add(unsigned long long* a, float t) {
#if ASP_ABLATE_ACC == 1
    asm volatile("" ::"v"(t), "v"(a));
#elif ASP_ABLATE_ACC == 2
    atomicAdd(a, (unsigned long long)__double_as_longlong((double)t));
#elif ASP_ABLATE_ACC == 3
    atomicAdd((unsigned*)a, __float_as_uint(t));
#else
    if constexpr (ACC == kAccFix)
        atomicAdd(a, f2fix(t));
    else
        atomicAdd((double*)a, (double)t);
#endif
}

// Accumulator word -> map value.
template <int ACC>
__device__ __forceinline__ float acc_value(unsigned long long s, int k) {
    if constexpr (ACC == kAccFix)
        return (float)ldexp((double)(long long)s, -k);
    else
        return (float)__longlong_as_double((long long)s);
}

template <int ACC>
__device__ __forceinline__ unsigned long long acc_sum(unsigned long long a, unsigned long long b) {
    if constexpr (ACC == kAccFix)
        return a + b;
    else
        return (unsigned long long)__double_as_longlong(__longlong_as_double((long long)a) +
                                                        __longlong_as_double((long long)b));
}

__device__ __forceinline__ float bcast(float x, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}
__device__ __forceinline__ int bcast(int x, int lane) {
    return __builtin_amdgcn_readlane(x, lane);
}

}  // namespace asp
