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
// re-decided by the reference's own fp64 arithmetic, including the chunk cull.  The band
// also covers the rounding of fp64 inputs to the fp32 working copies, so when the caller
// hands over its fp64 arrays (Src64, asp_project2d_f64) the re-decision reads them and
// the neighbour sets are the reference's on the fp64 inputs themselves.  DESIGN.md §3.
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
#ifndef ASP_DEP_BLOCK
#define ASP_DEP_BLOCK 512
#endif
constexpr int kDepBlock = ASP_DEP_BLOCK;  // deposit workgroup (8 waves; 2 per CU)
constexpr int kTile = 64;          // GPU tile edge in pixels
constexpr int kTileShift = 6;
constexpr int kRow = kTile + 1;    // LDS tile row stride in words (one pad word per row)
constexpr int kTileWords = kTile * kRow;  // LDS words of one map's tile
constexpr int kWideTilesDefault = 256;  // particles overlapping more tiles take the wide path
constexpr int kScaleBits = 49;     // per-tile bound n_t * max|c| maps to <= 2^49 (f2fix: < 2^51)
constexpr int kAccF64 = 0;         // LDS fp64 accumulation
constexpr int kAccFix = 1;         // LDS int64 fixed point (deterministic)

struct Grid {
    double x_min, y_min;
    double psx;       // (x_max - x_min) / nx                        _projector.py:34
    double psy_pix;   // (y_max - y_min) / nx  (S2 quirk)            .pyx:12
    double psy_cull;  // (y_max - y_min) / ny                        _projector.py:35
    float xminf, yminf;   // fp32 copies for the candidate-box estimate
    float ipsx, ipsy;     // fp32 reciprocal pitches (pixel pitches)
    float mg;         // bound on |corner coordinate|, absolute frame (error band)
    float mgl;        // the same for the records' box-origin / tile frames (128 pitches)
    int nx, ny, cs;   // nx: this call's WINDOW of image rows (== gnx without windows)
    int gnx;          // the image's nx (pitches, S2 quirk, chunk cull)
    int ox;           // first image row of the window (a multiple of kTile): images of
                      // more than kMaxTiles GPU tiles are projected as row windows
    int ncx, ncy;     // reference chunks per axis
    int ntx, nty, ntiles;  // GPU tiles
    int nonsquare;    // nx != ny: the y chunk cull is not implied by the r2 test
    int mixed;        // the cull reads other position columns than the pixel test (Src64)
    int wide_tiles;   // particles over more tiles than this take the wide path (K6)
    int gather_min;   // records with clipped boxes >= this on both axes are gathered (K4g)
    int gather_area;  // ... and so are clipped boxes of at least this many pixels
};

// The caller's particle arrays, resident in HBM, read by particle index where the exact
// values matter (fp64 re-decisions, tile-local coordinates): the fp64 arrays
// (asp_project2d_f64: positions rows of `stride` doubles, u64 / v64 the columns of the
// pixel test, cu64 / cv64 those of the chunk cull -- the same unless the reference's axis
// spelling makes them differ, Grid::mixed; h64 contiguous), or, with u64 == nullptr,
// the fp32 inputs u32 / v32 / h32 themselves (asp_project2d).
struct Src64 {
    const double* u64;
    const double* v64;
    const double* cu64;
    const double* cv64;
    const double* h64;
    long long stride;
    const float* u32;
    const float* v32;
    const float* h32;
};

struct Box {
    int x0, x1, y0, y1;  // inclusive pixel ranges
};

// Per-record state for the pair loop.
struct Prep {
    float u, v, h;  // u, v: tile-local in the deposits (corner tables in the same frame)
    float lo;    // fp32 r2 < lo: inside for sure;  lo <= r2 <= hi: decide in fp64;
    float hi;    // r2 > hi: outside  (lo, hi = (2h)^2 -/+ error band; +-inf: always fp64)
    float hinv;  // 1/h
    float s0, s1;  // a * norm(h) (kAccF64) or a * norm(h) * 2^k_tile (kAccFix)
    float thr;   // (2h)^2 in fp32
    float band;  // |r2 - thr| <= band: the fp32 decision is not trusted (inf: never)
    int p;       // particle index (the fp64 re-decision reads the caller's arrays there)
    Box b;
};

struct Item {       // one deposit work item: a run of records of one GPU tile
    long long start;
    int tile;
    int count;      // 0: empty tile (write zeros)
    int slab;       // -1: the tile's only item (writes the map); >= 0: partial slab
    int mode;       // 0 (kept for the binning scans shared with the cube)
};

struct Merge {      // a tile split over several items: sum their slabs
    int tile;
    int slab0;
    int nslab;
    int pad;
};

__device__ __forceinline__ double corner_x(const Grid& g, int xi) {  // xi: window row
    return g.x_min + (double)(xi + g.ox) * g.psx;   // .pyx:13
}
__device__ __forceinline__ double corner_y(const Grid& g, int yi) {
    return g.y_min + (double)yi * g.psy_pix;        // .pyx:14
}

// _projector.py:38-48 for the chunk holding pixel (xi, yi) (xi a window row).  fp64,
// reference order:
// (w_min + chunk_start * pitch) - 2*h  <=  w  <  (w_min + chunk_end * pitch) + 2*h.
__device__ __forceinline__ bool cull_pass(const Grid& g, double u, double v, double h,
                                          int xi, int yi) {
    xi += g.ox;
    int xi0 = (xi / g.cs) * g.cs, yi0 = (yi / g.cs) * g.cs;
    int xe = min(xi0 + g.cs, g.gnx), ye = min(yi0 + g.cs, g.ny);
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

// The fp64 values the reference sees for particle p: pixel-test coordinates (U, V),
// cull coordinates (CU, CV) and h.
struct Vals {
    double U, V, CU, CV, H;
};
__device__ __forceinline__ Vals src_values(const Grid& g, const Src64& s, int p) {
    Vals r;
    if (s.u64) {
        const long long o = (long long)p * s.stride;
        r.U = s.u64[o];
        r.V = s.v64[o];
        r.H = s.h64[p];
        r.CU = g.mixed ? s.cu64[o] : r.U;
        r.CV = g.mixed ? s.cv64[o] : r.V;
    } else {
        r.U = r.CU = s.u32[p];
        r.V = r.CV = s.v32[p];
        r.H = s.h32[p];
    }
    return r;
}
// The exact fp64 value of particle p's pixel-test coordinate u (fp32 value u when the
// fp32 inputs are the inputs) -- the source of tile-local coordinates.
__device__ __forceinline__ double src_u(const Src64& s, int p, float u) {
    return s.u64 ? s.u64[(long long)p * s.stride] : (double)u;
}
__device__ __forceinline__ double src_v(const Src64& s, int p, float v) {
    return s.v64 ? s.v64[(long long)p * s.stride] : (double)v;
}

// Candidate pixel box of a particle: a superset of the pixels that can pass the exact
// test.  fp32 estimate of (w - 2|h| - w_min) / pitch with a margin delta that bounds its
// rounding error: at most ~6 roundings of 2^-24 relative to (|w| + |w_min| + 2|h|) / pitch
// (w_min and 1/pitch to fp32, the difference, the product, the two offsets) plus the
// rounding of fp64 inputs to fp32 (2^-24 |w|, 2^-23 |h|), so 2^-20 leaves a 2x margin;
// plus 2^-12 px so that a corner at exactly 2h stays a candidate.  Where the cull is not
// implied by the disc -- the y axis of non-square images (S2), both axes when the cull
// reads other columns (Grid::mixed) -- the range is clipped to the chunks whose cull
// accepts the particle, computed exactly from the inputs (fp64 ones when given), so
// every pixel of the box passes the cull.  False when nothing can pass.
// CULL = false: the caller has checked that the grid needs no chunk clipping (square
// image, cull reads the pixel columns), so that code is not compiled in.
template <bool CULL = true>
__device__ __forceinline__ bool footprint(const Grid& g, const Src64& s, int p, float u, float v,
                                          float h, Box& b) {
    float hd = fabsf(2.0f * h);
    if (!(hd > 0.0f) || !__builtin_isfinite(hd)) {
        // h == 0: r2 < 0 never holds (S12).  Non-finite: excluded.
        return false;
    }
    if (!__builtin_isfinite(u) || !__builtin_isfinite(v)) return false;
    float cx = (u - g.xminf) * g.ipsx, rx = hd * g.ipsx;
    float cy = (v - g.yminf) * g.ipsy, ry = hd * g.ipsy;
    float dx = (fabsf(u) + fabsf(g.xminf) + hd) * g.ipsx * 0x1p-20f + 0x1p-12f;
    float dy = (fabsf(v) + fabsf(g.yminf) + hd) * g.ipsy * 0x1p-20f + 0x1p-12f;
    // image rows clipped to the window [ox, ox + nx), then window-relative
    float fx0 = fmaxf(ceilf(cx - rx - dx), (float)g.ox);
    float fx1 = fminf(floorf(cx + rx + dx), (float)(g.ox + g.nx - 1));
    float fy0 = fmaxf(ceilf(cy - ry - dy), 0.0f);
    float fy1 = fminf(floorf(cy + ry + dy), (float)(g.ny - 1));
    if (!(fx0 <= fx1) || !(fy0 <= fy1)) return false;
    b.x0 = (int)fx0 - g.ox;
    b.x1 = (int)fx1 - g.ox;
    b.y0 = (int)fy0;
    b.y1 = (int)fy1;
    if (CULL && (g.nonsquare || g.mixed)) {
        const Vals x = src_values(g, s, p);
        int c0, c1;
        chunk_range(x.CV, x.H, g.y_min, g.psy_cull, g.ny, g.cs, c0, c1);
        b.y0 = max(b.y0, c0 * g.cs);
        b.y1 = min(b.y1, min((c1 + 1) * g.cs, g.ny) - 1);
        if (b.y0 > b.y1) return false;
        if (g.mixed) {
            chunk_range(x.CU, x.H, g.x_min, g.psx, g.gnx, g.cs, c0, c1);
            b.x0 = max(b.x0, c0 * g.cs - g.ox);
            b.x1 = min(b.x1, min((c1 + 1) * g.cs, g.gnx) - 1 - g.ox);
            if (b.x0 > b.x1) return false;
        }
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
// inside which the fp32 decision is not trusted (+inf: every pair goes to fp64).  mg
// bounds the coordinates of the frame the decision is taken in: g.mg for absolute
// corners (|X| <= M), g.mgl for the records' box-origin frame (offsets < 64 pitches).
__device__ __forceinline__ float rec_thr(float h) {
    float D = 2.0f * h;
    return D * D;
}
__device__ __forceinline__ float rec_band(float mg, float h) {
    float Da = fabsf(2.0f * h);
    float eps = 0x1p-21f * (mg + Da);
    float band = 4.0f * Da * eps + 2.0f * eps * eps + 0x1p-20f * Da * Da;
    // Negative h narrows the chunk cull below the disc: decide every pair in fp64.
    if (h < 0.0f || !__builtin_isfinite(band)) band = __builtin_inff();
    return band;
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
__device__ __forceinline__ bool prep_record(const Grid& g, const Src64& s, int p, float u,
                                            float v, float h, float a0, float a1, int k0,
                                            int k1, Prep& P) {
    if (!footprint(g, s, p, u, v, h, P.b)) return false;
    P.u = u;
    P.v = v;
    P.h = h;
    P.p = p;
    set_band(P, rec_thr(h), rec_band(g.mg, h));
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

// Reference decision in fp64 (.pyx:13-14, :20-31 and the chunk cull): the slow path, on
// the caller's values of particle p.
__device__ __forceinline__ bool exact_pair(const Grid& g, const Src64& s, int p, int xi, int yi) {
    const Vals x = src_values(g, s, p);
    double dx = x.U - corner_x(g, xi);
    double dy = x.V - corner_y(g, yi);
    double r2 = dx * dx + dy * dy;
    double t = 2.0 * x.H;
    return (r2 < t * t) && cull_pass(g, x.CU, x.CV, x.H, xi, yi);
}

// The full decision for one (record, pixel) pair given the fp32 corner coordinates in
// the frame of (P.u, P.v) (tile-local in the deposits, absolute in k_neighbours).
// Returns inclusion and the fp32 r2 used for the kernel value.
__device__ __forceinline__ bool decide(const Grid& g, const Src64& s, const Prep& P, int xi,
                                       int yi, float X, float Y, float& r2) {
    float dx = P.u - X;
    float dy = P.v - Y;
    r2 = dx * dx + dy * dy;
    bool in = r2 < P.lo;
    if (r2 >= P.lo && r2 <= P.hi) in = exact_pair(g, s, P.p, xi, yi);
    return in;
}

// Round a scaled term (|f| < 2^62) to int64, toward zero: for a = |f|, hi = floor(a/2^32)
// and lo = a - hi*2^32 in [0, 2^32) are both exact in fp32 (lo is a multiple of ulp(a)
// below 2^32, so it needs <= 23 significant bits); the sign is applied in two's
// complement.  A pure function of f, so the fixed-point sums are reproducible.
__device__ __forceinline__ unsigned long long f2fix(float f) {
    // |f| <= 2^kScaleBits < 2^51: fl64(f) + 1.5 * 2^52 holds round(f) in its low mantissa
    // bits (round to nearest even), so one fp64 add and a 64-bit integer subtract convert
    // (the truncating fp32 split this replaces took ~10 instructions per term)
    const double magic = 6755399441055744.0;  // 1.5 * 2^52
    return (unsigned long long)(__double_as_longlong((double)f + magic) -
                                __double_as_longlong(magic));
}

// Add one term to an LDS tile accumulator word.
template <int ACC>
__device__ __forceinline__ void acc_add(unsigned long long* a, float t) {
    if constexpr (ACC == kAccFix)
        atomicAdd(a, f2fix(t));
    else
        atomicAdd((double*)a, (double)t);
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

typedef float f2 __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_* ops)

// Shape f(q) / kShapeScale for kernels that vanish continuously at q = 2 (cubic,
// Wendland), written so that q >= 2 gives exactly 0 without a comparison, two pixels per
// packed instruction: t = clamp(1 - q/2) (the VOP3P clamp bit; 1 - q/2 <= 1 as q >= 0).
// Cubic: f = (2 - q)^3 / 4 - max(1 - q, 0)^3 = 2 t^3 - s^3 with s = clamp(1 - q) -- one
// expression on [0, 2] (for q < 1 it expands to 1 - 1.5 q^2 + 0.75 q^3), no branch;
// computed as f / 2 = t^3 - s^3 / 2.  Wendland C2: t^4 (1 + 2q).
template <int KID>
constexpr float kShapeScale = KID == 0 ? 2.0f : 1.0f;

// clamp(1 - q/2, 0, 1) and clamp(1 - q, 0, 1) on two lanes of fp32 at once (inline
// constants, both halves).  The leading s_nop covers the transcendental-result hazard
// (q comes straight from v_sqrt_f32).
__device__ __forceinline__ f2 pk_one_minus_half_clamp(f2 q) {
    f2 d;
    asm("s_nop 0\n\tv_pk_fma_f32 %0, %1, -0.5, 1.0 op_sel_hi:[1,0,0] clamp" : "=v"(d) : "v"(q));
    return d;
}
__device__ __forceinline__ f2 pk_one_minus_clamp(f2 q) {
    f2 d;
    asm("s_nop 0\n\tv_pk_fma_f32 %0, %1, -1.0, 1.0 op_sel_hi:[1,0,0] clamp" : "=v"(d) : "v"(q));
    return d;
}

template <int KID>
__device__ __forceinline__ f2 edge_shape2(f2 q) {
    const f2 t = pk_one_minus_half_clamp(q);
    if constexpr (KID == 0) {
        const f2 s = pk_one_minus_clamp(q);
        return __builtin_elementwise_fma((f2){-0.5f, -0.5f}, s * s * s, t * t * t);
    } else {
        const f2 t2 = t * t;
        return (t2 * t2) * __builtin_elementwise_fma((f2){2.0f, 2.0f}, q, (f2){1.0f, 1.0f});
    }
}

}  // namespace asp
