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
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace asp {

constexpr int kBlock = 256;     // threads per workgroup (4 waves)
constexpr int kTile = 64;       // GPU tile edge in pixels (LDS accumulator 64x64 per map)
constexpr int kTileShift = 6;
constexpr int kWideTiles = 64;  // particles overlapping more GPU tiles take the wide path

struct Grid {
    double x_min, y_min;
    double psx;       // (x_max - x_min) / nx                        _projector.py:34
    double psy_pix;   // (y_max - y_min) / nx  (S2 quirk)            .pyx:12
    double psy_cull;  // (y_max - y_min) / ny                        _projector.py:35
    float mg;         // bound on |corner coordinate| over the grid (error band)
    int nx, ny, cs;
    int ncx, ncy;     // reference chunks per axis
    int ntx, nty, ntiles;  // GPU tiles
    int nonsquare;    // nx != ny: the y chunk cull is not implied by the r2 test
};

struct Box {
    int x0, x1, y0, y1;  // inclusive pixel ranges
};

// Per-record state for the pair loop.
struct Prep {
    float u, v, h;
    float thr;   // (2h)^2 in fp32
    float band;  // |r2_32 - thr_32| <= band  ->  decide in fp64
    float hinv;  // 1/h
    float c0, c1;  // a0 * norm(h), a1 * norm(h)
    Box b;
};

struct Item {       // one deposit work item: a run of records of one GPU tile
    long long start;
    int tile;
    int count;
    int multi;      // tile split over several items -> accumulate with atomics
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

// Candidate pixel box of a particle: every pixel that can pass the exact test lies in
// it (margin 1e-6 px >> fp64 rounding of the estimate).  False when nothing can pass.
__device__ __forceinline__ bool footprint(const Grid& g, float u, float v, float h, Box& b) {
    if (!__builtin_isfinite(u) || !__builtin_isfinite(v) || !__builtin_isfinite(h)) return false;
    double hd = fabs(2.0 * (double)h);
    if (!(hd > 0.0)) return false;  // h == 0: r2 < 0 never holds (S12)
    double ud = u, vd = v;
    double fx0 = ceil((ud - hd - g.x_min) / g.psx - 1e-6);
    double fx1 = floor((ud + hd - g.x_min) / g.psx + 1e-6);
    double fy0 = ceil((vd - hd - g.y_min) / g.psy_pix - 1e-6);
    double fy1 = floor((vd + hd - g.y_min) / g.psy_pix + 1e-6);
    fx0 = fmax(fx0, 0.0);
    fy0 = fmax(fy0, 0.0);
    fx1 = fmin(fx1, (double)(g.nx - 1));
    fy1 = fmin(fy1, (double)(g.ny - 1));
    if (!(fx0 <= fx1) || !(fy0 <= fy1)) return false;
    b.x0 = (int)fx0;
    b.x1 = (int)fx1;
    b.y0 = (int)fy0;
    b.y1 = (int)fy1;
    if (g.nonsquare) {  // S2: the y cull pitch differs from the pixel pitch
        int c0, c1;
        chunk_range(vd, (double)h, g.y_min, g.psy_cull, g.ny, g.cs, c0, c1);
        b.y0 = max(b.y0, c0 * g.cs);
        b.y1 = min(b.y1, min((c1 + 1) * g.cs, g.ny) - 1);
        if (b.y0 > b.y1) return false;
    }
    return true;
}

template <int KID>
__device__ __forceinline__ double kernel_norm64(double h) {
    if constexpr (KID == 0) return 1.0 / (M_PI * (h * h * h));          // _kernels.pyx:16,18
    else if constexpr (KID == 1) return 21.0 / (16.0 * M_PI * (h * h * h));
    else return 1.0;
}

// Kernel shape f(q), W = norm(h) * f(q).
template <int KID>
__device__ __forceinline__ float kernel_shape(float q) {
    if constexpr (KID == 0) {  // M4 cubic spline (_kernels.pyx:14-19)
        float q2 = q * q;
        float a = 1.0f - 1.5f * q2 + 0.75f * (q2 * q);
        float t = 2.0f - q;
        float b = 0.25f * (t * t * t);
        return q < 1.0f ? a : (q < 2.0f ? b : 0.0f);
    } else if constexpr (KID == 1) {  // Wendland C2, support 2h
        float t = fmaxf(1.0f - 0.5f * q, 0.0f);
        float t2 = t * t;
        return (t2 * t2) * (1.0f + 2.0f * q);
    } else {
        return 1.0f;
    }
}

template <int KID>
__device__ __forceinline__ bool prep_record(const Grid& g, float u, float v, float h, float a0,
                                            float a1, Prep& P) {
    if (!footprint(g, u, v, h, P.b)) return false;
    P.u = u;
    P.v = v;
    P.h = h;
    float D = 2.0f * h;
    float Da = fabsf(D);
    P.thr = D * D;
    float eps = 0x1p-22f * (g.mg + Da);
    float band = 4.0f * Da * eps + 2.0f * eps * eps + 0x1p-20f * Da * Da;
    // Negative h narrows the chunk cull below the disc: decide every pair in fp64.
    P.band = (h < 0.0f || !__builtin_isfinite(band)) ? __builtin_inff() : band;
    P.hinv = 1.0f / h;
    double nrm = kernel_norm64<KID>((double)h);
    P.c0 = (float)((double)a0 * nrm);
    P.c1 = (float)((double)a1 * nrm);
    return true;
}

// Reference decision in fp64 (.pyx:13-14, :20-31 and the chunk cull): the slow path.
__device__ __attribute__((noinline)) bool exact_pair(const Grid& g, float u, float v, float h,
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
    bool in = r2 < P.thr;
    if (fabsf(r2 - P.thr) <= P.band) in = exact_pair(g, P.u, P.v, P.h, xi, yi);
    return in;
}

__device__ __forceinline__ float bcast(float x, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}
__device__ __forceinline__ int bcast(int x, int lane) {
    return __builtin_amdgcn_readlane(x, lane);
}

}  // namespace asp
