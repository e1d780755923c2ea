/*
 * oracle/asp_oracle.c -- CPU restatement of the reference's projection path.
 *
 * TEST INFRASTRUCTURE ONLY.  Linked by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the *checker* / CPU baseline.  The product path
 * (astro-sph-tools_amd/) never loads this library.
 *
 * Parity pin: tests/test_oracle_golden.py checks this file against the golden vectors
 * G1-G7 produced by running the reference itself (tests/golden/make_golden.py).  The
 * gather path below is BIT-EXACT to the reference on every fixture (same fp64
 * operation order, libm pow, NumPy's blocked pairwise summation).
 *
 * Reference being restated (paths under /root/reference/src/astro_sph_tools/):
 *   tools/projections/_projector.py:75-120   create_image  (tile loop, stitch)
 *   tools/projections/_projector.py:13-73    process_chunk (bounding-box cull, pixel loop)
 *   tools/projections/_pixel_calculations.pyx:9-36  calculate_pixel_value
 *   tools/projections/_kernels.pyx:9-20      quartic_spline_kernel (M4 cubic spline)
 * plus the build-defined Wendland-C2 kernel and an indicator kernel
 * (W = 1 inside 2h) used for neighbour counting.
 *
 * Axis selection is done by the caller: (u, v) are the two projected coordinates
 * (X -> (y, z), Y -> (x, z), Z -> (x, y); _projector.py:38-46, .pyx:20-28).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_CUBIC 0
#define ORC_WENDLAND_C2 1
#define ORC_INDICATOR 2

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

int oracle_version(void) { return 1; }

/* _kernels.pyx:9-20 (verbatim arithmetic: q = r/h, libm pow, pi from libc.math). */
static double kernel_w(int kid, double r, double h)
{
    double q = r / h;
    if (kid == ORC_CUBIC) {
        if (q < 1.0)
            return (1 - 1.5 * pow(q, 2) + 0.75 * pow(q, 3)) / (M_PI * pow(h, 3));
        else if (q < 2.0)
            return (0.25 * pow((2 - q), 3)) / (M_PI * pow(h, 3));
        return 0.0;
    }
    if (kid == ORC_WENDLAND_C2) {
        /* W = 21/(16 pi h^3) (1 - q/2)^4 (1 + 2q), q < 2  (tests/golden/make_golden.py:
         * wendland_c2_numpy evaluates the same expression with NumPy). */
        if (q < 2.0) {
            double t = 1.0 - 0.5 * q;
            return 21.0 / (16.0 * M_PI * pow(h, 3)) * pow(t, 4) * (1.0 + 2.0 * q);
        }
        return 0.0;
    }
    return 1.0; /* indicator: every included pair counts 1 */
}

/* The same kernels for the O(pairs) restatement below, with powers as products and the
 * normalisation per particle (nrm = 1/(pi h^3), or 21/(16 pi h^3)): within an ulp or two
 * of kernel_w, which the scatter restatement's own (sequential) summation order already
 * exceeds; the bit-exact gather path keeps kernel_w. */
static double kernel_w_fast(int kid, double q, double nrm)
{
    if (kid == ORC_CUBIC) {
        if (q < 1.0)
            return (1 - 1.5 * (q * q) + 0.75 * (q * q * q)) * nrm;
        else if (q < 2.0) {
            double t = 2 - q;
            return (0.25 * (t * t * t)) * nrm;
        }
        return 0.0;
    }
    if (kid == ORC_WENDLAND_C2) {
        if (q < 2.0) {
            double t = 1.0 - 0.5 * q;
            double t2 = t * t;
            return nrm * (t2 * t2) * (1.0 + 2.0 * q);
        }
        return 0.0;
    }
    return 1.0;
}

void oracle_kernel_eval(int kid, const double *r, const double *h, double *w, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        w[i] = kernel_w(kid, r[i], h[i]);
}

/* NumPy's float64 add.reduce: 0.0-seeded accumulation of pairwise sums over blocks of
 * 8192 (ufunc buffer size); each block summed by pairwise_sum (8-way unrolled leaves of
 * <= 128 elements, split at n/2 rounded down to a multiple of 8). */
static double np_pairwise(const double *a, int64_t n)
{
    if (n < 8) {
        double res = -0.0;
        for (int64_t i = 0; i < n; ++i)
            res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; ++j)
            r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j)
                r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i)
            res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

static double np_sum(const double *a, int64_t n)
{
    double res = 0.0;
    for (int64_t s = 0; s < n; s += 8192)
        res += np_pairwise(a + s, (n - s) < 8192 ? (n - s) : 8192);
    return res;
}

typedef struct {
    double x_min, x_max, y_min, y_max;
    int nx, ny, cs;
    double psx;      /* (x_max - x_min) / nx                         _projector.py:34 */
    double psy_cull; /* (y_max - y_min) / ny                         _projector.py:35 */
    double psy_pix;  /* (y_max - y_min) / nx   (S2: image_size[0])   .pyx:12, _projector.py:68 */
} grid_t;

static grid_t make_grid(int nx, int ny, int cs, double x_min, double x_max, double y_min,
                        double y_max)
{
    grid_t g;
    g.x_min = x_min; g.x_max = x_max; g.y_min = y_min; g.y_max = y_max;
    g.nx = nx; g.ny = ny; g.cs = cs;
    g.psx = (x_max - x_min) / nx;
    g.psy_cull = (y_max - y_min) / ny;
    g.psy_pix = (y_max - y_min) / nx;
    return g;
}

/* _projector.py:38-48: mask of particle p for the chunk starting at (xi0, yi0). */
static int cull_pass(const grid_t *g, double u, double v, double h, int xi0, int yi0)
{
    int xi_end = xi0 + g->cs < g->nx ? xi0 + g->cs : g->nx;
    int yi_end = yi0 + g->cs < g->ny ? yi0 + g->cs : g->ny;
    double h2 = 2 * h;
    double xlo = g->x_min + xi0 * g->psx, xhi = g->x_min + xi_end * g->psx;
    double ylo = g->y_min + yi0 * g->psy_cull, yhi = g->y_min + yi_end * g->psy_cull;
    return (u >= xlo - h2) & (u < xhi + h2) & (v >= ylo - h2) & (v < yhi + h2);
}

/* .pyx:11-14 pixel corner, .pyx:20-31 distance and neighbour mask.  Returns 1 and r2
 * when (xi, yi) sees the particle (the chunk cull is the caller's business). */
static int pixel_pass(const grid_t *g, double u, double v, double h, int xi, int yi,
                      double *r2_out)
{
    double x = g->x_min + (double)xi * g->psx;
    double y = g->y_min + (double)yi * g->psy_pix;
    double dx = u - x, dy = v - y;
    double r2 = dx * dx + dy * dy;
    double t = 2.0 * h;
    *r2_out = r2;
    return r2 < t * t;
}

/*
 * create_image restatement (gather; _projector.py:75-120).  Chunks are visited in the
 * reference's order; chunk_ids (optional, n_chunk_ids entries of cx * n_cy + cy)
 * restricts the work to a subset -- used for the bounded CPU-baseline sample, where
 * the other pixels are left untouched.  img is (nx, ny) C-order, img[xi * ny + yi].
 */
int oracle_create_image(const double *u, const double *v, const double *cu, const double *cv,
                        const double *h, const double *A,
                        int64_t n, int nx, int ny, int cs, double x_min, double x_max,
                        double y_min, double y_max, int kid, const int64_t *chunk_ids,
                        int64_t n_chunk_ids, int nthreads, double *img)
{
    /* cu, cv: the columns the cull reads (NULL: u, v).  The reference picks them with an
     * enum comparison (_projector.py:38-46) and the pixel columns with str().encode()
     * (.pyx:20-28), so some axis spellings cull on other columns than they test. */
    if (!cu) cu = u;
    if (!cv) cv = v;
    if (nx <= 0 || ny <= 0 || cs <= 0)
        return -1;
    grid_t g = make_grid(nx, ny, cs, x_min, x_max, y_min, y_max);
    int ncx = (nx + cs - 1) / cs, ncy = (ny + cs - 1) / cs;
    int64_t nchunks = chunk_ids ? n_chunk_ids : (int64_t)ncx * ncy;
    if (!chunk_ids)
        memset(img, 0, sizeof(double) * (size_t)nx * ny);
#ifdef _OPENMP
    if (nthreads > 0)
        omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int err = 0;
#pragma omp parallel
    {
        int64_t cap = 1024;
        int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * cap);
        double *prod = (double *)malloc(sizeof(double) * cap);
        double *rr = (double *)malloc(sizeof(double) * cap);
        double *hh = (double *)malloc(sizeof(double) * cap);
#pragma omp for schedule(dynamic, 1)
        for (int64_t c = 0; c < nchunks; ++c) {
            int64_t cid = chunk_ids ? chunk_ids[c] : c;
            int cx = (int)(cid / ncy), cy = (int)(cid % ncy);
            int xi0 = cx * cs, yi0 = cy * cs;
            int xi_end = xi0 + cs < nx ? xi0 + cs : nx;
            int yi_end = yi0 + cs < ny ? yi0 + cs : ny;
            /* cull (_projector.py:38-51): members in ascending particle order */
            int64_t m = 0;
            for (int64_t p = 0; p < n; ++p) {
                if (cull_pass(&g, cu[p], cv[p], h[p], xi0, yi0)) {
                    if (m == cap) {
                        cap *= 2;
                        idx = (int64_t *)realloc(idx, sizeof(int64_t) * cap);
                        prod = (double *)realloc(prod, sizeof(double) * cap);
                        rr = (double *)realloc(rr, sizeof(double) * cap);
                        hh = (double *)realloc(hh, sizeof(double) * cap);
                    }
                    idx[m++] = p;
                }
            }
            if (!idx || !prod || !rr || !hh) {
                err = -2;
                continue;
            }
            for (int xi = xi0; xi < xi_end; ++xi)
                for (int yi = yi0; yi < yi_end; ++yi) {
                    /* .pyx:30-34: r = sqrt(r2[mask]); W = k(r, h[mask]); sum(A[mask]*W) */
                    int64_t k = 0;
                    for (int64_t j = 0; j < m; ++j) {
                        int64_t p = idx[j];
                        double r2;
                        if (pixel_pass(&g, u[p], v[p], h[p], xi, yi, &r2)) {
                            rr[k] = sqrt(r2);
                            hh[k] = h[p];
                            prod[k] = (double)p; /* stash particle id */
                            ++k;
                        }
                    }
                    for (int64_t j = 0; j < k; ++j) {
                        int64_t p = (int64_t)prod[j];
                        prod[j] = A[p] * kernel_w(kid, rr[j], hh[j]);
                    }
                    img[(int64_t)xi * ny + yi] = np_sum(prod, k);
                }
        }
        free(idx); free(prod); free(rr); free(hh);
    }
    return err;
}

/* Chunk membership CSR (the set process_chunk culls to; _projector.py:38-51), chunks in
 * (cx, cy) row-major order.  offsets has ncx*ncy+1 entries; returns total or -needed. */
int64_t oracle_chunk_members(const double *u, const double *v, const double *h, int64_t n,
                             int nx, int ny, int cs, double x_min, double x_max, double y_min,
                             double y_max, int64_t *offsets, int32_t *index, int64_t cap)
{
    grid_t g = make_grid(nx, ny, cs, x_min, x_max, y_min, y_max);
    int ncx = (nx + cs - 1) / cs, ncy = (ny + cs - 1) / cs;
    int64_t t = 0;
    offsets[0] = 0;
    for (int cx = 0; cx < ncx; ++cx)
        for (int cy = 0; cy < ncy; ++cy) {
            for (int64_t p = 0; p < n; ++p)
                if (cull_pass(&g, u[p], v[p], h[p], cx * cs, cy * cs)) {
                    if (t < cap)
                        index[t] = (int32_t)p;
                    ++t;
                }
            offsets[cx * ncy + cy + 1] = t;
        }
    return t <= cap ? t : -t;
}

/* Neighbour CSR for a list of pixels (pixel id = xi * ny + yi): particles that pass the
 * pixel's chunk cull AND r2 < (2h)^2, ascending.  Returns total or -needed. */
int64_t oracle_pixel_neighbours(const double *u, const double *v, const double *h, int64_t n,
                                int nx, int ny, int cs, double x_min, double x_max,
                                double y_min, double y_max, const int64_t *pix, int64_t npix,
                                int64_t *offsets, int32_t *index, int64_t cap)
{
    grid_t g = make_grid(nx, ny, cs, x_min, x_max, y_min, y_max);
    int64_t t = 0;
    offsets[0] = 0;
    for (int64_t q = 0; q < npix; ++q) {
        int xi = (int)(pix[q] / ny), yi = (int)(pix[q] % ny);
        int xi0 = (xi / cs) * cs, yi0 = (yi / cs) * cs;
        for (int64_t p = 0; p < n; ++p) {
            double r2;
            if (cull_pass(&g, u[p], v[p], h[p], xi0, yi0) &&
                pixel_pass(&g, u[p], v[p], h[p], xi, yi, &r2)) {
                if (t < cap)
                    index[t] = (int32_t)p;
                ++t;
            }
        }
        offsets[q + 1] = t;
    }
    return t <= cap ? t : -t;
}

/* Chunk range of one particle along one axis: every chunk c with lo(c) <= w < hi(c).
 * Both cull bounds are monotone in c (fl(+), fl(*) monotone), so the set is an interval;
 * found from an estimate, then walked to the exact edges with the reference formula. */
static void chunk_range(double w, double h, double w_min, double ps, int npx, int cs,
                        int *c_lo, int *c_hi)
{
    int nc = (npx + cs - 1) / cs;
    double h2 = 2 * h;
    if (!isfinite(w) || !isfinite(h)) { /* non-finite inputs: excluded */
        *c_lo = 0;
        *c_hi = -1;
        return;
    }
    /* lower condition w >= (w_min + c*cs*ps) - 2h holds for c <= c_max */
#define LO_OK(c) (w >= (w_min + (double)((c) * cs) * ps) - h2)
#define HI_OK(c) (w < (w_min + (double)(((c) + 1) * cs < npx ? ((c) + 1) * cs : npx) * ps) + h2)
    double est = floor((w + h2 - w_min) / (cs * ps));
    int cmax = est < -1 ? -1 : (est > nc - 1 ? nc - 1 : (int)est);
    while (cmax >= 0 && !LO_OK(cmax))
        --cmax;
    while (cmax + 1 <= nc - 1 && LO_OK(cmax + 1))
        ++cmax;
    double est2 = ceil((w - h2 - w_min) / (cs * ps)) - 1;
    int cmin = est2 < 0 ? 0 : (est2 > nc ? nc : (int)est2);
    while (cmin <= nc - 1 && !HI_OK(cmin))
        ++cmin;
    while (cmin - 1 >= 0 && HI_OK(cmin - 1))
        --cmin;
#undef LO_OK
#undef HI_OK
    *c_lo = cmin;
    *c_hi = cmax;
}

/*
 * Particle-centric restatement, O(pairs): same inclusion semantics as the gather path
 * (chunk cull of the pixel's chunk AND r2 < (2h)^2, all fp64 in the reference's
 * operation order), contributions summed in particle order per pixel (sequential, not
 * pairwise: differs from the reference by summation rounding only, ~1e-16 relative).
 * Threads own disjoint bands of x rows, so the result is deterministic.
 * out0 gets sum(A0 W); out1 (nullable) gets sum(A1 W).
 */
int oracle_project_scatter(const double *u, const double *v, const double *cu, const double *cv,
                           const double *h, const double *A0,
                           const double *A1, int64_t n, int nx, int ny, int cs, double x_min,
                           double x_max, double y_min, double y_max, int kid, int nthreads,
                           double *out0, double *out1)
{
    if (!cu) cu = u; /* cull columns, as oracle_create_image */
    if (!cv) cv = v;
    if (nx <= 0 || ny <= 0 || cs <= 0)
        return -1;
    grid_t g = make_grid(nx, ny, cs, x_min, x_max, y_min, y_max);
    memset(out0, 0, sizeof(double) * (size_t)nx * ny);
    if (out1)
        memset(out1, 0, sizeof(double) * (size_t)nx * ny);
    int nt = 1;
#ifdef _OPENMP
    nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    (void)nthreads;
#endif
    int nband = nt * 4 < nx ? nt * 4 : nx;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int b = 0; b < nband; ++b) {
        int bx0 = (int)((int64_t)nx * b / nband), bx1 = (int)((int64_t)nx * (b + 1) / nband);
        for (int64_t p = 0; p < n; ++p) {
            double up = u[p], vp = v[p], hp = h[p];
            double h2 = 2.0 * hp;
            if (!(h2 * h2 > 0.0))
                continue; /* r2 < 0 never holds (S12) */
            double rad = fabs(h2);
            double fx0 = floor((up - rad - x_min) / g.psx) - 2, fx1 = ceil((up + rad - x_min) / g.psx) + 2;
            double fy0 = floor((vp - rad - y_min) / g.psy_pix) - 2, fy1 = ceil((vp + rad - y_min) / g.psy_pix) + 2;
            if (!(fx1 >= bx0 && fx0 < bx1 && fy1 >= 0 && fy0 < ny))
                continue;
            int x0 = fx0 < bx0 ? bx0 : (int)fx0, x1 = fx1 > bx1 - 1 ? bx1 - 1 : (int)fx1;
            int y0 = fy0 < 0 ? 0 : (int)fy0, y1 = fy1 > ny - 1 ? ny - 1 : (int)fy1;
            int cx0, cx1, cy0, cy1;
            chunk_range(cu[p], hp, x_min, g.psx, nx, cs, &cx0, &cx1);
            chunk_range(cv[p], hp, y_min, g.psy_cull, ny, cs, &cy0, &cy1);
            if (cx0 > cx1 || cy0 > cy1)
                continue;
            if (x0 < cx0 * cs) x0 = cx0 * cs;
            if (x1 > (cx1 + 1) * cs - 1) x1 = (cx1 + 1) * cs - 1;
            if (y0 < cy0 * cs) y0 = cy0 * cs;
            if (y1 > (cy1 + 1) * cs - 1) y1 = (cy1 + 1) * cs - 1;
            const double nrm = kid == ORC_CUBIC ? 1.0 / (M_PI * (hp * hp * hp))
                               : 21.0 / (16.0 * M_PI * (hp * hp * hp));
            const double hinv = 1.0 / hp;
            for (int xi = x0; xi <= x1; ++xi)
                for (int yi = y0; yi <= y1; ++yi) {
                    double r2;
                    if (pixel_pass(&g, up, vp, hp, xi, yi, &r2)) {
                        double w = kernel_w_fast(kid, sqrt(r2) * hinv, nrm);
                        int64_t o = (int64_t)xi * ny + yi;
                        out0[o] += A0[p] * w;
                        if (out1)
                            out1[o] += A1[p] * w;
                    }
                }
        }
    }
    return 0;
}

/* Per-particle chunk ranges [cx0, cx1] x [cy0, cy1] (empty when lo > hi): the bin
 * assignment the reference's cull implies, for bit-exact comparison with the GPU. */
void oracle_chunk_ranges(const double *u, const double *v, const double *h, int64_t n, int nx,
                         int ny, int cs, double x_min, double x_max, double y_min, double y_max,
                         int32_t *cx0, int32_t *cx1, int32_t *cy0, int32_t *cy1)
{
    grid_t g = make_grid(nx, ny, cs, x_min, x_max, y_min, y_max);
    for (int64_t p = 0; p < n; ++p) {
        int a, b, c, d;
        chunk_range(u[p], h[p], x_min, g.psx, nx, cs, &a, &b);
        chunk_range(v[p], h[p], y_min, g.psy_cull, ny, cs, &c, &d);
        cx0[p] = a; cx1[p] = b; cy0[p] = c; cy1[p] = d;
    }
}

/* ==================================================================================
 * 3-D density cube (build-defined; SURVEY.md §8(a) "512^3 cube" -- the reference has no
 * volumetric path, so this restatement IS the definition and parity is pinned by it
 * alone).  It extends the 2-D pixel semantics (.pyx:11-14, :30-34) to voxels:
 *   X_i = x_min + i * ((x_max - x_min) / nx), likewise Y_j (ny) and Z_k (nz) -- each axis
 *         with its own pitch (the 2-D S2 quirk is a reference bug, not carried over);
 *   r2  = ((x - X_i)^2 + (y - Y_j)^2) + (z - Z_k)^2, fp64, left to right;
 *   voxel (i, j, k) sees particle p iff r2 < (2 h)^2 (strict, as .pyx:31);
 *   cube[i, j, k - k_lo] = sum_p a_p W(sqrt(r2), h_p)   for planes k_lo <= k < k_hi,
 * with the same kernels as the map (3-D normalisation, so the cube of A = m is the SPH
 * density field sampled at voxel corners).  Layout (nx, ny, k_hi - k_lo) C-order.
 * ================================================================================== */
typedef struct {
    double x_min, y_min, z_min, px, py, pz;
    int nx, ny, nz;
} grid3_t;

static grid3_t make_grid3(int nx, int ny, int nz, double x_min, double x_max, double y_min,
                          double y_max, double z_min, double z_max)
{
    grid3_t g;
    g.x_min = x_min; g.y_min = y_min; g.z_min = z_min;
    g.px = (x_max - x_min) / nx;
    g.py = (y_max - y_min) / ny;
    g.pz = (z_max - z_min) / nz;
    g.nx = nx; g.ny = ny; g.nz = nz;
    return g;
}

static int voxel_pass(const grid3_t *g, double x, double y, double z, double h, int i, int j,
                      int k, double *r2_out)
{
    double dx = x - (g->x_min + (double)i * g->px);
    double dy = y - (g->y_min + (double)j * g->py);
    double dz = z - (g->z_min + (double)k * g->pz);
    double r2 = dx * dx + dy * dy + dz * dz;
    double t = 2.0 * h;
    *r2_out = r2;
    return r2 < t * t;
}

/* Candidate index range along one axis (a superset: one cell of slack each side). */
static int axis_cells(double w, double rad, double w_min, double pitch, int lo, int hi,
                      int *a, int *b)
{
    double f0 = floor((w - rad - w_min) / pitch) - 1, f1 = ceil((w + rad - w_min) / pitch) + 1;
    if (!(f1 >= lo && f0 <= hi))
        return 0;
    *a = f0 < lo ? lo : (int)f0;
    *b = f1 > hi ? hi : (int)f1;
    return 1;
}

/* O(pairs) scatter; threads own disjoint bands of x planes (deterministic).  Terms are
 * added in particle order per voxel. */
int oracle_project3d(const double *x, const double *y, const double *z, const double *h,
                     const double *A, int64_t n, int nx, int ny, int nz, int k_lo, int k_hi,
                     double x_min, double x_max, double y_min, double y_max, double z_min,
                     double z_max, int kid, int nthreads, double *out)
{
    if (nx <= 0 || ny <= 0 || nz <= 0 || k_lo < 0 || k_hi > nz || k_lo >= k_hi)
        return -1;
    grid3_t g = make_grid3(nx, ny, nz, x_min, x_max, y_min, y_max, z_min, z_max);
    int nzl = k_hi - k_lo;
    memset(out, 0, sizeof(double) * (size_t)nx * ny * nzl);
    int nt = 1;
#ifdef _OPENMP
    nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    (void)nthreads;
#endif
    int nband = nt * 4 < nx ? nt * 4 : nx;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int b = 0; b < nband; ++b) {
        int bx0 = (int)((int64_t)nx * b / nband), bx1 = (int)((int64_t)nx * (b + 1) / nband);
        for (int64_t p = 0; p < n; ++p) {
            double hp = h[p], t = 2.0 * hp;
            if (!(t * t > 0.0))
                continue;
            double rad = fabs(t);
            int i0, i1, j0, j1, k0, k1;
            if (!axis_cells(x[p], rad, x_min, g.px, bx0, bx1 - 1, &i0, &i1) ||
                !axis_cells(y[p], rad, y_min, g.py, 0, ny - 1, &j0, &j1) ||
                !axis_cells(z[p], rad, z_min, g.pz, k_lo, k_hi - 1, &k0, &k1))
                continue;
            for (int i = i0; i <= i1; ++i)
                for (int j = j0; j <= j1; ++j)
                    for (int k = k0; k <= k1; ++k) {
                        double r2;
                        if (voxel_pass(&g, x[p], y[p], z[p], hp, i, j, k, &r2))
                            out[((int64_t)i * ny + j) * nzl + (k - k_lo)] +=
                                A[p] * kernel_w(kid, sqrt(r2), hp);
                    }
        }
    }
    return 0;
}

/* Neighbour CSR for a list of voxels (id = (i * ny + j) * nz + k), ascending particle
 * indices, brute force over all particles.  Returns total or -needed. */
int64_t oracle_voxel_neighbours(const double *x, const double *y, const double *z,
                                const double *h, int64_t n, int nx, int ny, int nz,
                                double x_min, double x_max, double y_min, double y_max,
                                double z_min, double z_max, const int64_t *vox, int64_t nvox,
                                int64_t *offsets, int32_t *index, int64_t cap)
{
    grid3_t g = make_grid3(nx, ny, nz, x_min, x_max, y_min, y_max, z_min, z_max);
    int64_t t = 0;
    offsets[0] = 0;
    for (int64_t q = 0; q < nvox; ++q) {
        int k = (int)(vox[q] % nz), j = (int)((vox[q] / nz) % ny), i = (int)(vox[q] / nz / ny);
        for (int64_t p = 0; p < n; ++p) {
            double r2;
            if (voxel_pass(&g, x[p], y[p], z[p], h[p], i, j, k, &r2)) {
                if (t < cap)
                    index[t] = (int32_t)p;
                ++t;
            }
        }
        offsets[q + 1] = t;
    }
    return t <= cap ? t : -t;
}
