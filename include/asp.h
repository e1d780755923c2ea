/*
 * asp.h -- C-ABI of the MI355X-native SPH particle-to-grid projector (libasp_hip.so).
 *
 * Drop-in boundary for astro_sph_tools' map-rendering path.  Each entry point names
 * the reference interface it replaces (paths under
 * /root/reference/src/astro_sph_tools/).  The Python mirror of the reference API
 * (astro-sph-tools_amd/asp_amd/) binds these with ctypes; INTEGRATION.md shows the
 * binding a maintainer would add to the reference itself.
 *
 * Conventions
 *  - plain pointers and sizes only; no C++ or torch types cross this boundary;
 *  - every function returns ASP_OK (0) or a negative ASP_ERR_* code, and sets a
 *    thread-local message readable with asp_last_error();
 *  - inputs are borrowed and never written; outputs are written in full;
 *  - particle inputs are float32 structure-of-arrays, already axis-selected: (u, v) are
 *    the two projected coordinates (X -> (y, z), Y -> (x, z), Z -> (x, y);
 *    _projector.py:38-46, _pixel_calculations.pyx:20-28);
 *  - images are (nx, ny) C-order float32, element [xi * ny + yi] (_projector.py:88,117);
 *  - by default pointers are HOST pointers (the library stages them through HBM);
 *    with ASP_F_DEVICE_PTRS they are device pointers on `device` and the call is
 *    ordered on `stream` (a hipStream_t, NULL = the legacy default stream);
 *  - thread-safe: a per-device workspace cache guarded by a mutex; one call at a time
 *    per device enqueues work, and each call's stream first waits for the previous
 *    call's work (an event), so calls on different streams never share buffers in flight.
 */
#ifndef ASP_H
#define ASP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ASP_API_VERSION 1

/* kernel_id: the SPH kernel W(r, h), support 2h, 3-D normalisation, evaluated at the
 * projected 2-D distance (reference semantics S6). */
#define ASP_KERNEL_CUBIC_SPLINE 0 /* _kernels.pyx:9-20 quartic_spline_kernel (M4 cubic)  */
#define ASP_KERNEL_WENDLAND_C2 1  /* 21/(16 pi h^3) (1-q/2)^4 (1+2q), build-defined      */
#define ASP_KERNEL_INDICATOR 2    /* W = 1 for every included pair: neighbour counting    */

/* flags */
#define ASP_F_DEVICE_PTRS 0x1 /* inputs/outputs are device pointers on `device`            */
#define ASP_F_RATIO 0x2       /* two outputs: out0 <- out0 / out1 (0 where out1 == 0)      */
#define ASP_F_ACCUMULATE 0x4  /* add into out0/out1 instead of overwriting                 */
#define ASP_F_DETERMINISTIC 0x8 /* int64 fixed-point accumulation: bitwise reproducible and
                                 * input-order independent maps; relative precision degrades
                                 * for pixels below ~2^-37 n_t max|A W| of their 64x64 tile
                                 * (DESIGN.md §4).  Default: fp64 accumulation.  Not with
                                 * ASP_F_RATIO (ASP_ERR_INVALID): a ratio of fixed-point
                                 * components is imprecise in kernel-tail pixels.           */
#define ASP_F_DEVICE_OUTPUTS 0x10 /* host (pageable) inputs, device outputs: the reader's
                                   * arrays in, a device map out for the RCCL sum; the
                                   * inputs go through pinned bounce buffers (two 32 MiB
                                   * pieces, CPU copy overlapping the DMA)                 */

/* asp_project2d_f64 axis: cull on axis c's columns (the reference's mixed spellings) */
#define ASP_AXIS_CULL(c) (((c) + 1) << 4)

/* errors */
#define ASP_OK 0
#define ASP_ERR_INVALID -1     /* bad argument (ValueError on the Python side)             */
#define ASP_ERR_HIP -2         /* HIP runtime error                                         */
#define ASP_ERR_NOMEM -3       /* device allocation failed                                  */
#define ASP_ERR_UNSUPPORTED -4 /* valid request this build does not implement               */

/* Library version (ASP_API_VERSION * 10000 + build number). */
int asp_version(void);

/* Message for the last failing call on this thread ("" if none). */
const char *asp_last_error(void);

/* Number of visible HIP devices (0 on a host without a GPU; never fails). */
int asp_device_count(void);

/*
 * 2-D projection: replaces create_image (_projector.py:75-120) together with
 * process_chunk (:13-73), calculate_pixel_value (_pixel_calculations.pyx:9-36) and the
 * kernel (_kernels.pyx:9-20).
 *
 *   out0[xi, yi] = sum_p a0[p] * W(r_p, h_p)   over p passing the reference's cull of
 *                  the chunk_size tile holding (xi, yi) AND r_p^2 < (2 h_p)^2,
 *   r_p^2 = (u_p - X_xi)^2 + (v_p - Y_yi)^2,  X_xi = u_min + xi * (u_max-u_min)/nx,
 *   Y_yi = v_min + yi * (v_max - v_min)/nx   (sic: nx -- reference quirk S2).
 *
 * Neighbour membership is decided with the reference's fp64 arithmetic on the fp64
 * values of the fp32 inputs (bit-exact neighbour sets for those inputs; for raw fp64
 * reader arrays use asp_project2d_f64); values are accumulated in fp32 terms.  a1/out1 (both non-NULL or both
 * NULL) give a second map over the same neighbour sets (mass-weighted maps:
 * a0 = m*T, a1 = m, with ASP_F_RATIO).  n == 0 is valid (all-zero image).
 * chunk_size >= 1 is the reference's tile size; it only changes results for
 * non-square images (quirk S2), exactly as in the reference.
 */
int asp_project2d(const float *u, const float *v, const float *h, const float *a0,
                  const float *a1, int64_t n, double u_min, double u_max, double v_min,
                  double v_max, int32_t nx, int32_t ny, int32_t chunk_size, int32_t kernel_id,
                  int32_t flags, float *out0, float *out1, int32_t device, void *stream);

/*
 * Image rows [row_lo, row_hi) of asp_project2d's map only -- the row-slab (image-plane)
 * decomposition of SURVEY.md §8(e) / H2, the reference's own image chunks
 * (_projector.py:89-111) distributed: out0 / out1 hold (row_hi - row_lo) x ny pixels,
 * element [(xi - row_lo) * ny + yi], each equal to the pixel asp_project2d writes for the
 * whole image (same corners, pitches, chunk cull and decisions; particles whose footprint
 * misses the rows are skipped).  Any 0 <= row_lo < row_hi <= nx (the GPU tiles of the
 * call start at row_lo).  Other arguments as asp_project2d.
 */
int asp_project2d_rows(const float *u, const float *v, const float *h, const float *a0,
                       const float *a1, int64_t n, double u_min, double u_max, double v_min,
                       double v_max, int32_t nx, int32_t ny, int32_t chunk_size, int32_t row_lo,
                       int32_t row_hi, int32_t kernel_id, int32_t flags, float *out0,
                       float *out1, int32_t device, void *stream);

/*
 * Several property maps from ONE binning (the callers render m, m*T, ion masses ... of
 * the same particles: io/data_structures/_SnapshotBase.py:618-906): out_k = the
 * asp_project2d map of props[k] for k < nprops <= 6, every map over the same neighbour
 * sets.  The particles are counted and scattered once; the records carry the first two
 * properties' coefficients and, beside them, those of properties 2..5, which further
 * deposit passes read.  nprops <= 2 is asp_project2d; more need ASP_F_DEVICE_PTRS (device
 * pointers) and fp64 accumulation (no ASP_F_RATIO / ASP_F_DETERMINISTIC: form ratios
 * with asp_ratio).  props / outs are host arrays of nprops device pointers.
 */
int asp_project2d_props(const float *u, const float *v, const float *h,
                        const float *const *props, int32_t nprops, int64_t n, double u_min,
                        double u_max, double v_min, double v_max, int32_t nx, int32_t ny,
                        int32_t chunk_size, int32_t kernel_id, int32_t flags,
                        float *const *outs, int32_t device, void *stream);

/*
 * The same on the reader's float64 arrays (positions (n, 3), h, props[k] float64, all on
 * the device: ASP_F_DEVICE_PTRS), with the exact fp64 decisions of asp_project2d_f64.
 */
int asp_project2d_props_f64(const double *positions, const double *h,
                            const double *const *props, int32_t nprops, int64_t n,
                            int32_t axis, double u_min, double u_max, double v_min,
                            double v_max, int32_t nx, int32_t ny, int32_t chunk_size,
                            int32_t kernel_id, int32_t flags, float *const *outs,
                            int32_t device, void *stream);

/*
 * SPH-weighted property maps -- north_star's "mass/rho-weighted scatter" over the SoA
 * (x, y, z, h, m, rho, A): out_k = sum_j (m_j / rho_j) props[k]_j W(r_ij, h_j), the SPH
 * estimate of the field props[k] integrated along the line of sight, with rho the
 * reader's densities (io/data_structures/_SnapshotBase.py:833, get_densities) and m its
 * masses (:618-700).  rho NULL: the mass-weighted sums sum_j m_j props[k]_j W.  Each
 * property's fp32 working copy is fl32(props[k] * (m / rho)), evaluated in fp64 and
 * rounded once on the device; binning, neighbour decisions and the deposit are
 * asp_project2d_props'(_f64) -- so with nprops = 2 and ASP_F_RATIO, out0 is the
 * (m/rho)-weighted mean of props[0] over props[1]'s weights.  Host pointers are accepted
 * for nprops <= 2 (as asp_project2d / asp_project2d_f64); mass / rho live where the
 * properties live.
 */
int asp_project2d_sph(const float *u, const float *v, const float *h, const float *mass,
                      const float *rho, const float *const *props, int32_t nprops, int64_t n,
                      double u_min, double u_max, double v_min, double v_max, int32_t nx,
                      int32_t ny, int32_t chunk_size, int32_t kernel_id, int32_t flags,
                      float *const *outs, int32_t device, void *stream);
int asp_project2d_sph_f64(const double *positions, const double *h, const double *mass,
                          const double *rho, const double *const *props, int32_t nprops,
                          int64_t n, int32_t axis, double u_min, double u_max, double v_min,
                          double v_max, int32_t nx, int32_t ny, int32_t chunk_size,
                          int32_t kernel_id, int32_t flags, float *const *outs, int32_t device,
                          void *stream);

/*
 * create_image on the reader's own float64 arrays: the drop-in for create_image
 * (_projector.py:75-120) as it is called, with positions (n, 3) float64 row-major (the
 * reader's get_positions, _SnapshotBase.py:708-722), smoothing lengths and properties
 * float64, and the projection axis (0 = X -> (y, z), 1 = Y -> (x, z), 2 = Z -> (x, y);
 * _projector.py:38-46).  The reference decides the chunk cull (_projector.py:38-46, enum
 * comparison) and the pixel test (_pixel_calculations.pyx:20-28, str().encode()) from
 * the axis separately, so some spellings (a str "x") cull on other columns than they
 * test: axis | ASP_AXIS_CULL(c) reproduces that, culling on axis c's columns.  The library stages float32 working copies in HBM and keeps the
 * float64 arrays resident: every (particle, pixel) decision is the reference's fp64 test
 * on the ORIGINAL fp64 values (bit-exact neighbour sets for any fp64 input, not only
 * fp32-representable ones); values accumulate as in asp_project2d.  Host pointers unless
 * ASP_F_DEVICE_PTRS (then device pointers, ordered on `stream`).  Other arguments and
 * flags as asp_project2d.
 */
int asp_project2d_f64(const double *positions, const double *h, const double *a0,
                      const double *a1, int64_t n, int32_t axis, double u_min, double u_max,
                      double v_min, double v_max, int32_t nx, int32_t ny, int32_t chunk_size,
                      int32_t kernel_id, int32_t flags, float *out0, float *out1, int32_t device,
                      void *stream);

/*
 * The kernel_func plugin point (_projector.py:26, 86; _pixel_calculations.pyx:30-33): for
 * an arbitrary user kernel W(r, h) -- Python code that cannot run on the device -- the
 * device produces the neighbour pairs and the host evaluates W on them, in a SESSION that
 * stages and bins the particles once per map:
 *
 *   asp_pairs_begin: stage positions (n, 3) / h (axis, extent, chunk_size as
 *     asp_project2d_f64), bin them and count every GPU tile's pairs: tile_pairs[t] for the
 *     ceil(nx/64) * ceil(ny/64) tiles t = tx * ceil(ny/64) + ty (host array).  *session
 *     receives the handle (NULL on error).  With ASP_F_DEVICE_PTRS positions / h are device
 *     arrays that must stay alive until asp_pairs_end, and the emit outputs are device
 *     pointers too.
 *   asp_pairs_emit: for the tiles tile_lo <= t < tile_hi, every (pixel, particle) pair
 *     create_image includes (the exact decision of asp_project2d_f64): particle[k] (index
 *     into the inputs) and r2[k] = dx*dx + dy*dy in fp64 as the reference forms it
 *     (.pyx:13-14, :20-30), k in [offsets[q], offsets[q+1]) for the q-th pixel of the
 *     range -- pixels tile by tile, (lx * 64 + ly) inside a tile, pixels outside the image
 *     empty; offsets ((tile_hi - tile_lo) * 4096 + 1 entries) start at 0 and end at the
 *     sum of tile_pairs over the range, the size particle / r2 must have.  Order inside a
 *     pixel unspecified.  The session keeps the binned records resident between emits
 *     (images of more than 4096 tiles: per window of tile rows, re-binned when a range
 *     moves to the next window).
 *   asp_pairs_end: release the session (NULL is a no-op).
 * A session is used by one thread at a time; it owns its buffers, so other calls on the
 * device may run between its emits.
 */
int asp_pairs_begin(const double *positions, const double *h, int64_t n, int32_t axis,
                    double u_min, double u_max, double v_min, double v_max, int32_t nx,
                    int32_t ny, int32_t chunk_size, int32_t flags, int32_t device, void *stream,
                    int64_t *tile_pairs, void **session);
int asp_pairs_emit(void *session, int32_t tile_lo, int32_t tile_hi, int64_t *offsets,
                   int32_t *particle, double *r2);
int asp_pairs_end(void *session);

/*
 * 3-D voxel cube (build-defined; SURVEY.md §8(a) "512^3 cube" -- no reference
 * counterpart, it extends create_image's pixel semantics (_pixel_calculations.pyx:11-14,
 * :30-34) to voxels; CPU restatement: oracle/asp_oracle.c oracle_project3d):
 *
 *   out[i, j, k - k_lo] = sum_p a[p] * W(r_p, h_p)  over p with r_p^2 < (2 h_p)^2,
 *   r_p^2 = ((x_p - X_i)^2 + (y_p - Y_j)^2) + (z_p - Z_k)^2   (fp64, bit-exact sets),
 *   X_i = x_min + i * (x_max - x_min)/nx, Y_j and Z_k likewise with ny and nz.
 *
 * Only planes k_lo <= k < k_hi are produced (Z-slab ownership across GPUs); out is
 * (nx, ny, k_hi - k_lo) C-order float32.  At most 16384 bricks of 16x16x32 voxels per
 * call (a whole 512^3 cube fits).  flags: ASP_F_DEVICE_PTRS, ASP_F_ACCUMULATE.
 */
int asp_project3d(const float *x, const float *y, const float *z, const float *h,
                  const float *a, int64_t n, double x_min, double x_max, double y_min,
                  double y_max, double z_min, double z_max, int32_t nx, int32_t ny, int32_t nz,
                  int32_t k_lo, int32_t k_hi, int32_t kernel_id, int32_t flags, float *out,
                  int32_t device, void *stream);

/*
 * Kernel evaluation on the device: replaces quartic_spline_kernel(r, h)
 * (_kernels.pyx:9-20) for kernel_id 0; fp64 in and out, same formula and branch order.
 * Host pointers unless ASP_F_DEVICE_PTRS.
 */
int asp_kernel_eval(int32_t kernel_id, const double *r, const double *h, double *w, int64_t n,
                    int32_t flags, int32_t device, void *stream);

/*
 * Bin assignment (the reference's process_chunk cull, _projector.py:38-48): for every
 * particle, the inclusive range of chunk indices [cx0, cx1] x [cy0, cy1] whose cull it
 * passes (empty when cx0 > cx1 or cy0 > cy1).  Computed on the device in fp64 with the
 * reference's operation order; bit-exact membership.  Host pointers unless
 * ASP_F_DEVICE_PTRS.
 */
int asp_chunk_ranges(const float *u, const float *v, const float *h, int64_t n, double u_min,
                     double u_max, double v_min, double v_max, int32_t nx, int32_t ny,
                     int32_t chunk_size, int32_t *cx0, int32_t *cx1, int32_t *cy0,
                     int32_t *cy1, int32_t flags, int32_t device, void *stream);

/*
 * Neighbour sets of selected pixels (calculate_pixel_value's mask,
 * _pixel_calculations.pyx:30-31, restricted to the chunk cull): for pixel k
 * (id = xi * ny + yi), the ascending particle indices in
 * index[offsets[k] .. offsets[k+1]).  Uses the same device inclusion test as
 * asp_project2d.  *total receives the number of pairs; when it exceeds cap, nothing
 * beyond cap is written and the call returns ASP_OK with *total > cap.
 * Host pointers only (a test/inspection entry point).
 */
int asp_pixel_neighbours(const float *u, const float *v, const float *h, int64_t n,
                         double u_min, double u_max, double v_min, double v_max, int32_t nx,
                         int32_t ny, int32_t chunk_size, const int64_t *pixels, int64_t npix,
                         int64_t *offsets, int32_t *index, int64_t cap, int64_t *total,
                         int32_t device);

/*
 * Weighted-map finalisation: out0[i] <- out1[i] != 0 ? out0[i] / out1[i] : 0 for the n
 * elements (what ASP_F_RATIO does inside asp_project2d; used after a cross-GPU sum of
 * the two component maps).  Device pointers only, ordered on `stream`.
 */
int asp_ratio(float *out0, const float *out1, int64_t n, int32_t device, void *stream);

/* Periodic-box operations: pb_flags of asp_stage_particles, op of asp_periodic. */
#define ASP_PB_WRAP 0x1             /* make_periodic (_periodic_box_manipulations.py:36-48) */
#define ASP_PB_SHIFT_ORIGIN 0x2     /* shift_origin (:54-57): x - origin, then wrapped       */
#define ASP_PB_SHIFT_CENTRE 0x4     /* shift_centre (:63-69): x + (L/2 - centre), wrapped    */
#define ASP_PB_ORIGIN_IS_CENTRE 0x8 /* the box is [-L/2, L/2) instead of [0, L)              */
#define ASP_PB_IMAGES 0x10          /* asp_stage_particles: append periodic images           */
#define ASP_PB_DISPLACEMENT 0x20    /* asp_periodic: calculate_wrapped_displacement (:10-20) */

/*
 * Snapshot -> projector staging.  Replaces the host-side step of
 * create_image that takes the reader's arrays (io/data_structures/_SnapshotBase.py:599-725:
 * positions (n, 3) float64 row-major, smoothing lengths and properties float64) to the
 * float32 structure of arrays asp_project2d consumes, with the axis selection of
 * _projector.py:38-46 (axis 0 = X -> (y, z), 1 = Y -> (x, z), 2 = Z -> (x, y)); the
 * conversion (round to nearest, as NumPy's astype(float32)) runs on the device.
 *   u, v, hf, a0f, a1f: DEVICE float32 outputs on `device` of capacity cap (hf, a0f, a1f
 *   may be NULL, as may their inputs h, a0, a1).  Inputs are host pointers, copied in
 *   chunks with copy and conversion overlapped, unless ASP_F_DEVICE_PTRS.
 * Periodic box, pb_flags: at most one of ASP_PB_WRAP,
 *   ASP_PB_SHIFT_ORIGIN, ASP_PB_SHIFT_CENTRE (centre = the new origin / centre, 3 values;
 *   the reference helpers' fp64 arithmetic on the two projected coordinates), optionally
 *   ASP_PB_ORIGIN_IS_CENTRE, and ASP_PB_IMAGES: every particle inside the box
 *   [lo, lo + L)^2 (lo = 0, or -L/2) whose reach 2|h| (+ a 2^-20 margin) crosses a face
 *   gets a copy one box width over (up to 3 per particle), appended after the n
 *   originals in an unspecified order -- projecting the result over the box gives the
 *   periodic map.  *n_out = n + images; if that exceeds cap the images beyond cap are
 *   dropped and the call returns ASP_ERR_INVALID with *n_out set to the size needed.
 */
int asp_stage_particles(const double *positions, const double *h, const double *a0,
                        const double *a1, int64_t n, int32_t axis, const double *centre,
                        double box_width, int32_t pb_flags, float *u, float *v, float *hf,
                        float *a0f, float *a1f, int64_t cap, int64_t *n_out, int32_t flags,
                        int32_t device, void *stream);

/*
 * The periodic-box helpers of tools/_periodic_box_manipulations.py on the device, fp64,
 * bit-identical to the reference: op = ASP_PB_WRAP (make_periodic / calculate_periodic,
 * :36-48), ASP_PB_SHIFT_ORIGIN (shift_origin :54-57, b = new origin), ASP_PB_SHIFT_CENTRE
 * (shift_centre :63-69, b = new centre), ASP_PB_DISPLACEMENT
 * (calculate_wrapped_displacement :10-20, a = from, b = to).  out[i] for i < n; a and b
 * repeat with periods pa and pb (NumPy broadcasting of a (3,) vector over (N, 3)).
 * Device pointers, ordered on `stream`.
 */
int asp_periodic(int32_t op, const double *a, int64_t pa, const double *b, int64_t pb,
                 int64_t n, double box_width, int32_t origin_is_centre, double *out,
                 int32_t device, void *stream);

/*
 * calculate_wrapped_distance (_periodic_box_manipulations.py:22-34): per row of 3, the
 * length (squared != 0: its square) of the wrapped displacement; from / to repeat with
 * periods pf / pt (elements).  Device pointers, ordered on `stream`.
 */
int asp_wrapped_distance(const double *from, int64_t pf, const double *to, int64_t pt,
                         int64_t rows, double box_width, int32_t squared, double *out,
                         int32_t device, void *stream);

/*
 * Smoothing lengths from the k-th nearest neighbour: replaces
 * the scipy KDTree query of io/SWIFT/_SnapshotSWIFT.py:62-83 (dark matter: h = distance to
 * the k-th nearest particle, the particle itself counted, k = 32 there):
 *   h[i] = sqrt(d2_(k)),  d2 = ((x_i - x_j)^2 + (y_i - y_j)^2) + (z_i - z_j)^2  (fp64),
 * d2_(k) the k-th smallest over all j, j = i included -- scipy's Euclidean distance, so
 * the result is bit-identical to the reference's; +inf when n < k (scipy's value for a
 * missing neighbour).  positions (n, 3) float64 row-major, h float64; 1 <= k <= 64,
 * n < 2^31.  Host pointers unless ASP_F_DEVICE_PTRS (then ordered on `stream`).
 */
int asp_knn_smoothing_lengths(const double *positions, int64_t n, int32_t k, double *h,
                              int32_t flags, int32_t device, void *stream);

/*
 * Ionisation-table interpolation: replaces the scipy
 * RegularGridInterpolator of data_structures/_IonisationTable.py:44-58 (linear,
 * bounds_error=False, fill_value=-inf; the HM01 tables of
 * io/ionisation_tables/_HM01.py:61-92 are 3-D over (log10 n_H, log10 T, redshift)).
 * table: (n0, n1, n2) float64 C-order on strictly ascending axes g0, g1, g2; points:
 * (n, 3) rows, or (n, 2) rows with `zvalue` inserted at axis `zaxis` (ncol = 2;
 * evaluate_at_redshift, :54-58).  out[i] = the interpolated value, bit-identical to scipy
 * 1.15's linear evaluation (fill outside the table, NaN for NaN input);
 * mode 1: out[i] = (a0[i] * a1[i]) * value, mode 2: (a0[i] * a1[i]) * 10^value -- the ion
 * masses m * X_element * f_ion that feed asp_project2d for an ion column map.  Device
 * pointers, ordered on `stream`.
 */
int asp_table_interp3(const double *table, int32_t n0, int32_t n1, int32_t n2,
                      const double *g0, const double *g1, const double *g2,
                      const double *points, int32_t ncol, int32_t zaxis, double zvalue,
                      int64_t n, double fill, int32_t mode, const double *a0, const double *a1,
                      double *out, int32_t device, void *stream);

/*
 * The same for any number of table axes (IonisationTableBase takes N input dimensions,
 * _IonisationTable.py:31-49): table (shape[0], ..., shape[ndim-1]) float64 C-order, axes[d]
 * a device pointer to axis d (a HOST array of ndim pointers; shape is a host array too),
 * 1 <= ndim <= 6.  points: (n, ndim) rows, or (n, ndim - 1) rows with `zvalue` inserted at
 * axis `zaxis`.  order 0: scipy's _evaluate_linear (weights multiplied first, every ndim);
 * order 1: its Cython 2-D fast path (value times w0 times w1), which scipy takes for a
 * writeable native-float64 2-D table.  Bit-identical to scipy 1.15; fill / NaN / mode as
 * asp_table_interp3.
 */
int asp_table_interp(const double *table, int32_t ndim, const int32_t *shape,
                     const double *const *axes, const double *points, int32_t ncol,
                     int32_t zaxis, double zvalue, int64_t n, double fill, int32_t mode,
                     int32_t order, const double *a0, const double *a1, double *out,
                     int32_t device, void *stream);

/*
 * Statistics of the last asp_project2d call on `device` (inspection / roofline):
 * stats[0] = records binned (particle x GPU-tile insertions), stats[1] = work items,
 * stats[2] = wide particles, stats[3] = GPU tile edge (pixels), stats[4] = GPU tiles,
 * stats[5] = records per work item, stats[6] = split tiles, stats[7] = partial slabs,
 * stats[8] = records in the large (gathered) stream; with the environment variable
 * ASP_COUNT_EVALS set (diagnostic: one extra kernel, a host sync), the (pixel, particle)
 * lane-slots the deposit kernels spend: stats[9] total = stats[10] small / mid-size stream
 * + stats[11] gathered large stream + stats[12] wide particles (else 0); stats[13] how the
 * records were scattered (1 the speculative scatter enqueued before the counter read-back
 * was kept, 2 record-placement trials, 3 the speculative scatter found the buffers too
 * small and was relaunched after growing them, 0 one plain launch; the largest code over
 * the passes), stats[14] scatter runs of the placement trials.  Images of more than 4096
 * tiles and batched calls: the sums over all passes.
 */
int asp_last_stats(int32_t device, int64_t *stats, int32_t nstats);

/*
 * Stage timing with HIP events recorded on the call's stream around every launch
 * (enable != 0 starts and resets, 0 stops).  asp_profile_read returns, per stage, the
 * summed milliseconds and the number of launches since the last reset.  Stages:
 * 0 memset, 1 count, 2 colscan, 3 tilescan, 4 scatter, 5 scale, 6 deposit, 7 merge,
 * 8 wide, 9 ratio; cube (asp_project3d): 10 count, 11 colscan, 12 tilescan, 13 scatter,
 * 14 deposit, 15 merge; 16 gather (2-D gathered deposit of the large-record stream).
 */
int asp_profile(int32_t device, int32_t enable);
/* As asp_profile(device, 1), but events only around the stages whose bit is set in
 * `stage_mask` (bit k = stage k; 0 stops).  Each event pair costs the stream a few
 * microseconds, so a timed run marks only the kernel it reports (bench.py). */
int asp_profile_stages(int32_t device, uint32_t stage_mask);
int asp_profile_read(int32_t device, double *ms_sum, int64_t *launches, int32_t nstages);

/* Release the cached device workspace of `device` (-1: all devices). */
int asp_release(int32_t device);

#ifdef __cplusplus
}
#endif

#endif /* ASP_H */
