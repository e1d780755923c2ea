// asp_stage.hip -- the two rows either side of the projection path:
//
//   (f)1 snapshot -> device SoA: the reader's float64 arrays (positions (n, 3) row-major,
//        _SnapshotBase.py:599-725) become the projector's float32 structure of arrays in
//        HBM, axis-selected as create_image does (_projector.py:38-46) -- the fp64 -> fp32
//        conversion the Python wrapper used to do on the host, as a device pass that
//        streams the fp64 fields through HBM once;
//   (f)2 periodic boxes: the reference's helpers (tools/_periodic_box_manipulations.py:
//        10-72: wrapped displacement / distance, make_periodic, shift_origin,
//        shift_centre) on the device with the same fp64 operations, and periodic images
//        for maps of a periodic box (a particle within reach of a box face gets a copy one
//        box width over, so its footprint wraps).
//
// All of it is element-wise fp64 work: HBM-bound streaming kernels, no LDS, no MFMA.
// Every fp64 expression is the reference's (NumPy's) operation sequence, so results are
// bit-identical to it (tests/test_gpu_stage.py against tests/golden/g8_periodic.npz).
#include <hip/hip_runtime.h>

#include <cstring>
#include <thread>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/asp.h"
#include "asp_host.hpp"

namespace asp {

constexpr int kStageBlock = 256;

__device__ __forceinline__ double sign1(double x) {  // np.sign (NaN stays NaN)
    return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x);
}

// make_periodic (_periodic_box_manipulations.py:36-43) on one coordinate: ONE wrap by a
// box width, as the reference does (values further out stay out; NaN stays NaN).
//   positions[wrap] = -np.sign(positions[wrap] (+ half_box_width)) * box_width + positions[wrap]
__device__ __forceinline__ double wrap1(double x, double L, int centred) {
    if (centred) {
        double hb = L / 2;
        if (x < -hb || x >= hb) x = -sign1(x + hb) * L + x;
    } else {
        if (x < 0.0 || x >= L) x = -sign1(x) * L + x;
    }
    return x;
}

// calculate_wrapped_displacement (:10-20) on one component: d = to - from, and where
// |d| > L / 2, d - sign(d) * L.
__device__ __forceinline__ double wrap_delta(double d, double L) {
    return fabs(d) > L / 2 ? d - sign1(d) * L : d;
}

// The element-wise periodic operations, out[i] for i < n.  a (period pa) and b (period
// pb) are broadcast by repetition, as NumPy broadcasts a (3,) origin over (N, 3).
//   ASP_PB_WRAP          make_periodic(a)                               (:36-48)
//   ASP_PB_SHIFT_ORIGIN  make_periodic(a - b)                           (:54-57)
//   ASP_PB_SHIFT_CENTRE  make_periodic(a + ((L / 2) - b))  (centred: shift_origin, :63-69)
//   ASP_PB_DISPLACEMENT  wrap_delta(b - a)   (a = from, b = to)         (:10-20)
__global__ __launch_bounds__(kStageBlock) void k_periodic(int op, const double* __restrict__ a,
                                                          long long pa, const double* __restrict__ b,
                                                          long long pb, long long n, double L,
                                                          int centred, double* __restrict__ out) {
    long long i = (long long)blockIdx.x * kStageBlock + threadIdx.x;
    long long stride = (long long)gridDim.x * kStageBlock;
    for (; i < n; i += stride) {
        double x = a[pa == n ? i : i % pa];
        double r;
        if (op == ASP_PB_WRAP) {
            r = wrap1(x, L, centred);
        } else if (op == ASP_PB_SHIFT_ORIGIN || (op == ASP_PB_SHIFT_CENTRE && centred)) {
            r = wrap1(x - b[pb == n ? i : i % pb], L, centred);
        } else if (op == ASP_PB_SHIFT_CENTRE) {
            r = wrap1(x + ((L / 2) - b[pb == n ? i : i % pb]), L, 0);
        } else {
            r = wrap_delta(b[pb == n ? i : i % pb] - x, L);
        }
        out[i] = r;
    }
}

// calculate_wrapped_distance (:22-34) for rows of 3: the displacement, then
// (d0^2 + d1^2) + d2^2 (NumPy's sum over a length-3 axis) and sqrt unless squared.
__global__ __launch_bounds__(kStageBlock) void k_wrapped_distance(
    const double* __restrict__ from, long long pf, const double* __restrict__ to, long long pt,
    long long rows, double L, int squared, double* __restrict__ out) {
    long long j = (long long)blockIdx.x * kStageBlock + threadIdx.x;
    if (j >= rows) return;
    const long long ne = 3 * rows;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        long long e = 3 * j + k;
        double d = wrap_delta(to[pt == ne ? e : e % pt] - from[pf == ne ? e : e % pf], L);
        s = k == 0 ? d * d : s + d * d;
    }
    out[j] = squared ? s : sqrt(s);
}

// Staging parameters (fp64, from the host).
struct StageArgs {
    int a, b;      // position columns projected to (u, v)
    int op;        // 0, ASP_PB_WRAP, ASP_PB_SHIFT_ORIGIN or ASP_PB_SHIFT_CENTRE
    int centred;   // origin_is_centre
    double L;      // box width
    double s[3];   // the shift operand (new centre / origin)
    int images;    // append periodic images
    double lo;     // box interval [lo, lo + L) of both projected axes
};

__device__ __forceinline__ double stage_coord(const StageArgs& S, double x, int c) {
    if (S.op == ASP_PB_WRAP) return wrap1(x, S.L, S.centred);
    if (S.op == ASP_PB_SHIFT_ORIGIN || (S.op == ASP_PB_SHIFT_CENTRE && S.centred))
        return wrap1(x - S.s[c], S.L, S.centred);
    if (S.op == ASP_PB_SHIFT_CENTRE) return wrap1(x + ((S.L / 2) - S.s[c]), S.L, 0);
    return x;
}

// Periodic image shifts on one axis: the k (copy at x + k L) whose reach [x + kL - R,
// x + kL + R] meets the box [lo, lo + L); only particles inside the box get copies.  R
// carries a 2^-20 L margin, far above the rounding of these fp64 expressions, so no copy
// that can contribute is missed (an extra one would contribute nothing: the projection
// decides every pair exactly).
__device__ __forceinline__ void image_range(double x, double R, double lo, double L, int& k0,
                                            int& k1) {
    k0 = (int)floor((lo - x - R) / L) + 1;
    k1 = (int)ceil((lo + L - x + R) / L) - 1;
}

constexpr int kMaxImageShift = 3;  // reach <= ~3 box widths per side (else an error)

// Particles [i0, i1) (row i at index i - i0 of this chunk's arrays): outputs at index i;
// periodic images appended at n + (claimed slot) while below cap.  The map of the staged
// set over the box is then the sum over all periodic images of every particle.
__global__ __launch_bounds__(kStageBlock) void k_stage(
    StageArgs S, const double* __restrict__ pos, const double* __restrict__ h,
    const double* __restrict__ a0, const double* __restrict__ a1, long long i0, long long i1,
    long long n, float* __restrict__ u, float* __restrict__ v, float* __restrict__ hf,
    float* __restrict__ a0f, float* __restrict__ a1f, long long cap,
    unsigned long long* __restrict__ nimg) {
    long long i = i0 + (long long)blockIdx.x * kStageBlock + threadIdx.x;
    bool live = i < i1;
    long long r = i - i0;
    double x = 0.0, y = 0.0, hd = 0.0, p0 = 0.0, p1 = 0.0;
    if (live) {
        x = stage_coord(S, pos[3 * r + S.a], S.a);
        y = stage_coord(S, pos[3 * r + S.b], S.b);
        if (h) hd = h[r];
        if (a0) p0 = a0[r];
        if (a1) p1 = a1[r];
        u[i] = (float)x;
        v[i] = (float)y;
        if (hf) hf[i] = (float)hd;
        if (a0f) a0f[i] = (float)p0;
        if (a1f) a1f[i] = (float)p1;
    }
    if (!S.images) return;
    int kx0 = 0, kx1 = 0, ky0 = 0, ky1 = 0;
    if (live) {
        const double R = 2.0 * fabs(hd) * (1.0 + 0x1p-20) + 0x1p-20 * S.L;
        const bool inside = x >= S.lo && x < S.lo + S.L && y >= S.lo && y < S.lo + S.L;
        if (inside && R > 0.0 && R <= kMaxImageShift * S.L) {  // h == 0 or NaN: none
            image_range(x, R, S.lo, S.L, kx0, kx1);
            image_range(y, R, S.lo, S.L, ky0, ky1);
        } else if (inside && R > kMaxImageShift * S.L && R == R) {
            atomicAdd(nimg + 1, 1ull);  // reach beyond the supported shifts: reported
        }
    }
    const int k = (kx1 - kx0 + 1) * (ky1 - ky0 + 1) - 1;
    // one claim per wave; a lane's images follow those of the lanes below it
    unsigned long long m = __ballot(k > 0);
    if (!m) return;
    int lane = threadIdx.x & 63;
    int before = 0, tot = 0;
    for (int l = 0; l < 64; ++l) {
        int kl = __shfl(k, l);
        before += l < lane ? kl : 0;
        tot += kl;
    }
    int leader = __builtin_ctzll(m);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(nimg, (unsigned long long)tot);
    base = __shfl(base, leader);
    if (k == 0) return;
    long long slot = n + (long long)base + before;
    for (int kx = kx0; kx <= kx1; ++kx)
        for (int ky = ky0; ky <= ky1; ++ky) {
            if (kx == 0 && ky == 0) continue;
            if (slot < cap) {
                u[slot] = (float)(x + kx * S.L);
                v[slot] = (float)(y + ky * S.L);
                if (hf) hf[slot] = (float)hd;
                if (a0f) a0f[slot] = (float)p0;
                if (a1f) a1f[slot] = (float)p1;
            }
            ++slot;
        }
}

static unsigned grid_for(long long n) {
    long long b = (n + kStageBlock - 1) / kStageBlock;
    return (unsigned)std::max<long long>(1, std::min<long long>(b, 1LL << 20));
}

constexpr long long kStageChunk = 1LL << 22;  // particles per host -> device chunk

static int stage_particles(const double* pos, const double* h, const double* a0,
                           const double* a1, long long n, int axis, const double* centre,
                           double box_width, int pb_flags, float* u, float* v, float* hf,
                           float* a0f, float* a1f, long long cap, long long* n_out, int flags,
                           int device, hipStream_t st) {
    if (n < 0) return fail(ASP_ERR_INVALID, "n < 0");
    if (axis < 0 || axis > 2)
        return fail(ASP_ERR_INVALID, "projection axis must be 0 (X), 1 (Y) or 2 (Z)");
    if (n > 0 && (!pos || !u || !v)) return fail(ASP_ERR_INVALID, "NULL positions or outputs");
    if (cap < n) return fail(ASP_ERR_INVALID, "output capacity below n");
    const int op = pb_flags & (ASP_PB_WRAP | ASP_PB_SHIFT_ORIGIN | ASP_PB_SHIFT_CENTRE);
    if (op != 0 && op != ASP_PB_WRAP && op != ASP_PB_SHIFT_ORIGIN && op != ASP_PB_SHIFT_CENTRE)
        return fail(ASP_ERR_INVALID, "at most one of ASP_PB_WRAP, _SHIFT_ORIGIN, _SHIFT_CENTRE");
    const bool images = (pb_flags & ASP_PB_IMAGES) != 0;
    if ((op || images) && !(box_width > 0.0 && std::isfinite(box_width)))
        return fail(ASP_ERR_INVALID, "box_width must be finite and > 0");
    if ((op == ASP_PB_SHIFT_ORIGIN || op == ASP_PB_SHIFT_CENTRE) && !centre)
        return fail(ASP_ERR_INVALID, "the shift needs a centre / origin (3 values)");
    if (images && !h) return fail(ASP_ERR_INVALID, "periodic images need smoothing lengths");
    StageArgs S{};
    static const int cols[3][2] = {{1, 2}, {0, 2}, {0, 1}};  // _projector.py:38-46
    S.a = cols[axis][0];
    S.b = cols[axis][1];
    S.op = op;
    S.centred = (pb_flags & ASP_PB_ORIGIN_IS_CENTRE) != 0;
    S.L = box_width;
    for (int k = 0; k < 3; ++k) S.s[k] = centre ? centre[k] : 0.0;
    S.images = images;
    S.lo = S.centred ? -(box_width / 2) : 0.0;
    ASP_TRY(set_device(device));
    Workspace& ws = g_ws[device];
    std::lock_guard<std::mutex> lock(ws.mu);
    ASP_TRY(ws_begin(ws, st));
    WsEnd ws_end_(ws, st);
    ASP_TRY(ensure(ws.aux[5], 2 * sizeof(unsigned long long)));
    unsigned long long* dimg = (unsigned long long*)ws.aux[5].p;
    ASP_HIP(hipMemsetAsync(dimg, 0, 2 * sizeof(unsigned long long), st));
    if ((flags & ASP_F_DEVICE_PTRS) || n == 0) {
        if (n > 0) {
            hipLaunchKernelGGL(k_stage, dim3(grid_for(n)), dim3(kStageBlock), 0, st, S, pos, h, a0,
                               a1, 0LL, n, n, u, v, hf, a0f, a1f, cap, dimg);
            ASP_HIP(hipGetLastError());
        }
    } else {
        // Host arrays: chunks copied (pinned bounce buffers) into two device staging sets
        // alternately (stream st, side stream): the copy of chunk c + 1 overlaps the
        // conversion of chunk c.
        ASP_TRY(ensure_side(ws));
        const long long C = std::min<long long>(kStageChunk, n);
        for (int s = 0; s < 2; ++s) ASP_TRY(ensure(ws.aux[s], (size_t)C * 6 * sizeof(double)));
        hipStream_t ss[2] = {st, ws.side};
        ASP_HIP(hipEventRecord(ws.scan_ev, st));
        ASP_HIP(hipStreamWaitEvent(ws.side, ws.scan_ev, 0));  // behind the counter reset
        int c = 0;
        for (long long i0 = 0; i0 < n; i0 += C, ++c) {
            const long long m = std::min(C, n - i0);
            hipStream_t s = ss[c & 1];
            double* d = (double*)ws.aux[c & 1].p;
            double *dp = d, *dh = d + 3 * C, *d0 = d + 4 * C, *d1 = d + 5 * C;
            ASP_TRY(h2d_staged(ws, dp, pos + 3 * i0, (size_t)m * 3 * sizeof(double), s));
            if (h) ASP_TRY(h2d_staged(ws, dh, h + i0, (size_t)m * sizeof(double), s));
            if (a0) ASP_TRY(h2d_staged(ws, d0, a0 + i0, (size_t)m * sizeof(double), s));
            if (a1) ASP_TRY(h2d_staged(ws, d1, a1 + i0, (size_t)m * sizeof(double), s));
            hipLaunchKernelGGL(k_stage, dim3(grid_for(m)), dim3(kStageBlock), 0, s, S, dp,
                               h ? dh : nullptr, a0 ? d0 : nullptr, a1 ? d1 : nullptr, i0, i0 + m,
                               n, u, v, hf, a0f, a1f, cap, dimg);
            ASP_HIP(hipGetLastError());
        }
        ASP_HIP(hipEventRecord(ws.done_ev, ws.side));
        ASP_HIP(hipStreamWaitEvent(st, ws.done_ev, 0));
    }
    unsigned long long nimg[2] = {0, 0};
    ASP_HIP(hipMemcpyAsync(nimg, dimg, sizeof(nimg), hipMemcpyDeviceToHost, st));
    ASP_HIP(hipStreamSynchronize(st));
    ASP_TRY(ws_end_.finish());
    if (nimg[1])
        return fail(ASP_ERR_UNSUPPORTED, std::to_string(nimg[1]) + " particles reach beyond " +
                                             std::to_string(kMaxImageShift) +
                                             " box widths (2|h| > 3 L): periodic images unsupported");
    *n_out = n + (long long)nimg[0];
    if (*n_out > cap)
        return fail(ASP_ERR_INVALID, "periodic images exceed the output capacity (" +
                                         std::to_string(*n_out) + " > " + std::to_string(cap) +
                                         "); n_out holds the size needed");
    return ASP_OK;
}

// ----------------------------------------------------------------------------------
// Pinned staging (reader arrays -> HBM).  A DMA from pageable
// memory is staged by the runtime piece by piece with the CPU waiting on each; here two
// 32 MiB pinned buffers alternate: piece k is copied into buffer k % 2 by 4 host threads
// while the DMA of piece k - 1 runs, then its DMA is enqueued on the caller's stream.  A
// buffer is refilled only after its previous DMA completed (event).
// ----------------------------------------------------------------------------------
constexpr size_t kPinBytes = (size_t)32 << 20;
constexpr int kPinThreads = 4;

static void par_copy(char* d, const char* s, size_t n) {
    if (n < ((size_t)4 << 20)) {
        memcpy(d, s, n);
        return;
    }
    const size_t part = ((n + kPinThreads - 1) / kPinThreads + 4095) & ~(size_t)4095;
    std::thread th[kPinThreads - 1];
    int nt = 0;
    for (int t = 1; t < kPinThreads; ++t) {
        const size_t o = part * t;
        if (o >= n) break;
        th[nt++] = std::thread([=] { memcpy(d + o, s + o, std::min(part, n - o)); });
    }
    memcpy(d, s, std::min(part, n));
    for (int t = 0; t < nt; ++t) th[t].join();
}

int h2d_staged(Workspace& ws, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes == 0) return ASP_OK;
    for (int b = 0; b < 2; ++b) {
        if (!ws.pin[b]) {
            ASP_HIP(hipHostMalloc(&ws.pin[b], kPinBytes, hipHostMallocDefault));
            ASP_HIP(hipEventCreateWithFlags(&ws.pin_ev[b], hipEventDisableTiming));
            ws.pin_busy[b] = false;
        }
    }
    for (size_t off = 0; off < bytes; off += kPinBytes) {
        const int b = ws.pin_next & 1;
        ws.pin_next ^= 1;
        const size_t len = std::min(kPinBytes, bytes - off);
        if (ws.pin_busy[b]) ASP_HIP(hipEventSynchronize(ws.pin_ev[b]));
        par_copy((char*)ws.pin[b], (const char*)src + off, len);
        ASP_HIP(hipMemcpyAsync((char*)dst + off, ws.pin[b], len, hipMemcpyHostToDevice, st));
        ASP_HIP(hipEventRecord(ws.pin_ev[b], st));
        ws.pin_busy[b] = true;
    }
    return ASP_OK;
}

void release_pinned(Workspace& ws) {
    for (int b = 0; b < 2; ++b) {
        if (ws.pin_busy[b]) (void)hipEventSynchronize(ws.pin_ev[b]);
        if (ws.pin[b]) (void)hipHostFree(ws.pin[b]);
        if (ws.pin_ev[b]) (void)hipEventDestroy(ws.pin_ev[b]);
        ws.pin[b] = nullptr;
        ws.pin_ev[b] = nullptr;
        ws.pin_busy[b] = false;
    }
}

// Reader arrays already on the device -> fp32 working copies (no periodic options).
int stage_device(const double* pos, const double* h, const double* a0, const double* a1,
                 long long n, int axis, float* u, float* v, float* hf, float* a0f, float* a1f,
                 hipStream_t st) {
    if (n == 0) return ASP_OK;
    StageArgs S{};
    static const int cols[3][2] = {{1, 2}, {0, 2}, {0, 1}};  // _projector.py:38-46
    S.a = cols[axis][0];
    S.b = cols[axis][1];
    hipLaunchKernelGGL(k_stage, dim3(grid_for(n)), dim3(kStageBlock), 0, st, S, pos, h, a0, a1,
                       0LL, n, n, u, v, hf, a0f, a1f, n, (unsigned long long*)nullptr);
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}

}  // namespace asp

using namespace asp;

extern "C" {

int asp_stage_particles(const double* positions, const double* h, const double* a0,
                        const double* a1, int64_t n, int32_t axis, const double* centre,
                        double box_width, int32_t pb_flags, float* u, float* v, float* hf,
                        float* a0f, float* a1f, int64_t cap, int64_t* n_out, int32_t flags,
                        int32_t device, void* stream) {
    t_err.clear();
    long long no = 0;
    int rc = stage_particles(positions, h, a0, a1, n, axis, centre, box_width, pb_flags, u, v,
                             hf, a0f, a1f, cap, &no, flags, device, (hipStream_t)stream);
    if (n_out) *n_out = no;
    return rc;
}

int asp_periodic(int32_t op, const double* a, int64_t pa, const double* b, int64_t pb,
                 int64_t n, double box_width, int32_t origin_is_centre, double* out,
                 int32_t device, void* stream) {
    t_err.clear();
    if (op != ASP_PB_WRAP && op != ASP_PB_SHIFT_ORIGIN && op != ASP_PB_SHIFT_CENTRE &&
        op != ASP_PB_DISPLACEMENT)
        return fail(ASP_ERR_INVALID, "unknown periodic operation");
    if (n < 0 || pa < 1 || (op != ASP_PB_WRAP && pb < 1)) return fail(ASP_ERR_INVALID, "bad sizes");
    if (n == 0) return ASP_OK;
    if (!a || !out || (op != ASP_PB_WRAP && !b)) return fail(ASP_ERR_INVALID, "NULL array");
    ASP_TRY(set_device(device));
    hipLaunchKernelGGL(k_periodic, dim3(grid_for(n)), dim3(kStageBlock), 0, (hipStream_t)stream,
                       (int)op, a, (long long)pa, b, (long long)(op == ASP_PB_WRAP ? 1 : pb),
                       (long long)n, box_width, (int)(origin_is_centre != 0), out);
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}

int asp_wrapped_distance(const double* from, int64_t pf, const double* to, int64_t pt,
                         int64_t rows, double box_width, int32_t squared, double* out,
                         int32_t device, void* stream) {
    t_err.clear();
    if (rows < 0 || pf < 1 || pt < 1) return fail(ASP_ERR_INVALID, "bad sizes");
    if (rows == 0) return ASP_OK;
    if (!from || !to || !out) return fail(ASP_ERR_INVALID, "NULL array");
    ASP_TRY(set_device(device));
    hipLaunchKernelGGL(k_wrapped_distance, dim3(grid_for(rows)), dim3(kStageBlock), 0,
                       (hipStream_t)stream, from, (long long)pf, to, (long long)pt,
                       (long long)rows, box_width, (int)(squared != 0), out);
    ASP_HIP(hipGetLastError());
    return ASP_OK;
}

}  // extern "C"
