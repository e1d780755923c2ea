// asp_host.hpp -- host runtime shared by the 2-D and 3-D projectors: errors, the
// per-device workspace cache (HBM buffers reused across calls), HIP-event stage timing.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/asp.h"

namespace asp {

inline thread_local std::string t_err;

inline int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}

#define ASP_HIP(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(ASP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Buf {
    void* p = nullptr;
    size_t cap = 0;
};

constexpr int kStages = 17;
constexpr int kMarks = 8;  // launches of one stage timed per call
enum Stage {
    kSMemset = 0, kSCount, kSColscan, kSTilescan, kSScatter, kSScale, kSDeposit, kSMerge,
    kSWide, kSRatio,
    // 3-D cube (asp_project3d)
    kS3Count = 10, kS3Colscan, kS3Tilescan, kS3Scatter, kS3Deposit, kS3Merge,
    kSBand = 16  // 2-D row-band deposit of non-small records
};

struct Workspace {
    std::mutex mu;
    // HIP-event profiling (asp_profile): per-stage start/stop events of the last call,
    // folded into the running sums at the next call or at asp_profile_read.
    bool prof = false;
    unsigned prof_mask = 0u;  // stages timed (bit k = stage k)
    // Two event sets, used by alternate calls: a call folds the set of the call two back,
    // which has completed by then (the previous call's counter read-back waited for it),
    // so profiling never makes the host wait for the GPU to drain between calls.
    hipEvent_t ev[2][kStages][kMarks][2] = {};
    int ev_live[2][kStages] = {};  // marks recorded per set (a stage may launch once per
                                   // particle chunk)
    int pset = 0;                  // the set the current call records into
    double stage_ms[kStages] = {};
    long long stage_n[kStages] = {};
    Buf knn[7];  // asp_knn_smoothing_lengths
    Buf in[5], out[2], hist, cmx, tile_total, tile_start, tile_k, items, merges, counters, recs,
        wide, slabs, morton, aux[6];
    int* h_counters = nullptr;  // pinned
    int morton_ntx = -1, morton_nty = -1;
    Buf morton3;  // brick order of the 3-D cube
    int morton3_key[3] = {-1, -1, -1};
    long long stats[9] = {0};
    // Chunked 2-D pipeline: deposits run on a side stream, each behind its chunk's scatter.
    hipStream_t side = nullptr;
    hipEvent_t chunk_ev[kMarks] = {};
    hipEvent_t done_ev = nullptr;
    hipEvent_t scan_ev = nullptr;  // 2-D pipeline: binning scans done (st)
    hipEvent_t cnt_ev = nullptr;   // ... and their counters copied to the host (side)
};

inline int ensure_side(Workspace& ws) {
    if (ws.side) return ASP_OK;
    ASP_HIP(hipStreamCreateWithFlags(&ws.side, hipStreamNonBlocking));
    for (int c = 0; c < kMarks; ++c)
        ASP_HIP(hipEventCreateWithFlags(&ws.chunk_ev[c], hipEventDisableTiming));
    ASP_HIP(hipEventCreateWithFlags(&ws.done_ev, hipEventDisableTiming));
    ASP_HIP(hipEventCreateWithFlags(&ws.scan_ev, hipEventDisableTiming));
    ASP_HIP(hipEventCreateWithFlags(&ws.cnt_ev, hipEventDisableTiming));
    return ASP_OK;
}

inline Workspace g_ws[64];

inline int prof_fold_set(Workspace& ws, int set) {
    for (int k = 0; k < kStages; ++k) {
        for (int j = 0; j < ws.ev_live[set][k]; ++j) {
            ASP_HIP(hipEventSynchronize(ws.ev[set][k][j][1]));
            float ms = 0.0f;
            ASP_HIP(hipEventElapsedTime(&ms, ws.ev[set][k][j][0], ws.ev[set][k][j][1]));
            ws.stage_ms[k] += ms;
            ws.stage_n[k] += 1;
        }
        ws.ev_live[set][k] = 0;
    }
    return ASP_OK;
}

// At the start of a call: switch sets, folding what the call two back recorded there.
inline int prof_next(Workspace& ws) {
    ws.pset ^= 1;
    return prof_fold_set(ws, ws.pset);
}

// Everything recorded so far (asp_profile_read).
inline int prof_fold(Workspace& ws) {
    int rc = prof_fold_set(ws, ws.pset ^ 1);
    return rc != ASP_OK ? rc : prof_fold_set(ws, ws.pset);
}

struct StageMark {
    Workspace& ws;
    int k;
    hipStream_t st;
    bool on;
    StageMark(Workspace& w, int stage, hipStream_t s)
        : ws(w), k(stage), st(s),
          on(w.prof && ((w.prof_mask >> stage) & 1u) && w.ev_live[w.pset][stage] < kMarks) {
        if (on) (void)hipEventRecord(ws.ev[ws.pset][k][ws.ev_live[ws.pset][k]][0], st);
    }
    void done() {
        if (on) {
            (void)hipEventRecord(ws.ev[ws.pset][k][ws.ev_live[ws.pset][k]][1], st);
            ws.ev_live[ws.pset][k] += 1;
        }
    }
};

inline int ensure(Buf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return ASP_OK;
    if (b.p) {
        hipError_t e = hipFree(b.p);
        (void)e;
        b.p = nullptr;
        b.cap = 0;
    }
    size_t want = bytes + bytes / 4;
    hipError_t e = hipErrorOutOfMemory;
    if (want >= (size_t(1) << 28) && getenv("ASP_CONTIG") && atoi(getenv("ASP_CONTIG")))
        e = hipExtMallocWithFlags(&b.p, want, hipDeviceMallocContiguous);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        e = hipMalloc(&b.p, want);
    } else if (getenv("ASP_DEBUG_ALLOC")) {
        fprintf(stderr, "[asp] contiguous ");
    }
    if (e != hipSuccess) {
        e = hipMalloc(&b.p, bytes);
        want = bytes;
    }
    if (e != hipSuccess) {
        b.p = nullptr;
        return fail(ASP_ERR_NOMEM, "hipMalloc(" + std::to_string(bytes) + ") failed: " +
                                       hipGetErrorString(e));
    }
    b.cap = want;
    if (want >= (size_t(1) << 28) && getenv("ASP_DEBUG_ALLOC"))
        fprintf(stderr, "[asp] hipMalloc %zu B at %p\n", want, b.p);
    return ASP_OK;
}

#define ASP_TRY(expr)                  \
    do {                               \
        int rc_ = (expr);              \
        if (rc_ != ASP_OK) return rc_; \
    } while (0)

#define ASP_LAUNCHED()                                                                    \
    do {                                                                                  \
        hipError_t e_ = hipGetLastError();                                                \
        if (e_ != hipSuccess)                                                             \
            return fail(ASP_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)


}  // namespace asp
