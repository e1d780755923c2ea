// asp_binning.hpp -- tile/brick binning stages shared by the 2-D map and the 3-D cube.
//
// The count pass of either geometry leaves hist[block][tile] (insertions per workgroup
// and tile); these two kernels turn it into record offsets and the deposit work list.
// Nothing here depends on the geometry: a "tile" is a 64x64 pixel tile (2-D) or a
// 16x16x32 voxel brick (3-D).
#pragma once

#include "asp_device.hpp"

namespace asp {


// Counter words (int) shared by the pipeline stages.
enum Ctr {
    cItems = 0,     // work items (K2b)
    cRecs = 1,      // records (K2b)
    cWideCount = 2, // wide particles (K1)
    cChunk = 3,     // records per item (K2b)
    cWideCursor = 4,// wide list fill (K3)
    cSlabs = 5,     // int64 partial slabs (K2b)
    cMerges = 6,    // split tiles (K2b)
    cWideMax0 = 7,  // max |c0| over wide particles, fp32 bits (K3)
    cWideMax1 = 8,  // max |c1| over wide particles, fp32 bits (K3)
    cNum = 16
};

// ----------------------------------------------------------------------------------
// K2a: per tile, exclusive prefix of hist over blocks (in place); tile totals.
// 64 tiles per workgroup (one per lane), the 4 waves split the block range.
// ----------------------------------------------------------------------------------
static __global__ __launch_bounds__(kBlock) void k_colscan(int* __restrict__ hist, int nblk, int ntiles,
                                                    int* __restrict__ tile_total) {
    __shared__ int part[4][64];
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int t = blockIdx.x * 64 + lane;
    int b0 = (int)((long long)nblk * w / 4), b1 = (int)((long long)nblk * (w + 1) / 4);
    int s = 0;
    if (t < ntiles) {
        int b = b0;
        for (; b + 8 <= b1; b += 8) {
            int c[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = hist[(long long)(b + k) * ntiles + t];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                hist[(long long)(b + k) * ntiles + t] = s;
                s += c[k];
            }
        }
        for (; b < b1; ++b) {
            int c = hist[(long long)b * ntiles + t];
            hist[(long long)b * ntiles + t] = s;
            s += c;
        }
    }
    part[w][lane] = s;
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += part[k][lane];
    if (t < ntiles) {
        if (off)
            for (int b = b0; b < b1; ++b) hist[(long long)b * ntiles + t] += off;
        if (w == 3) tile_total[t] = off + s;
    }
}

// ----------------------------------------------------------------------------------
// K2b: single workgroup.  Tile start offsets in Morton order of the tiles (spatially
// adjacent tiles' records are adjacent in HBM), the deposit work list (also Morton
// order: every tile gets >= 1 item, empty tiles a zero item) and the merge list.
// ----------------------------------------------------------------------------------
constexpr int kScanThreads = 1024;
constexpr int kTargetItems = 2048;
constexpr int kMinItemRecords = 2048;

static __device__ __forceinline__ void block_scan_ll(long long* s, int tid) {
    for (int o = 1; o < kScanThreads; o <<= 1) {
        long long x = tid >= o ? s[tid - o] : 0;
        __syncthreads();
        s[tid] += x;
        __syncthreads();
    }
}

static __global__ __launch_bounds__(kScanThreads) void k_tilescan(const int* __restrict__ tile_total,
                                                           const int* __restrict__ morton,
                                                           int ntiles,
                                                           long long* __restrict__ tile_start,
                                                           Item* __restrict__ items,
                                                           Merge* __restrict__ merges,
                                                           int* __restrict__ ctr) {
    __shared__ long long s_rec[kScanThreads], s_item[kScanThreads], s_slab[kScanThreads],
        s_merge[kScanThreads];
    int tid = threadIdx.x;
    int per = (ntiles + kScanThreads - 1) / kScanThreads;
    int r0 = min(ntiles, tid * per), r1 = min(ntiles, r0 + per);
    long long loc = 0;
    for (int r = r0; r < r1; ++r) loc += tile_total[morton[r]];
    s_rec[tid] = loc;
    __syncthreads();
    block_scan_ll(s_rec, tid);
    long long total = s_rec[kScanThreads - 1];
    long long base = s_rec[tid] - loc;
    int ch = (int)max((long long)kMinItemRecords, (total + kTargetItems - 1) / kTargetItems);
    long long nit = 0, nsl = 0, nmg = 0;
    for (int r = r0; r < r1; ++r) {
        int t = morton[r];
        int c = tile_total[t];
        tile_start[t] = base;
        base += c;
        int k = c > 0 ? (c + ch - 1) / ch : 1;
        nit += k;
        if (k > 1) {
            nsl += k;
            nmg += 1;
        }
    }
    s_item[tid] = nit;
    s_slab[tid] = nsl;
    s_merge[tid] = nmg;
    __syncthreads();
    block_scan_ll(s_item, tid);
    block_scan_ll(s_slab, tid);
    block_scan_ll(s_merge, tid);
    long long ib = s_item[tid] - nit, sb = s_slab[tid] - nsl, mb = s_merge[tid] - nmg;
    for (int r = r0; r < r1; ++r) {
        int t = morton[r];
        int c = tile_total[t];
        int k = c > 0 ? (c + ch - 1) / ch : 1;
        long long s0 = tile_start[t];
        for (int j = 0; j < k; ++j) {
            Item it;
            it.start = s0 + (long long)j * ch;
            it.tile = t;
            it.count = c > 0 ? min(ch, c - j * ch) : 0;
            it.slab = k > 1 ? (int)(sb + j) : -1;
            it.pad = 0;
            items[ib + j] = it;
        }
        ib += k;
        if (k > 1) {
            Merge m;
            m.tile = t;
            m.slab0 = (int)sb;
            m.nslab = k;
            m.pad = 0;
            merges[mb++] = m;
            sb += k;
        }
    }
    if (tid == kScanThreads - 1) {
        ctr[cItems] = (int)s_item[kScanThreads - 1];
        ctr[cRecs] = (int)min(total, (long long)0x7fffffff);
        ctr[cChunk] = ch;
        ctr[cSlabs] = (int)s_slab[kScanThreads - 1];
        ctr[cMerges] = (int)s_merge[kScanThreads - 1];
    }
}

}  // namespace asp
