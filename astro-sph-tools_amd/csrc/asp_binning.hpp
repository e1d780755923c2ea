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
    cLarge = 9,     // records in the large stream (K2b)
    cNum = 16
};

// ----------------------------------------------------------------------------------
// K2a: per tile, exclusive prefix of hist over blocks (in place); tile totals.
// 64 tiles per workgroup (one per lane), the kColscanWaves waves split the block range
// (a latency-bound walk down 64 columns of hist: more waves, shorter walks).  Blocks come
// in chunks of cb (blockIdx.y = chunk): the prefix restarts at every chunk and chunk c's
// totals go to tile_total[c * ntiles + t] (one chunk: cb >= nblk, gridDim.y = 1).
// ----------------------------------------------------------------------------------
constexpr int kColscanWaves = 16;
constexpr int kColscanBlock = 64 * kColscanWaves;
constexpr int kColscanRows = 64;  // rows per wave held in registers (1024 blocks / 16 waves)
static __global__ __launch_bounds__(kColscanBlock) void k_colscan(int* __restrict__ hist, int nblk,
                                                           int ntiles,
                                                           int* __restrict__ tile_total, int cb) {
    __shared__ int part[kColscanWaves][64];
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int t = blockIdx.x * 64 + lane;
    int c0 = (int)min((long long)nblk, (long long)blockIdx.y * cb);
    int cn = min(nblk - c0, cb);
    tile_total += (long long)blockIdx.y * ntiles;
    int b0 = c0 + (int)((long long)cn * w / kColscanWaves);
    int b1 = c0 + (int)((long long)cn * (w + 1) / kColscanWaves);
    int s = 0;
    // <= kColscanRows rows per wave (nblk <= 1024): one load of every row into registers,
    // the exclusive prefix there, one store with the other waves' offset added
    const bool regs = b1 - b0 <= kColscanRows;
    int c[kColscanRows];
    if (t < ntiles) {
        if (regs) {
#pragma unroll
            for (int k = 0; k < kColscanRows; ++k)
                c[k] = b0 + k < b1 ? hist[(long long)(b0 + k) * ntiles + t] : 0;
#pragma unroll
            for (int k = 0; k < kColscanRows; ++k) {
                int x = c[k];
                c[k] = s;
                s += x;
            }
        } else {
            int b = b0;
            for (; b + 8 <= b1; b += 8) {
                int cc[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) cc[k] = hist[(long long)(b + k) * ntiles + t];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    hist[(long long)(b + k) * ntiles + t] = s;
                    s += cc[k];
                }
            }
            for (; b < b1; ++b) {
                int cc = hist[(long long)b * ntiles + t];
                hist[(long long)b * ntiles + t] = s;
                s += cc;
            }
        }
    }
    part[w][lane] = s;
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += part[k][lane];
    if (t < ntiles) {
        if (regs) {
#pragma unroll
            for (int k = 0; k < kColscanRows; ++k)
                if (b0 + k < b1) hist[(long long)(b0 + k) * ntiles + t] = c[k] + off;
        } else if (off) {
            for (int b = b0; b < b1; ++b) hist[(long long)b * ntiles + t] += off;
        }
        if (w == kColscanWaves - 1) tile_total[t] = off + s;
    }
}

// ----------------------------------------------------------------------------------
// K2b: single workgroup.  Tile start offsets in Morton order of the tiles (spatially
// adjacent tiles' records are adjacent in HBM), the deposit work list (also Morton
// order: every tile gets >= 1 item, empty tiles a zero item) and the merge list.
//
// nstream = 2 (2-D map): column t + ntiles of tile_total holds tile t's LARGE records
// (clipped box >= gather_min pixels on both axes), stored right after its small/mid-size
// run and handed out in items of their own (Item::mode = 1, the gathered deposit K4g),
// chunked independently: each stream aims at its own item count.
// ----------------------------------------------------------------------------------
constexpr int kScanThreads = 1024;
// Regular items per call (split granularity of the small/mid stream): the 2-D map's tiles
// (kTargetItems2d; the cube sets its own, 1024, asp_project3d.hip).  2-D, same-box A/B
// (profiles/r03/items/): 1024 / 2048 / 4096 items give the 10^8 map 3.229-3.234 /
// 3.234-3.236 / 3.269-3.276 ms and the 1.25e7 shard (the N = 8 rank) 0.517 / 0.537 /
// 0.601 ms -- fewer, longer items cost the shard less merge and tilescan work.
#ifndef ASP_TARGET_ITEMS
#define ASP_TARGET_ITEMS 1024
#endif
constexpr int kTargetItems2d = ASP_TARGET_ITEMS;
constexpr int kMinItemRecords = 2048;
constexpr int kTargetItems1 = 4096;    // mode-1 items (a record there costs ~10-1000x)
constexpr int kMinItemRecords1 = 256;

// Inclusive scan of s[0 .. kScanThreads) in place: wave scans (DPP/permute shuffles), one
// wave scans the 16 wave totals; three block barriers instead of 2 log2(1024).
static __device__ __forceinline__ void block_scan_ll(long long* s, int tid) {
    __shared__ long long part[kScanThreads / 64];
    const int lane = tid & 63, w = tid >> 6;
    long long x = s[tid];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        long long y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    if (w == 0) {
        long long q = lane < kScanThreads / 64 ? part[lane] : 0;
#pragma unroll
        for (int o = 1; o < kScanThreads / 64; o <<= 1) {
            long long y = __shfl_up(q, o);
            if (lane >= o) q += y;
        }
        if (lane < kScanThreads / 64) part[lane] = q;
    }
    __syncthreads();
    if (w > 0) x += part[w - 1];
    s[tid] = x;
    __syncthreads();
}

// Exclusive scan of M values per thread over the block in one pass (shared barriers): x[m]
// becomes the sum over lower threads, tot[m] the block total.
template <int M>
static __device__ __forceinline__ void block_scan_multi(long long (&x)[M], long long (&tot)[M],
                                                        int tid) {
    __shared__ long long part[M][kScanThreads / 64];
    const int lane = tid & 63, w = tid >> 6;
    long long inc[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        inc[m] = x[m];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            long long y = __shfl_up(inc[m], o);
            if (lane >= o) inc[m] += y;
        }
        if (lane == 63) part[m][w] = inc[m];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            long long q = lane < kScanThreads / 64 ? part[m][lane] : 0;
#pragma unroll
            for (int o = 1; o < kScanThreads / 64; o <<= 1) {
                long long y = __shfl_up(q, o);
                if (lane >= o) q += y;
            }
            if (lane < kScanThreads / 64) part[m][lane] = q;
        }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < M; ++m) {
        tot[m] = part[m][kScanThreads / 64 - 1];
        x[m] = (w > 0 ? part[m][w - 1] : 0) + inc[m] - x[m];
    }
    __syncthreads();  // part is rewritten by the next scan
}

// items of one tile: regular ones of ch records, large ones of chl records
static __device__ __forceinline__ void tile_items(int cs, int cl, int ch, int chl, int& ks,
                                                  int& kl) {
    ks = cs > 0 ? (cs + ch - 1) / ch : 0;
    kl = cl > 0 ? (cl + chl - 1) / chl : 0;
    if (ks + kl == 0) ks = 1;  // empty tile: one zero item writes the zeros
}

constexpr int kScanPer = 16;  // max tiles per scan thread held in registers (<= 16384 tiles)

constexpr int kOrderBuckets = 33;  // log2 classes of counts < 2^31, plus empty items

// PART 0: everything; 1: the tile starts and the record counters only (what the scatter
// needs); 2: the rest (work items, merge list, dispatch order and their counters: what the
// deposit needs) -- the 2-D map runs part 2 on its side stream beside the scatter (round 6)
template <int PER, int PART = 0>  // tiles per thread held in registers: ntiles <= PER * kScanThreads
static __global__ __launch_bounds__(kScanThreads) void k_tilescan(
    const int* __restrict__ tile_total, const int* __restrict__ morton, int ntiles, int nstream,
    long long* __restrict__ tile_start, Item* __restrict__ items, Merge* __restrict__ merges,
    int* __restrict__ ctr, int* __restrict__ order, int identity, int target) {
    __shared__ int ocnt[kOrderBuckets];
    int tid = threadIdx.x;
    if (tid < kOrderBuckets) ocnt[tid] = 0;
    int per = (ntiles + kScanThreads - 1) / kScanThreads;  // <= kScanPer (host-checked)
    int r0 = min(ntiles, tid * per), r1 = min(ntiles, r0 + per);
    // this thread's tiles, their small- and large-record counts: all loads issued up front
    // (two dependent rounds: morton, then the totals) and kept in registers
    int tt[PER], cs_[PER], cl_[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) tt[q] = r0 + q < r1 ? morton[r0 + q] : 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        bool in = r0 + q < r1;
        cs_[q] = in ? tile_total[tt[q]] : 0;
        cl_[q] = in && nstream == 2 ? tile_total[tt[q] + ntiles] : 0;
    }
    auto span = [](int cs, int cl) { return (long long)(cs + cl); };  // a tile's run
    long long sa[2] = {0, 0}, ta[2];  // all records; stream-1 records
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        sa[0] += span(cs_[q], cl_[q]);
        sa[1] += cl_[q];
    }
    block_scan_multi<2>(sa, ta, tid);
    const long long total = ta[0], total1 = ta[1];
    const long long base0 = sa[0];
    if (PART == 1) {
        long long b = base0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (r0 + q >= r1) continue;
            tile_start[tt[q]] = b;
            if (nstream == 2) tile_start[tt[q] + ntiles] = b + cs_[q];
            b += span(cs_[q], cl_[q]);
        }
        if (tid == kScanThreads - 1) {
            ctr[cRecs] = (int)min(total, (long long)0x7fffffff);
            ctr[cLarge] = (int)min(total1, (long long)0x7fffffff);
        }
        return;
    }
    int ch = (int)max((long long)kMinItemRecords,
                      (total - total1 + target - 1) / target);
    int chl = (int)max((long long)kMinItemRecords1, (total1 + kTargetItems1 - 1) / kTargetItems1);
    long long sb3[3] = {0, 0, 0}, tb[3];  // items, slabs, merges of this thread's tiles
    long long base = base0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (r0 + q >= r1) continue;
        int t = tt[q], cs = cs_[q], cl = cl_[q];
        if (PART == 0) {
            tile_start[t] = base;
            if (nstream == 2) tile_start[t + ntiles] = base + cs;
        }
        base += span(cs, cl);
        int ks, kl;
        tile_items(cs, cl, ch, chl, ks, kl);
        sb3[0] += ks + kl;
        if (ks + kl > 1) {
            sb3[1] += ks + kl;
            sb3[2] += 1;
        }
    }
    block_scan_multi<3>(sb3, tb, tid);
    // this thread's items in order: f(item index, item)
    auto for_items = [&](auto&& f) {
        long long ib = sb3[0], sb = sb3[1];
        long long b = base0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (r0 + q >= r1) continue;
            int t = tt[q], cs = cs_[q], cl = cl_[q];
            int ks, kl;
            tile_items(cs, cl, ch, chl, ks, kl);
            int k = ks + kl;
            long long s0 = b;
            b += span(cs, cl);
            for (int j = 0; j < k; ++j) {
                Item it;
                bool lg = j >= ks;
                int jj = lg ? j - ks : j;
                int c = lg ? cl : cs, chunk = lg ? chl : ch;
                it.start = (lg ? s0 + cs : s0) + (long long)jj * chunk;
                it.tile = t;
                it.count = c > 0 ? min(chunk, c - jj * chunk) : 0;
                it.slab = k > 1 ? (int)(sb + j) : -1;
                it.mode = lg ? 1 : 0;
                f(ib + j, it);
            }
            ib += k;
            if (k > 1) sb += k;
        }
    };
    for_items([&](long long i, const Item& it) { items[i] = it; });
    {  // the merge list
        long long mb = sb3[2], sb = sb3[1];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (r0 + q >= r1) continue;
            int ks, kl;
            tile_items(cs_[q], cl_[q], ch, chl, ks, kl);
            int k = ks + kl;
            if (k > 1) {
                Merge m;
                m.tile = tt[q];
                m.slab0 = (int)sb;
                m.nslab = k;
                m.pad = 0;
                merges[mb++] = m;
                sb += k;
            }
        }
    }
    // K2c, dispatch order of the deposit work items -- largest first (longest-processing-
    // time scheduling: the items of the dense central tiles used to start late in Morton
    // order and finish last): items bucketed by floor(log2(count)), buckets in decreasing
    // size, order within a bucket unspecified.  order[b] = the item workgroup b takes.
    // (Was a kernel of its own on the critical path before the deposit.)
    if (order) {
        auto bucket = [](int c) { return c <= 0 ? kOrderBuckets - 1 : __builtin_clz((unsigned)c) - 1; };
        if (identity) {  // A/B switch (ASP_ITEM_ORDER=0): Morton order as produced
            for_items([&](long long i, const Item&) { order[i] = (int)i; });
        } else {
            for_items([&](long long, const Item& it) { atomicAdd(&ocnt[bucket(it.count)], 1); });
            __syncthreads();
            if (tid == 0) {
                int s = 0;
                for (int b = 0; b < kOrderBuckets; ++b) {
                    const int c = ocnt[b];
                    ocnt[b] = s;
                    s += c;
                }
            }
            __syncthreads();
            for_items([&](long long i, const Item& it) {
                order[atomicAdd(&ocnt[bucket(it.count)], 1)] = (int)i;
            });
        }
    }
    if (tid == kScanThreads - 1) {
        ctr[cItems] = (int)tb[0];
        ctr[cChunk] = ch;
        ctr[cSlabs] = (int)tb[1];
        ctr[cMerges] = (int)tb[2];
        if (PART == 0) {
            ctr[cRecs] = (int)min(total, (long long)0x7fffffff);
            ctr[cLarge] = (int)min(total1, (long long)0x7fffffff);
        }
    }
}

}  // namespace asp
