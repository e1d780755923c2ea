// Microbenchmark: does writing the scatter's records as 64-B PAIRS (two consecutive
// records of a (workgroup, tile) run, one 64-B-aligned write location) instead of single
// 32-B records halve the scatter's store cost?  1e8 records, 4096 tiles (uniform), 256
// workgroups x 512 threads, 1024 records per batch (2 per lane) -- k_scatter's shape.
//   A: k_scatter today: slot = LDS atomic on the run cursor, lanes 2j / 2j + 1 write the
//      two 16-B halves of record j (one store instruction covers 32 records);
//   P: pairs: runs padded to even length; per batch the records of a tile are ranked
//      (LDS counter), processed in rank order (sub-rounds): an even slot parks its record
//      in the tile's LDS slot (4096 x 32 B = 128 KiB), the odd slot writes both (64 B);
//      leftovers flushed with a hole record at the end.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_pairs tools/microbench/pairs.hip && /tmp/mb_pairs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <utility>
#include <vector>

constexpr int T = 512;           // threads per workgroup
constexpr int U = 2;             // records per lane per batch
constexpr int NT = 4096;         // tiles
constexpr int B = 256;           // workgroups
constexpr int TABN = 1 << 22;    // skewed mode: tile ids drawn from a Plummer-like table
__device__ const int* g_tab = nullptr;
__device__ unsigned long long g_tries = 0;  // exchange attempts (contention probe)
__device__ __forceinline__ int tile_of(unsigned hsh) {
    return g_tab ? g_tab[hsh & (TABN - 1)] : (int)(hsh & (NT - 1));
}

__device__ __host__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(T) void kA(float4* __restrict__ out, long long per_wg,
                                        const long long* __restrict__ base) {
    __shared__ int cur[NT];
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    for (int t = threadIdx.x; t < NT; t += T) cur[t] = (int)base[(long long)t * B + b];
    __syncthreads();
    for (long long j0 = 0; j0 < per_wg; j0 += T * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long long j = j0 + threadIdx.x * U + u;
            int t = tile_of(hash32((unsigned)(b * per_wg + j)));
            int slot = j < per_wg ? atomicAdd(&cur[t], 1) : -1;
            float4 v0 = make_float4((float)j, (float)t, 1.f, 2.f);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                int src = half * 32 + (lane >> 1);
                int s = __shfl(slot, src);
                float4 val = (lane & 1) ? make_float4(3.f, 0.f, 0.f, 0.f)
                                        : make_float4(__shfl(v0.x, src), __shfl(v0.y, src), 1.f, 2.f);
                if (s >= 0) out[2 * (long long)s + (lane & 1)] = val;
            }
        }
    }
}

template <int TWO_LANES>
__global__ __launch_bounds__(T) void kP(float4* __restrict__ out, long long per_wg,
                                        const long long* __restrict__ base,
                                        const long long* __restrict__ endp) {
    extern __shared__ __attribute__((aligned(16))) float4 pend[];  // 2 per tile (32 B)
    int* cur = (int*)(pend + 2 * NT);
    unsigned* bc = (unsigned*)(cur + NT);  // per-batch rank counters, two 16-bit per word
    int& maxq = *(int*)(bc + NT / 2);
    const int b = blockIdx.x;
    for (int t = threadIdx.x; t < NT; t += T) {
        cur[t] = (int)base[(long long)t * B + b];
        if (t < NT / 2) bc[t] = 0u;
    }
    if (threadIdx.x == 0) maxq = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (long long j0 = 0; j0 < per_wg; j0 += T * U) {
        int tt[U], q[U];
        float4 r0[U], r1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long long j = j0 + threadIdx.x * U + u;
            tt[u] = tile_of(hash32((unsigned)(b * per_wg + j)));
            q[u] = -1;
            r0[u] = make_float4((float)j, (float)tt[u], 1.f, 2.f);
            r1[u] = make_float4(3.f, 0.f, 0.f, 0.f);
            if (j < per_wg) {
                const int sh = 16 * (tt[u] & 1);
                q[u] = (int)((atomicAdd(&bc[tt[u] >> 1], 1u << sh) >> sh) & 0xffffu);
                if (q[u] > 0) atomicMax(&maxq, q[u]);
            }
        }
        __syncthreads();
        int slot[U];
#pragma unroll
        for (int u = 0; u < U; ++u) slot[u] = q[u] >= 0 ? cur[tt[u]] + q[u] : -1;
        const int mq = maxq;
        __syncthreads();  // every lane has read cur / bc / maxq
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q[u] == 0) {
                const int sh = 16 * (tt[u] & 1);
                cur[tt[u]] += (int)((bc[tt[u] >> 1] >> sh) & 0xffffu);
            }
        __syncthreads();  // every tile's count read before the words are cleared
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q[u] == 0) bc[tt[u] >> 1] = 0u;
        if (threadIdx.x == 0) maxq = 0;
        for (int r = 0; r <= mq; ++r) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool act = q[u] == r;
                if (act && !(slot[u] & 1)) {  // first of its pair: park it
                    pend[2 * tt[u]] = r0[u];
                    pend[2 * tt[u] + 1] = r1[u];
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool act = q[u] == r && (slot[u] & 1);
                if constexpr (TWO_LANES == 0) {
                    if (act) {  // second: write the pair (64 B, one lane)
                        float4* d = out + 2 * (long long)(slot[u] - 1);
                        d[0] = pend[2 * tt[u]];
                        d[1] = pend[2 * tt[u] + 1];
                        d[2] = r0[u];
                        d[3] = r1[u];
                    }
                }
            }
            __syncthreads();
        }
    }
    // flush: a run left with an odd count ends in a parked record + a hole
    for (int t = threadIdx.x; t < NT; t += T) {
        const int c = cur[t];
        if ((long long)c < endp[(long long)t * B + b] && (c & 1)) {
            float4* d = out + 2 * (long long)(c - 1);
            d[0] = pend[2 * t];
            d[1] = pend[2 * t + 1];
            d[2] = make_float4(0.f, 0.f, 0.f, 0.f);
            d[3] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    (void)lane;
}

// M: the lock-free mailbox handoff (k_scatter_pair's protocol): one 64-bit LDS word per
// tile {run cursor, state}; state -1 empty, -2 busy, >= 0 parked (index into the park
// slot).  One exchange decides: empty -> park, parked -> take and write the pair at the
// cursor, busy -> retry.  No barriers.
template <int PROBE>
__global__ __launch_bounds__(T) void kM(float4* __restrict__ out, long long per_wg,
                                        const long long* __restrict__ base,
                                        const long long* __restrict__ endp) {
    extern __shared__ __attribute__((aligned(16))) float4 pend[];  // 2 per tile (32 B)
    unsigned long long* wd = (unsigned long long*)(pend + 2 * NT);  // {cursor << 32 | state}
    const int b = blockIdx.x;
    for (int t = threadIdx.x; t < NT; t += T)
        wd[t] = ((unsigned long long)(unsigned)base[(long long)t * B + b] << 32) | 0xffffffffull;
    __syncthreads();
    constexpr unsigned long long kBusy = 0xfffffffeull;
    for (long long j0 = 0; j0 < per_wg; j0 += T * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long long j = j0 + threadIdx.x * U + u;
            const bool live = j < per_wg;
            int t = tile_of(hash32((unsigned)(b * per_wg + j)));
            float4 r0 = make_float4((float)j, (float)t, 1.f, 2.f), r1 = make_float4(3.f, 0.f, 0.f, 0.f);
            bool done = !live;
            do {
                if (!done) {
                    const unsigned long long x = atomicExch(&wd[t], kBusy);
                    if (PROBE) atomicAdd(&g_tries, 1ull);
                    const unsigned st = (unsigned)x;
                    const unsigned cur = (unsigned)(x >> 32);
                    if (st == 0xffffffffu) {  // empty: park
                        pend[2 * t] = r0;
                        pend[2 * t + 1] = r1;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __hip_atomic_store(&wd[t], ((unsigned long long)cur << 32) | 0u,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        done = true;
                    } else if (st != 0xfffffffeu) {  // parked: take, write the pair
                        const float4 f0 = pend[2 * t], f1 = pend[2 * t + 1];
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __hip_atomic_store(&wd[t], ((unsigned long long)(cur + 2) << 32) | 0xffffffffull,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        float4* d = out + 2 * (long long)cur;
                        d[0] = f0;
                        d[1] = f1;
                        d[2] = r0;
                        d[3] = r1;
                        done = true;
                    }  // busy: the exchange left it busy; retry
                }
            } while (__ballot(!done) != 0ull);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < NT; t += T) {
        const unsigned long long x = wd[t];
        if ((unsigned)x == 0u) {
            float4* d = out + 2 * (long long)(x >> 32);
            d[0] = pend[2 * t];
            d[1] = pend[2 * t + 1];
            d[2] = make_float4(0.f, 0.f, 0.f, 0.f);
            d[3] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}


// S: the mailbox with the wave's records SORTED by tile first (64-lane bitonic sort of
// (tile, lane) keys): every tile then appears in one run of consecutive lanes, whose leader
// alone exchanges the tile's word -- no two lanes of a wave collide on a word (the mailbox's
// retries under Plummer skew).  The run's records pair up in order after a parked partner;
// an odd one out parks.  Slots and actions are pushed back to the records' own lanes
// (ds_permute).
__device__ __forceinline__ unsigned wave_sort64(unsigned key, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const unsigned o = (unsigned)__shfl_xor((int)key, j);
            const bool up = (lane & k) == 0, lower = (lane & j) == 0;
            key = (lower == up) ? min(key, o) : max(key, o);
        }
    return key;
}
__device__ __forceinline__ int push(int to_lane, int v) {
    return __builtin_amdgcn_ds_permute(to_lane * 4, v);
}
template <int PROBE>
__global__ __launch_bounds__(T) void kS(float4* __restrict__ out, long long per_wg,
                                        const long long* __restrict__ base,
                                        const long long* __restrict__ endp) {
    extern __shared__ __attribute__((aligned(16))) float4 pend[];  // 2 per tile (32 B)
    unsigned long long* wd = (unsigned long long*)(pend + 2 * NT);  // {cursor << 32 | state}
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63;
    for (int t = threadIdx.x; t < NT; t += T)
        wd[t] = ((unsigned long long)(unsigned)base[(long long)t * B + b] << 32) | 0xffffffffull;
    __syncthreads();
    constexpr unsigned long long kBusy = 0xfffffffeull;
    constexpr unsigned kNone = 0x3ffffffu;
    for (long long j0 = 0; j0 < per_wg; j0 += T * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long j = j0 + threadIdx.x * U + u;
            const bool live = j < per_wg;
            const int tm = tile_of(hash32((unsigned)(b * per_wg + j)));
            const float4 r0 = make_float4((float)j, (float)tm, 1.f, 2.f), r1 = make_float4(3.f, 0.f, 0.f, 0.f);
            // sorted order: lane l holds the l-th smallest (tile, lane)
            const unsigned key = wave_sort64(((live ? (unsigned)tm : kNone) << 6) | (unsigned)lane, lane);
            const unsigned t = key >> 6;
            const int src = (int)(key & 63u);
            const bool valid = t != kNone;
            const unsigned tprev = (unsigned)__shfl_up((int)t, 1);
            const bool start = lane == 0 || t != tprev;
            const unsigned long long S = __ballot(start);
            const unsigned long long below = S & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
            const int seg0 = 63 - __clzll(below);
            const unsigned long long above = S & ~(lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
            const int seg1 = above ? __ffsll((long long)above) - 1 : 64;
            const int r = lane - seg0, m = seg1 - seg0;
            // the leader exchanges the tile's word; a segment whose word was busy (another
            // wave mid-hand-off) retries.  Every hand-off completes inside the iteration that
            // won the word (no lane holds a word across iterations: no deadlock).
            bool pending = valid && r == 0;
            int slot = -1, rdp = 0, phi = 0;
            float4 f0 = make_float4(0.f, 0.f, 0.f, 0.f), f1 = f0;
            do {
                unsigned long long x = 0;
                bool got = false;
                if (pending) {
                    x = atomicExch(&wd[t], kBusy);
                    if (PROBE) atomicAdd(&g_tries, 1ull);
                    got = (unsigned)x != 0xfffffffeu;
                }
                const bool sg = __shfl((int)got, seg0) != 0;
                const unsigned lo = (unsigned)__shfl((int)(unsigned)x, seg0);
                const unsigned hi = (unsigned)__shfl((int)(unsigned)(x >> 32), seg0);
                const int parked = lo != 0xffffffffu;
                const int c = m + parked, npi = c & ~1;
                const int pos = r + parked;
                const bool act = valid && sg;
                int s_slot = act && pos < npi ? (int)hi + pos : -1;
                int s_rdp = act && r == 0 && parked;
                int s_park = act && (c & 1) && pos == c - 1;
                // back to the records' own lanes
                s_slot = push(src, s_slot);
                s_rdp = push(src, s_rdp);
                s_park = push(src, s_park);
                const int tt = push(src, (int)t);
                const int s_hi = push(src, (int)hi);
                if (s_rdp) {
                    f0 = pend[2 * tt];
                    f1 = pend[2 * tt + 1];
                    rdp = 1;
                    phi = s_hi;
                }
                asm volatile("" ::: "memory");
                if (s_park) {
                    pend[2 * tt] = r0;
                    pend[2 * tt + 1] = r1;
                }
                asm volatile("" ::: "memory");
                if (got)
                    __hip_atomic_store(&wd[t], ((unsigned long long)(hi + npi) << 32) |
                                                   ((c & 1) ? 0ull : 0xffffffffull),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (s_slot >= 0) slot = s_slot;
                pending = pending && !got;
            } while (__ballot(pending) != 0ull);
            if (rdp) {
                float4* d = out + 2 * (long long)phi;
                d[0] = f0;
                d[1] = f1;
            }
            if (slot >= 0) {
                float4* d = out + 2 * (long long)slot;
                d[0] = r0;
                d[1] = r1;
            }
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < NT; t += T) {
        const unsigned long long x = wd[t];
        if ((unsigned)x == 0u) {
            float4* d = out + 2 * (long long)(x >> 32);
            d[0] = pend[2 * t];
            d[1] = pend[2 * t + 1];
            d[2] = make_float4(0.f, 0.f, 0.f, 0.f);
            d[3] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

static int run(bool skew);
// The record buffer: kept across runs unless ASP_MB_REALLOC (placement: DESIGN.md §4)
static float4* g_buf = nullptr;
int main() {
    // same buffer: uniform, skewed, uniform, skewed; then a fresh buffer: uniform, skewed
    for (int pass = 0; pass < 3; ++pass) {
        if (pass == 2 && g_buf) { hipFree(g_buf); g_buf = nullptr; printf("== fresh buffer\n"); }
        int rc = run(false);
        if (rc) return rc;
        rc = run(true);
        if (rc) return rc;
    }
    return 0;
}
static int unused_main() {
    int rc = run(false);
    if (rc) return rc;
    return run(true);
}

static int run(bool skew) {
    const long long N = 100000000LL;
    const long long per_wg = N / B;
    // skewed: 64 x 64 tiles over [-4, 4]^2, Plummer surface density (1 + R^2)^-2
    std::vector<int> tab(TABN);
    {
        std::vector<double> w(NT), cdf(NT);
        double sum = 0;
        for (int t = 0; t < NT; ++t) {
            double x = -4 + 8.0 * ((t / 64) + 0.5) / 64, y = -4 + 8.0 * ((t % 64) + 0.5) / 64;
            double r2 = x * x + y * y;
            w[t] = 1.0 / ((1 + r2) * (1 + r2));
            sum += w[t];
            cdf[t] = sum;
        }
        int t = 0;
        for (int i = 0; i < TABN; ++i) {
            double q = (i + 0.5) / TABN * sum;
            while (cdf[t] < q) ++t;
            tab[i] = t;
        }
        // shuffle so the low hash bits pick random table entries
        for (int i = TABN - 1; i > 0; --i) std::swap(tab[i], tab[hash32((unsigned)i) % (unsigned)(i + 1)]);
    }
    int* dtab = nullptr;
    if (skew) {
        hipMalloc(&dtab, TABN * sizeof(int));
        hipMemcpy(dtab, tab.data(), TABN * sizeof(int), hipMemcpyHostToDevice);
    }
    hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &dtab, sizeof(dtab));
    auto tile_h = [&](unsigned hsh) { return skew ? tab[hsh & (TABN - 1)] : (int)(hsh & (NT - 1)); };
    printf("== %s tiles\n", skew ? "Plummer-skewed" : "uniform");
    std::vector<long long> cnt((size_t)NT * B, 0);
    for (int b = 0; b < B; ++b)
        for (long long j = 0; j < per_wg; ++j)
            cnt[(size_t)tile_h(hash32((unsigned)(b * per_wg + j))) * B + b]++;
    std::vector<long long> baseA(cnt.size()), baseP(cnt.size()), endP(cnt.size());
    long long sA = 0, sP = 0;
    for (size_t i = 0; i < cnt.size(); ++i) {
        baseA[i] = sA;
        sA += cnt[i];
        baseP[i] = sP;
        sP += (cnt[i] + 1) & ~1LL;  // runs padded to even: pairs are 64-B aligned
        endP[i] = sP;
    }
    float4* d;
    long long *dA, *dP, *dE;
    if (!g_buf && hipMalloc(&g_buf, (size_t)(100000000LL * 105 / 100 + 16) * 32) != hipSuccess) return 1;
    d = g_buf;
    printf("buffer %p\n", (void*)d);
    hipMalloc(&dA, cnt.size() * 8);
    hipMalloc(&dP, cnt.size() * 8);
    hipMalloc(&dE, cnt.size() * 8);
    hipMemcpy(dA, baseA.data(), cnt.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dP, baseP.data(), cnt.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dE, endP.data(), cnt.size() * 8, hipMemcpyHostToDevice);
    const size_t ldsP = (size_t)2 * NT * 16 + NT * 4 + NT * 2 + 16;  // < 160 KiB
    if (ldsP > 163840) return 2;
    if (hipFuncSetAttribute((const void*)kP<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)ldsP) != hipSuccess) {
        printf("cannot set LDS size %zu\n", ldsP);
        return 3;
    }
    const size_t ldsM = (size_t)2 * NT * 16 + NT * 8;
    hipFuncSetAttribute((const void*)kS<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsM);
    hipFuncSetAttribute((const void*)kS<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsM);
    hipFuncSetAttribute((const void*)kM<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsM);
    if (ldsM > 163840 || hipFuncSetAttribute((const void*)kM<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)ldsM) != hipSuccess) {
        printf("cannot set LDS size %zu\n", ldsM);
        return 4;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("records %lld, padded %lld (holes %.2f %%)\n", sA, sP, 100.0 * (sP - sA) / sA);
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 4; ++mode) {
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(kA, dim3(B), dim3(T), 0, 0, d, per_wg, dA);
            else if (mode == 1) hipLaunchKernelGGL(kP<0>, dim3(B), dim3(T), ldsP, 0, d, per_wg, dP, dE);
            else if (mode == 2) hipLaunchKernelGGL(kM<0>, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
            else hipLaunchKernelGGL(kS<0>, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            hipError_t err = hipGetLastError();
            printf("rep %d  %-28s %7.3f ms %s\n", rep,
                   mode == 0 ? "A 32-B records (paired lanes)" : mode == 1 ? "P 64-B pairs, sub-rounds" : mode == 2 ? "M 64-B pairs, mailbox" : "S mailbox, wave-sorted",
                   ms, err == hipSuccess ? "" : hipGetErrorString(err));
        }
    }
    for (int pm = 0; pm < 2; ++pm) {
        unsigned long long z = 0, tries = 0;
        hipMemcpyToSymbol(HIP_SYMBOL(g_tries), &z, sizeof(z));
        if (pm == 0) hipLaunchKernelGGL(kM<1>, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
        else hipLaunchKernelGGL(kS<1>, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
        hipDeviceSynchronize();
        hipMemcpyFromSymbol(&tries, HIP_SYMBOL(g_tries), sizeof(tries));
        printf("%s: %llu exchange attempts for %lld records (%.3f per record)\n", pm ? "S" : "M", tries, sA,
               (double)tries / (double)sA);
    }
    // check P's layout: every slot of every run written (j >= 0 or a hole of zeros)
    std::vector<float4> h((size_t)(sP) * 2);
    hipMemset(d, 0xff, (size_t)sP * 32);
    hipLaunchKernelGGL(kP<0>, dim3(B), dim3(T), ldsP, 0, d, per_wg, dP, dE);
    hipMemcpy(h.data(), d, (size_t)sP * 32, hipMemcpyDeviceToHost);
    long long bad = 0, holes = 0;
    for (long long s = 0; s < sP; ++s) {
        unsigned bits;
        std::memcpy(&bits, &h[2 * s].w, 4);
        if (bits == 0xffffffffu) ++bad;
        else if (h[2 * s].z == 0.f) ++holes;
    }
    printf("P layout: %lld unwritten slots, %lld holes\n", bad, holes);
    hipMemset(d, 0xff, (size_t)sP * 32);
    hipLaunchKernelGGL(kM<0>, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
    hipMemcpy(h.data(), d, (size_t)sP * 32, hipMemcpyDeviceToHost);
    bad = 0;
    long long recs = 0;
    for (long long s2 = 0; s2 < sP; ++s2) {
        unsigned bits;
        std::memcpy(&bits, &h[2 * s2].w, 4);
        if (bits == 0xffffffffu) ++bad;
        else if (h[2 * s2].z != 0.f) ++recs;
    }
    printf("M layout: %lld unwritten (the runs' padding beyond the flush), %lld records (want %lld)\n",
           bad, recs, sA);
    hipMemset(d, 0xff, (size_t)sP * 32);
    hipLaunchKernelGGL(kS<0>, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
    hipMemcpy(h.data(), d, (size_t)sP * 32, hipMemcpyDeviceToHost);
    {
        long long bad2 = 0, recs2 = 0;
        std::vector<char> seen((size_t)per_wg * B, 0);
        long long dup = 0;
        for (long long s2 = 0; s2 < sP; ++s2) {
            unsigned bits;
            std::memcpy(&bits, &h[2 * s2].w, 4);
            if (bits == 0xffffffffu) ++bad2;
            else if (h[2 * s2].z != 0.f) ++recs2;
        }
        (void)seen; (void)dup;
        printf("S layout: %lld unwritten, %lld records (want %lld)\n", bad2, recs2, sA);
    }
    hipFree(dA);
    hipFree(dP);
    hipFree(dE);
    if (dtab) hipFree(dtab);
    return 0;
}
