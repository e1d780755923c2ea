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

static int run(bool skew);
int main() {
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
    if (hipMalloc(&d, (size_t)(sP + 16) * 32) != hipSuccess) return 1;
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
    if (ldsM > 163840 || hipFuncSetAttribute((const void*)kM, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)ldsM) != hipSuccess) {
        printf("cannot set LDS size %zu\n", ldsM);
        return 4;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("records %lld, padded %lld (holes %.2f %%)\n", sA, sP, 100.0 * (sP - sA) / sA);
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 3; ++mode) {
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(kA, dim3(B), dim3(T), 0, 0, d, per_wg, dA);
            else if (mode == 1) hipLaunchKernelGGL(kP<0>, dim3(B), dim3(T), ldsP, 0, d, per_wg, dP, dE);
            else hipLaunchKernelGGL(kM, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            hipError_t err = hipGetLastError();
            printf("rep %d  %-28s %7.3f ms %s\n", rep,
                   mode == 0 ? "A 32-B records (paired lanes)" : mode == 1 ? "P 64-B pairs, sub-rounds" : "M 64-B pairs, mailbox",
                   ms, err == hipSuccess ? "" : hipGetErrorString(err));
        }
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
    hipLaunchKernelGGL(kM, dim3(B), dim3(T), ldsM, 0, d, per_wg, dP, dE);
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
    hipFree(d);
    hipFree(dA);
    hipFree(dP);
    hipFree(dE);
    if (dtab) hipFree(dtab);
    return 0;
}
