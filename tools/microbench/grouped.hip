// Microbenchmark for a tile-grouped binning: can the record scatter
// be made coalesced by partitioning the particles by tile group first?
//   A: read 5 fp32 arrays (1e8 particles), LDS counting sort of each 4096-particle batch by
//      tile group (16 groups of 256 tiles), reserve one range per (batch, group) with a
//      global atomic, write 24-B copies {u,v,h,a0,a1,p} group-contiguous (coalesced).
//   B: per group, workgroups read their share of the copies, LDS-sort each 2048 batch by
//      tile, reserve one range per (batch, tile), write 32-B records tile-contiguous.
// Uniform random tiles (hash of the particle index).  Times with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NT = 4096, G = 16, TPG = NT / G;
__device__ __host__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ __host__ __forceinline__ int tile_of(unsigned p) { return (int)(hash32(p) & (NT - 1)); }

constexpr int TA = 1024, BA = 4096;  // partition: threads, batch
struct __attribute__((packed)) Copy { float u, v, h, a0, a1; int p; };

__global__ __launch_bounds__(TA) void k_part(const float* __restrict__ u, const float* __restrict__ v,
                                             const float* __restrict__ h, const float* __restrict__ a0,
                                             const float* __restrict__ a1, long long n,
                                             float* __restrict__ gbuf, long long gcap,
                                             unsigned long long* __restrict__ gcur) {
    __shared__ float st[BA * 6];
    __shared__ int cnt[G], pre[G + 1];
    __shared__ long long gb[G];
    for (long long base = (long long)blockIdx.x * BA; base < n; base += (long long)gridDim.x * BA) {
        if (threadIdx.x < G) cnt[threadIdx.x] = 0;
        __syncthreads();
        int gq[4], pos[4];
        float val[4][5];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            long long i = base + k * TA + threadIdx.x;
            gq[k] = -1;
            if (i < n) {
                val[k][0] = u[i]; val[k][1] = v[i]; val[k][2] = h[i]; val[k][3] = a0[i]; val[k][4] = a1[i];
                gq[k] = tile_of((unsigned)i) / TPG;
                pos[k] = atomicAdd(&cnt[gq[k]], 1);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int s = 0;
            for (int g = 0; g < G; ++g) { pre[g] = s; s += cnt[g]; }
            pre[G] = s;
        }
        if (threadIdx.x < G) gb[threadIdx.x] = (long long)atomicAdd(&gcur[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (gq[k] < 0) continue;
            int q = pre[gq[k]] + pos[k];
            long long i = base + k * TA + threadIdx.x;
#pragma unroll
            for (int c = 0; c < 5; ++c) st[q * 6 + c] = val[k][c];
            st[q * 6 + 5] = __int_as_float((int)i);
        }
        __syncthreads();
        const int tot = pre[G];
        for (int e = threadIdx.x; e < tot * 6; e += TA) {   // word e of the sorted batch
            int q = e / 6;
            int g = 0;
            while (g + 1 < G && pre[g + 1] <= q) ++g;
            long long dst = (long long)g * gcap + gb[g] + (q - pre[g]);
            gbuf[dst * 6 + (e - q * 6)] = st[e];
        }
        __syncthreads();
    }
}

constexpr int TB = 1024, BB = 2048;  // scatter: threads, batch
__global__ __launch_bounds__(TB) void k_scat(const float* __restrict__ gbuf, long long gcap,
                                             const unsigned long long* __restrict__ gcnt, int wpg,
                                             float4* __restrict__ recs, int* __restrict__ tcur) {
    __shared__ float4 st[BB * 2];
    __shared__ int cnt[TPG], pre[TPG + 1], tb[TPG];
    const int g = blockIdx.x % G, w = blockIdx.x / G;
    const long long ng = (long long)gcnt[g];
    const long long lo = ng * w / wpg, hi = ng * (w + 1) / wpg;
    const float* src = gbuf + (long long)g * gcap * 6;
    for (long long base = lo; base < hi; base += BB) {
        for (int t = threadIdx.x; t < TPG; t += TB) cnt[t] = 0;
        __syncthreads();
        int lt[2], pos[2];
        float4 r0[2], r1[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            long long i = base + k * TB + threadIdx.x;
            lt[k] = -1;
            if (i < hi) {
                const float* c = src + i * 6;
                int p = __float_as_int(c[5]);
                r0[k] = make_float4(c[0], c[1], c[2], c[3]);
                r1[k] = make_float4(c[4], __int_as_float(p), 0.f, 0.f);
                lt[k] = tile_of((unsigned)p) - g * TPG;
                pos[k] = atomicAdd(&cnt[lt[k]], 1);
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {  // wave prefix over 256 counts
            int s = 0;
            for (int t = threadIdx.x * 4; t < threadIdx.x * 4 + 4; ++t) s += cnt[t];
            int incl = s;
            for (int d = 1; d < 64; d <<= 1) { int y = __shfl_up(incl, d); if ((int)threadIdx.x >= d) incl += y; }
            int run = incl - s;
            for (int t = threadIdx.x * 4; t < threadIdx.x * 4 + 4; ++t) { pre[t] = run; run += cnt[t]; }
            if (threadIdx.x == 63) pre[TPG] = incl;
        }
        for (int t = threadIdx.x; t < TPG; t += TB)
            if (cnt[t]) tb[t] = atomicAdd(&tcur[g * TPG + t], cnt[t]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (lt[k] < 0) continue;
            int q = pre[lt[k]] + pos[k];
            st[2 * q] = r0[k];
            st[2 * q + 1] = r1[k];
        }
        __syncthreads();
        const int tot = pre[TPG];
        for (int e = threadIdx.x; e < tot * 2; e += TB) {
            int q = e >> 1;
            int lo2 = 0, hi2 = TPG;  // tile of sorted record q: largest t with pre[t] <= q
            while (hi2 - lo2 > 1) { int m = (lo2 + hi2) >> 1; if (pre[m] <= q) lo2 = m; else hi2 = m; }
            long long dst = (long long)tb[lo2] + (q - pre[lo2]);
            recs[2 * dst + (e & 1)] = st[e];
        }
        __syncthreads();
    }
}

int main() {
    const long long n = 100000000LL;
    std::vector<float> hv(n);
    for (long long i = 0; i < n; ++i) hv[i] = (float)(i & 1023) * 0.001f;
    float *u, *v, *h, *a0, *a1;
    for (float** p : {&u, &v, &h, &a0, &a1}) { CK(hipMalloc(p, n * 4)); CK(hipMemcpy(*p, hv.data(), n * 4, hipMemcpyHostToDevice)); }
    // exact counts for the layouts
    std::vector<long long> tc(NT, 0);
    for (long long i = 0; i < n; ++i) tc[tile_of((unsigned)i)]++;
    std::vector<long long> gc(G, 0);
    for (int t = 0; t < NT; ++t) gc[t / TPG] += tc[t];
    long long gcap = 0;
    for (int g = 0; g < G; ++g) gcap = std::max(gcap, gc[g]);
    std::vector<int> ts(NT);
    long long s = 0;
    for (int t = 0; t < NT; ++t) { ts[t] = (int)s; s += tc[t]; }
    float* gbuf; float4* recs; unsigned long long* gcur; int* tcur;
    CK(hipMalloc(&gbuf, (size_t)G * gcap * 24)); CK(hipMalloc(&recs, (size_t)n * 32));
    CK(hipMalloc(&gcur, G * 8)); CK(hipMalloc(&tcur, NT * 4));
    hipEvent_t e0, e1, e2; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int wpg : {16, 32}) {
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemset(gcur, 0, G * 8));
            CK(hipMemcpy(tcur, ts.data(), NT * 4, hipMemcpyHostToDevice));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_part, dim3(cus * 2), dim3(TA), 0, 0, u, v, h, a0, a1, n, gbuf, gcap, gcur);
            CK(hipEventRecord(e1));
            hipLaunchKernelGGL(k_scat, dim3(G * wpg), dim3(TB), 0, 0, gbuf, gcap, gcur, wpg, recs, tcur);
            CK(hipEventRecord(e2)); CK(hipEventSynchronize(e2));
            float ta, tb2; CK(hipEventElapsedTime(&ta, e0, e1)); CK(hipEventElapsedTime(&tb2, e1, e2));
            if (rep) printf("wpg %d: partition %.3f ms (%.0f GB/s of 44 B/pt), scatter %.3f ms (%.0f GB/s of 56 B/pt)\n", wpg, ta, n * 44.0 / ta / 1e6, tb2, n * 56.0 / tb2 / 1e6);
        }
    }
    // check: every slot of every tile written once (counts)
    std::vector<int> tc2(NT);
    CK(hipMemcpy(tc2.data(), tcur, NT * 4, hipMemcpyDeviceToHost));
    long long bad = 0;
    for (int t = 0; t < NT; ++t) bad += (tc2[t] - ts[t]) != tc[t];
    printf("tile count mismatches: %lld\n", bad);
    return 0;
}
