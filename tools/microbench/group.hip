// Microbenchmark: record scatter with per-GROUP shared tile runs vs per-workgroup runs.
//
// k_scatter today gives every (workgroup, tile) pair its own run: 256 workgroups x 4096
// tiles = 1M open record lines, far more than the 4 MiB L2 of an XCD holds, so most
// 32-B records leave L2 as partial lines.  Here the workgroups of one group g = b % 8
// (one XCD under round-robin placement; speed only) share ONE run per tile, claimed by a
// returning device-scope atomicAdd per record: 4096 open lines per XCD.
//   P32   private runs (k_scatter's layout), LDS cursors, paired 32-B stores
//   G32   group runs, global cursors (one returning atomic per lane), paired 32-B stores
//   G32h  as G32, tiles drawn from a Plummer-like concentrated distribution
//   C32   coalesced stores (floor)
// Build & run:
//   hipcc -O3 --offload-arch=gfx950 -o tools/mb_group tools/microbench/group.hip && ./tools/mb_group
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int T = 1024;

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// MODE 0: private runs; 1: group runs; 2: coalesced.  CONC: concentrated tiles.
template <int MODE, bool CONC>
__global__ __launch_bounds__(T) void k(float4* __restrict__ out, long long cap16, int K,
                                       long long per_wg, const long long* __restrict__ base,
                                       int* __restrict__ gcur, const int* __restrict__ pick) {
    extern __shared__ int cur[];
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    if (MODE == 0 || MODE == 3) {
        for (int t = threadIdx.x; t < K; t += T) cur[t] = (int)base[(long long)b * K + t];
        __syncthreads();
    }
    const int g = b & 7;
    for (long long j0 = 0; j0 < per_wg; j0 += T) {
        long long j = j0 + threadIdx.x;
        bool live = j < per_wg;
        unsigned hsh = hash32((unsigned)(b * per_wg + j));
        int t = CONC ? pick[hsh & 65535] : (int)(hsh & (K - 1));
        int slot = -1;
        if (live) {
            if (MODE == 0 || MODE == 3) slot = atomicAdd(&cur[t], 1);
            else if (MODE == 1) slot = atomicAdd(&gcur[g * K + t], 1);
            else slot = (int)(b * per_wg + j);
        }
        float4 v0 = make_float4((float)j, (float)t, 1.f, 2.f);
        if (MODE == 3) {  // private runs, 64-B records: lanes 4i .. 4i+3 write record i
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                int src = q * 16 + (lane >> 2);
                int s = __shfl(slot, src);
                float4 val = make_float4(__shfl(v0.x, src), __shfl(v0.y, src), (float)(lane & 3), 2.f);
                long long idx = 4 * (long long)s + (lane & 3);
                if (s >= 0 && idx < cap16) out[idx] = val;
            }
            continue;
        }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            int src = half * 32 + (lane >> 1);
            int s = __shfl(slot, src);
            float4 val = (lane & 1) ? make_float4(3.f, 0.f, 0.f, 0.f)
                                    : make_float4(__shfl(v0.x, src), __shfl(v0.y, src), 1.f, 2.f);
            long long idx = 2 * (long long)s + (lane & 1);
            if (s >= 0 && idx < cap16) out[idx] = val;
        }
    }
}

int main() {
    const long long N = 100000000LL;
    const long long cap16 = (N + (1LL << 22)) * 4;
    float4* d;
    if (hipMalloc(&d, (size_t)cap16 * 16) != hipSuccess) return 1;
    const int K = 4096;
    // concentrated tile table: 64 x 64 tiles, weight ~ (1 + R^2)^-2 with R in [-4, 4]
    std::vector<int> pick(65536);
    {
        std::vector<double> w(K);
        double tot = 0;
        for (int t = 0; t < K; ++t) {
            double x = ((t / 64) + 0.5) / 8.0 - 4.0, y = ((t % 64) + 0.5) / 8.0 - 4.0;
            double r2 = x * x + y * y;
            w[t] = 1.0 / ((1 + r2) * (1 + r2));
            tot += w[t];
        }
        double acc = 0;
        int t = 0;
        for (int i = 0; i < 65536; ++i) {
            double q = (i + 0.5) / 65536.0 * tot;
            while (t < K - 1 && acc + w[t] < q) acc += w[t++];
            pick[i] = t;
        }
    }
    int* dpick;
    (void)hipMalloc(&dpick, 65536 * 4);
    (void)hipMemcpy(dpick, pick.data(), 65536 * 4, hipMemcpyHostToDevice);
    printf("B     mode  conc   ms (1e8 records, 32 B)\n");
    for (int B : {256}) {
        long long per_wg = (N + B - 1) / B;
        for (int conc = 0; conc < 2; ++conc) {
            // exact counts per (wg, tile) and per (group, tile) on the host
            std::vector<long long> cnt_wg((size_t)B * K, 0), cnt_g(8 * K, 0);
            for (int b = 0; b < B; ++b)
                for (long long j = 0; j < per_wg; ++j) {
                    unsigned x = (unsigned)(b * per_wg + j);
                    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
                    int t = conc ? pick[x & 65535] : (int)(x & (K - 1));
                    cnt_wg[(size_t)b * K + t]++;
                    cnt_g[(b & 7) * K + t]++;
                }
            // private layout: tile-major, then wg;  group layout: tile-major, then group
            std::vector<long long> base_wg((size_t)B * K);
            std::vector<int> base_g(8 * K);
            long long off = 0;
            for (int t = 0; t < K; ++t)
                for (int b = 0; b < B; ++b) { base_wg[(size_t)b * K + t] = off; off += cnt_wg[(size_t)b * K + t]; }
            off = 0;
            for (int t = 0; t < K; ++t)
                for (int g = 0; g < 8; ++g) { base_g[g * K + t] = (int)off; off += cnt_g[g * K + t]; }
            long long* dbase;
            int *dg, *dg0;
            (void)hipMalloc(&dbase, base_wg.size() * 8);
            (void)hipMemcpy(dbase, base_wg.data(), base_wg.size() * 8, hipMemcpyHostToDevice);
            (void)hipMalloc(&dg, 8 * K * 4);
            (void)hipMalloc(&dg0, 8 * K * 4);
            (void)hipMemcpy(dg0, base_g.data(), 8 * K * 4, hipMemcpyHostToDevice);
            for (int mode = 0; mode < 4; ++mode) {
                hipEvent_t a, e;
                (void)hipEventCreate(&a);
                (void)hipEventCreate(&e);
                float tot = 0;
                for (int r = 0; r < 4; ++r) {
                    (void)hipMemcpy(dg, dg0, 8 * K * 4, hipMemcpyDeviceToDevice);
                    (void)hipEventRecord(a);
                    if (mode == 0 && conc == 0) hipLaunchKernelGGL((k<0, false>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 0 && conc == 1) hipLaunchKernelGGL((k<0, true>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 1 && conc == 0) hipLaunchKernelGGL((k<1, false>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 1 && conc == 1) hipLaunchKernelGGL((k<1, true>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 2 && conc == 0) hipLaunchKernelGGL((k<2, false>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 2 && conc == 1) hipLaunchKernelGGL((k<2, true>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 3 && conc == 0) hipLaunchKernelGGL((k<3, false>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    if (mode == 3 && conc == 1) hipLaunchKernelGGL((k<3, true>), dim3(B), dim3(T), K * 4, 0, d, cap16, K, per_wg, dbase, dg, dpick);
                    (void)hipEventRecord(e);
                    (void)hipEventSynchronize(e);
                    float ms;
                    (void)hipEventElapsedTime(&ms, a, e);
                    if (r > 0) tot += ms;
                }
                printf("%-5d %-5s %-5d %7.3f\n", B, mode == 0 ? "P32" : mode == 1 ? "G32" : mode == 2 ? "C32" : "P64", conc, tot / 3);
                (void)hipEventDestroy(a);
                (void)hipEventDestroy(e);
            }
            (void)hipFree(dbase);
            (void)hipFree(dg);
            (void)hipFree(dg0);
        }
    }
    (void)hipFree(d);
    return 0;
}
