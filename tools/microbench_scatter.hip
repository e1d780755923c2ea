// Microbenchmark: the record-scatter store pattern of k_scatter on gfx950.
// B workgroups x 1024 threads write ~1e8 32-B records into K tile segments; every
// (workgroup, tile) pair owns a contiguous run (the production layout), and records arrive
// in pseudo-random tile order.  Measures how the store cost depends on K (open lines per
// workgroup) and on the record layout.  Build & run:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mbs tools/microbench_scatter.hip && /tmp/mbs
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int T = 1024;

// MODE 0: tile-major segments, workgroup runs inside (production)
// MODE 1: coalesced destinations (same bytes)
// MODE 2: no stores
// MODE 3: tile-major, workgroup runs ordered by (b % 8, b / 8) (XCD classes adjacent)
// MODE 4: records as two planes (16-B {u,v,h,a0} plane + 4-B a1 plane), production order
template <int MODE>
__global__ __launch_bounds__(T) void k(float4* __restrict__ recs, float* __restrict__ plane1,
                                       int K, int kshift, long long R, int B) {
    const int lane = threadIdx.x & 63;
    const long long nb = R * K;  // records per workgroup
    const int b = blockIdx.x;
    const int bpos = MODE == 3 ? (b % 8) * (B / 8) + b / 8 : b;
    for (long long j0 = 0; j0 < nb; j0 += T) {
        long long j = j0 + threadIdx.x;
        long long c = j >> kshift;                               // chunk: each tile once
        int t = (int)(((j & (K - 1)) * 2654435761u + c * 40503u) & (K - 1));
        long long slot = (long long)t * B * R + (long long)bpos * R + c;
        if (MODE == 1) slot = (long long)b * nb + j;
        float4 v0 = make_float4((float)j, (float)t, 1.f, 2.f);
        if constexpr (MODE == 2) {
            asm volatile("" ::"v"(v0.x), "v"((int)slot));
        } else if constexpr (MODE == 4) {
            recs[slot] = v0;
            plane1[slot] = 3.f;
        } else {
            // paired store: lanes 2i, 2i+1 write the halves of record i (32 lines / instr)
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                int src = half * 32 + (lane >> 1);
                long long s = __shfl(slot, src);
                float4 val = (lane & 1) ? make_float4(3.f, 0.f, 0.f, 0.f)
                                        : make_float4(__shfl(v0.x, src), __shfl(v0.y, src), 1.f, 2.f);
                recs[2 * s + (lane & 1)] = val;
            }
        }
    }
}

template <int MODE>
float run(float4* d, float* p1, int K, long long R, int B) {
    int ks = 0;
    while ((1 << ks) < K) ++ks;
    hipEvent_t a, e;
    hipEventCreate(&a);
    hipEventCreate(&e);
    hipLaunchKernelGGL(k<MODE>, dim3(B), dim3(T), 0, 0, d, p1, K, ks, R, B);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k<MODE>, dim3(B), dim3(T), 0, 0, d, p1, K, ks, R, B);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, a, e);
    return ms / 3;
}

int main() {
    const long long N = 100000000LL;
    float4* d;
    float* p1;
    if (hipMalloc(&d, (size_t)(N + (1 << 22)) * 32) != hipSuccess) return 1;
    if (hipMalloc(&p1, (size_t)(N + (1 << 22)) * 4) != hipSuccess) return 1;
    printf("K     B     recs      prod   coal   none   xcdord planes (ms)\n");
    for (int B : {256, 512, 1024}) {
        for (int K : {64, 256, 1024, 2048, 4096, 8192}) {
            long long R = (N / B + K - 1) / K;
            float t0 = run<0>(d, p1, K, R, B);
            float t1 = run<1>(d, p1, K, R, B);
            float t2 = run<2>(d, p1, K, R, B);
            float t3 = run<3>(d, p1, K, R, B);
            float t4 = run<4>(d, p1, K, R, B);
            printf("%-5d %-5d %-9lld %6.3f %6.3f %6.3f %6.3f %6.3f\n", K, B, R * K * B, t0, t1, t2, t3, t4);
        }
    }
    return 0;
}
