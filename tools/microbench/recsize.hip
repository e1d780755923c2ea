// Microbenchmark: cost of the record scatter vs the record SIZE / alignment on gfx950.
// B workgroups x 1024 threads write ~1e8 records into K tile segments; every (workgroup,
// tile) pair owns a contiguous run (k_scatter's layout); records arrive in pseudo-random
// tile order.  Variants:
//   S32   32-B records, two lanes per record (k_scatter's paired store)
//   S32x2 32-B records at a 64-B stride (the other 32 B untouched): line count of S64,
//         bytes of S32
//   S64   64-B records, four lanes per record
//   S128  128-B records (one full line), eight lanes per record
//   C32   32-B records to coalesced slots (reference)
// Every store is bounds-checked against the allocation.  Build & run:
//   hipcc -O3 --offload-arch=gfx950 -o tools/mb_recsize tools/microbench/recsize.hip
//   ./tools/mb_recsize
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int T = 1024;

// LPR: lanes per record (16 B each); STRIDE: record stride in 16-B units; COAL: coalesced
template <int LPR, int STRIDE, bool COAL>
__global__ __launch_bounds__(T) void k(float4* __restrict__ out, long long cap16, int K, int kshift,
                                       long long R, int B) {
    const int lane = threadIdx.x & 63;
    const int rpw = 64 / LPR;                 // records per wave instruction
    const long long nb = R * K;               // records per workgroup
    const int b = blockIdx.x;
    const int w = threadIdx.x >> 6;
    const long long TS = (long long)B * R + 61;  // tile stride in records
    for (long long j0 = (long long)w * rpw; j0 < nb; j0 += (long long)(T / 64) * rpw) {
        long long j = j0 + lane / LPR;         // this lane's record
        if (j >= nb) continue;
        long long c = j >> kshift;
        int t = (int)(((j & (K - 1)) * 2654435761u + c * 40503u) & (K - 1));
        long long slot = COAL ? (long long)b * nb + j : (long long)t * TS + (long long)b * R + c;
        long long idx = slot * STRIDE + (lane % LPR);
        if (idx < cap16) out[idx] = make_float4((float)j, (float)t, 1.f, 2.f);
    }
}

template <int LPR, int STRIDE, bool COAL>
float run(float4* d, long long cap16, int K, long long R, int B) {
    int ks = 0;
    while ((1 << ks) < K) ++ks;
    hipEvent_t a, e;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&e);
    hipLaunchKernelGGL((k<LPR, STRIDE, COAL>), dim3(B), dim3(T), 0, 0, d, cap16, K, ks, R, B);
    (void)hipEventRecord(a);
    for (int r = 0; r < 3; ++r)
        hipLaunchKernelGGL((k<LPR, STRIDE, COAL>), dim3(B), dim3(T), 0, 0, d, cap16, K, ks, R, B);
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms;
    (void)hipEventElapsedTime(&ms, a, e);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(e);
    return ms / 3;
}

int main() {
    const long long N = 100000000LL;
    const long long cap16 = (N + (1LL << 24)) * 8;  // 128 B per record + slack, in float4
    float4* d;
    if (hipMalloc(&d, (size_t)cap16 * 16) != hipSuccess) return 1;
    printf("K     B     S32    S32x2  S64    S128   C32   (ms, ~1e8 records)\n");
    for (int B : {256, 1024}) {
        for (int K : {1024, 4096}) {
            long long R = (N / B + K - 1) / K;
            float s32 = run<2, 2, false>(d, cap16, K, R, B);
            float s32x2 = run<2, 4, false>(d, cap16, K, R, B);
            float s64 = run<4, 4, false>(d, cap16, K, R, B);
            float s128 = run<8, 8, false>(d, cap16, K, R, B);
            float c32 = run<2, 2, true>(d, cap16, K, R, B);
            printf("%-5d %-5d %6.3f %6.3f %6.3f %6.3f %6.3f\n", K, B, s32, s32x2, s64, s128, c32);
        }
    }
    (void)hipFree(d);
    return 0;
}
