// Microbenchmark: cost of the record scatter vs the number of tile runs each workgroup
// keeps open (tiles per workgroup, TPW).  256 workgroups x 1024 threads write 1e8 32-B
// records (k_scatter's paired stores) into private (workgroup, tile) runs; workgroup b
// writes only to the TPW tiles of its tile group (b / 8) % (4096 / TPW) -- the groups
// are spread so that the 32 workgroups of one XCD (b % 8 equal) cover all groups.
// Open record lines per XCD = 32 x TPW.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mb_tpw tools/microbench/tpw.hip && ./tools/mb_tpw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int T = 1024;

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(T) void k(float4* __restrict__ out, long long cap16, int tpw,
                                       long long per_wg, const long long* __restrict__ base) {
    extern __shared__ int cur[];
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    for (int t = threadIdx.x; t < tpw; t += T) cur[t] = (int)base[(long long)b * tpw + t];
    __syncthreads();
    for (long long j0 = 0; j0 < per_wg; j0 += T) {
        long long j = j0 + threadIdx.x;
        int t = (int)(hash32((unsigned)(b * per_wg + j)) & (tpw - 1));
        int slot = j < per_wg ? atomicAdd(&cur[t], 1) : -1;
        float4 v0 = make_float4((float)j, (float)t, 1.f, 2.f);
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
    const int B = 256;
    const long long per_wg = N / B;
    const long long cap16 = (N + (1LL << 22)) * 2;
    float4* d;
    if (hipMalloc(&d, (size_t)cap16 * 16) != hipSuccess) return 1;
    printf("TPW   open/XCD  ms (1e8 x 32 B)\n");
    for (int tpw : {4096, 1024, 512, 256, 128, 64}) {
        int ng = 4096 / tpw;
        // exact per-(wg, local tile) counts; layout tile-major over global tiles
        std::vector<long long> cnt((size_t)B * tpw, 0), base((size_t)B * tpw);
        for (int b = 0; b < B; ++b)
            for (long long j = 0; j < per_wg; ++j) {
                unsigned x = (unsigned)(b * per_wg + j);
                x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
                cnt[(size_t)b * tpw + (x & (tpw - 1))]++;
            }
        long long off = 0;
        for (int g = 0; g < ng; ++g)
            for (int t = 0; t < tpw; ++t)
                for (int b = 0; b < B; ++b)
                    if ((b / 8) % ng == g) { base[(size_t)b * tpw + t] = off; off += cnt[(size_t)b * tpw + t]; }
        long long* dbase;
        (void)hipMalloc(&dbase, base.size() * 8);
        (void)hipMemcpy(dbase, base.data(), base.size() * 8, hipMemcpyHostToDevice);
        hipEvent_t a, e;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&e);
        hipLaunchKernelGGL(k, dim3(B), dim3(T), tpw * 4, 0, d, cap16, tpw, per_wg, dbase);
        (void)hipEventRecord(a);
        for (int r = 0; r < 3; ++r)
            hipLaunchKernelGGL(k, dim3(B), dim3(T), tpw * 4, 0, d, cap16, tpw, per_wg, dbase);
        (void)hipEventRecord(e);
        (void)hipEventSynchronize(e);
        float ms;
        (void)hipEventElapsedTime(&ms, a, e);
        printf("%-5d %-9d %7.3f\n", tpw, 32 * tpw, ms / 3);
        (void)hipFree(dbase);
    }
    (void)hipFree(d);
    return 0;
}
