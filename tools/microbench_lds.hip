// Microbenchmark: LDS accumulation primitives on gfx950 (random addresses in a 64x64x2
// fp32 tile, the deposit kernel's access pattern).  Build & run:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mb tools/microbench_lds.hip && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 8192;  // 2 x 64 x 64 floats
constexpr int ITERS = 4096;

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int span) {
    __shared__ float lds[N];
    __shared__ unsigned long long lds64[N / 2];
    for (int i = threadIdx.x; i < N; i += 256) lds[i] = 0.f;
    for (int i = threadIdx.x; i < N / 2; i += 256) lds64[i] = 0;
    __syncthreads();
    uint32_t s = hash(blockIdx.x * 256 + threadIdx.x);
    float val = 1.0f + (threadIdx.x & 7);
    for (int it = 0; it < ITERS; ++it) {
        s = hash(s + it);
        int a = (int)(s % (uint32_t)span);
        if constexpr (MODE == 0) atomicAdd(&lds[a], val);                      // ds_add_f32
        else if constexpr (MODE == 1) atomicAdd((unsigned*)&lds[a], (unsigned)val);  // ds_add_u32
        else if constexpr (MODE == 2) lds[a] = val;                            // ds_write_b32
        else if constexpr (MODE == 3) atomicAdd(&lds64[a >> 1], (unsigned long long)val);  // ds_add_u64
        else if constexpr (MODE == 4) { float t = lds[a]; lds[a] = t + val; }  // racy RMW
        else if constexpr (MODE == 5) {  // contiguous per wave (lanes consecutive)
            int b = ((s >> 6) % (uint32_t)(span / 64)) * 64 + (threadIdx.x & 63);
            b = __builtin_amdgcn_readfirstlane(b - (threadIdx.x & 63)) + (threadIdx.x & 63);
            atomicAdd(&lds[b], val);
        }
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = threadIdx.x; i < N; i += 256) acc += lds[i] + (float)lds64[i / 2];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
float run(float* d, int blocks, int span) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, d, span);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, d, span);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main() {
    int blocks = 256 * 8;
    float* d; hipMalloc(&d, blocks * 256 * sizeof(float));
    const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_write_b32", "ds_add_u64", "racy_rmw", "ds_add_f32 contiguous"};
    for (int span : {8192, 4096, 256}) {
        float t[6];
        t[0] = run<0>(d, blocks, span); t[1] = run<1>(d, blocks, span); t[2] = run<2>(d, blocks, span);
        t[3] = run<3>(d, blocks, span); t[4] = run<4>(d, blocks, span); t[5] = run<5>(d, blocks, span);
        double ops = (double)blocks * 256 * ITERS;
        for (int m = 0; m < 6; ++m)
            printf("span %5d %-24s %8.3f ms  %7.2f G lane-ops/s  %6.2f lane-ops/clk/CU@2.4GHz\n", span, names[m], t[m],
                   ops / t[m] / 1e6, ops / (t[m] * 1e-3) / 256 / 2.4e9);
    }
    return 0;
}
