// Microbenchmark: LDS accumulation primitives on gfx950 (random addresses in a 64x64x2
// fp32 tile, the deposit kernel's access pattern).  Build & run:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mb tools/microbench/lds.hip && /tmp/mb
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
    __shared__ unsigned long long hi64[MODE >= 10 ? N / 2 : 1];  // the two-word fixed point
    for (int i = threadIdx.x; i < N; i += 256) lds[i] = 0.f;
    for (int i = threadIdx.x; i < N / 2; i += 256) lds64[i] = 0;
    for (int i = threadIdx.x; i < (MODE >= 10 ? N / 2 : 1); i += 256) hi64[i] = 0;
    __syncthreads();
    uint32_t s = hash(blockIdx.x * 256 + threadIdx.x);
    float val = 1.0f + (threadIdx.x & 7);
    unsigned mask = (unsigned)span - 1u;  // span is a power of two
    for (int it = 0; it < ITERS; ++it) {
        s = s * 1664525u + 1013904223u;   // LCG: 2 VALU ops
        int a = (int)((s >> 7) & mask);
        if constexpr (MODE == 0) atomicAdd(&lds[a], val);                      // ds_add_f32
        else if constexpr (MODE == 1) atomicAdd((unsigned*)&lds[a], (unsigned)val);  // ds_add_u32
        else if constexpr (MODE == 2) lds[a] = val;                            // ds_write_b32
        else if constexpr (MODE == 3) atomicAdd(&lds64[a >> 1], (unsigned long long)val);  // ds_add_u64
        else if constexpr (MODE == 4) { float t = lds[a]; lds[a] = t + val; }  // racy RMW
        else if constexpr (MODE == 5) {  // ds_add_rtn_u32 (cursor-style, result used)
            unsigned r = atomicAdd((unsigned*)&lds[a], 1u);
            val += (float)(r & 1u);
        }
        else if constexpr (MODE == 6) atomicAdd((double*)&lds64[a >> 1], (double)val);  // ds_add_f64
        else if constexpr (MODE == 7) atomicMax((unsigned*)&lds[a], (unsigned)val);    // ds_max_u32
        else if constexpr (MODE == 8) {  // ds_add_f64, lanes of each 32-lane half on distinct banks
            int w = ((a >> 1) & ~31) | (threadIdx.x & 31);
            atomicAdd((double*)&lds64[w & (N / 2 - 1)], (double)val);
        } else if constexpr (MODE == 9) {  // ds_add_f64, the deposit's column-only bank mapping:
            int w = ((a >> 1) & ~63) | ((threadIdx.x * 37 + (a >> 7)) & 63);  // random column
            atomicAdd((double*)&lds64[w & (N / 2 - 1)], (double)val);
        } else if constexpr (MODE == 10) {  // two-word fixed point: hi and lo ds_add_u64 each
            // (verdict r05 item 3): t = val * 2^k, hi = floor(t), lo = frac(t) * 2^32
            const double t = (double)val * 0x1p20;
            const double fh = floor(t);
            const unsigned long long hi = (unsigned long long)(long long)fh;
            const unsigned long long lo = (unsigned long long)((t - fh) * 0x1p32);
            atomicAdd(&lds64[a >> 1], lo);
            atomicAdd(&hi64[a >> 1], hi);
        } else if constexpr (MODE == 11) {  // the same words, the conversion omitted
            atomicAdd(&lds64[a >> 1], (unsigned long long)val);
            atomicAdd(&hi64[a >> 1], (unsigned long long)s);
        }
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = threadIdx.x; i < N; i += 256)
        acc += lds[i] + (float)lds64[i / 2] + (MODE >= 10 ? (float)hi64[(i / 2) % (MODE >= 10 ? N / 2 : 1)] : 0.f);
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
    const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_write_b32", "ds_add_u64", "racy_rmw",
                           "ds_add_rtn_u32", "ds_add_f64", "ds_max_u32", "ds_add_f64 distinct",
                           "ds_add_f64 random col", "2x ds_add_u64 (2-word fix)",
                           "2x ds_add_u64 (no cvt)"};
    for (int span : {8192, 256}) {
        float t[12];
        t[0] = run<0>(d, blocks, span); t[1] = run<1>(d, blocks, span); t[2] = run<2>(d, blocks, span);
        t[3] = run<3>(d, blocks, span); t[4] = run<4>(d, blocks, span); t[5] = run<5>(d, blocks, span);
        t[6] = run<6>(d, blocks, span); t[7] = run<7>(d, blocks, span);
        t[8] = run<8>(d, blocks, span); t[9] = run<9>(d, blocks, span);
        t[10] = run<10>(d, blocks, span); t[11] = run<11>(d, blocks, span);
        double ops = (double)blocks * 256 * ITERS;
        for (int m = 0; m < 12; ++m)
            printf("span %5d %-24s %8.3f ms  %7.2f G lane-ops/s  %6.2f lane-ops/clk/CU@2.4GHz\n", span, names[m], t[m],
                   ops / t[m] / 1e6, ops / (t[m] * 1e-3) / 256 / 2.4e9);
    }
    return 0;
}
