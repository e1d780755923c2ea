// Microbenchmark: direct global-atomic deposit of pixel-scale footprints (3 x 3 pixels,
// two fp32 maps of 4096^2) from 10^8 randomly ordered particles -- the alternative to
// binning for the headline pixel-h workload.  Measures no-return fp32 atomics
// (unsafeAtomicAdd -> global_atomic_add_f32) throughput on random addresses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_dep(const float* __restrict__ x, const float* __restrict__ y, long long n,
                      float* __restrict__ m0, float* __restrict__ m1, int G, int B) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int px = (int)x[i], py = (int)y[i];
    float w = 1.0f + 1e-3f * (float)(i & 7);
    for (int dx = 0; dx < B; ++dx)
        for (int dy = 0; dy < B; ++dy) {
            int X = min(px + dx, G - 1), Y = min(py + dy, G - 1);
            long long o = (long long)X * G + Y;
            unsafeAtomicAdd(&m0[o], w);
            if (m1) unsafeAtomicAdd(&m1[o], 2.0f * w);
        }
}

// the same with plain stores (no atomics): the non-atomic write cost of the same pattern
__global__ void k_store(const float* __restrict__ x, const float* __restrict__ y, long long n,
                        float* __restrict__ m0, float* __restrict__ m1, int G, int B) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int px = (int)x[i], py = (int)y[i];
    float w = 1.0f + 1e-3f * (float)(i & 7);
    for (int dx = 0; dx < B; ++dx)
        for (int dy = 0; dy < B; ++dy) {
            int X = min(px + dx, G - 1), Y = min(py + dy, G - 1);
            long long o = (long long)X * G + Y;
            m0[o] = w;
            if (m1) m1[o] = w;
        }
}

int main(int argc, char** argv) {
    long long n = argc > 1 ? atoll(argv[1]) : 100000000LL;
    int G = 4096;
    std::vector<float> hx(n), hy(n);
    unsigned s = 12345;
    for (long long i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u; hx[i] = (float)((s >> 8) % (G - 3)) + 0.5f;
        s = s * 1664525u + 1013904223u; hy[i] = (float)((s >> 8) % (G - 3)) + 0.5f;
    }
    float *x, *y, *m0, *m1;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
    CK(hipMalloc(&m0, (size_t)G * G * 4)); CK(hipMalloc(&m1, (size_t)G * G * 4));
    CK(hipMemcpy(x, hx.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(y, hy.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int T = 256; const unsigned blocks = (unsigned)((n + T - 1) / T);
    for (int B = 1; B <= 3; ++B) {
        for (int two = 0; two < 2; ++two) {
            for (int mode = 0; mode < 2; ++mode) {
                float best = 1e30f;
                for (int rep = 0; rep < 4; ++rep) {
                    CK(hipMemset(m0, 0, (size_t)G * G * 4)); CK(hipMemset(m1, 0, (size_t)G * G * 4));
                    CK(hipEventRecord(a));
                    if (mode == 0) hipLaunchKernelGGL(k_dep, dim3(blocks), dim3(T), 0, 0, x, y, n, m0, two ? m1 : nullptr, G, B);
                    else hipLaunchKernelGGL(k_store, dim3(blocks), dim3(T), 0, 0, x, y, n, m0, two ? m1 : nullptr, G, B);
                    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
                    float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
                }
                double ops = (double)n * B * B * (two ? 2 : 1);
                printf("%s box %dx%d maps %d: %.3f ms  %.3g ops/s\n", mode ? "store " : "atomic", B, B, two + 1, best, ops / (best * 1e-3));
            }
        }
    }
    return 0;
}
