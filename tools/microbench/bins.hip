// Microbenchmark (round 5): does binning the scatter's records into COARSER bins (2 or 4
// GPU tiles per bin: fewer (workgroup, bin) runs open at once) speed up the scatter on the
// Plummer-skewed tile distribution of the headline map?  1e8 32-B records, 256 workgroups x
// 512 threads x 2 records per lane per batch (k_scatter's shape: LDS cursor per bin,
// paired 16-B stores), one record buffer for every variant (same placement), bins of
// 64x64 tiles merged 1x1 (4096 bins), 2x1 (2048), 2x2 (1024), 4x4 (256).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_bins tools/microbench/bins.hip && /tmp/mb_bins
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

constexpr int T = 512;
constexpr int U = 2;
constexpr int NB = 256;           // workgroups
constexpr int TABN = 1 << 22;     // tile ids drawn from a Plummer-like table
constexpr long long NREC = 100000000LL;

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// tile t = tx * 64 + ty -> bin of (tx >> sx, ty >> sy)
__device__ __host__ __forceinline__ int bin_of(int t, int sx, int sy) {
    const int tx = t >> 6, ty = t & 63;
    return ((tx >> sx) << (6 - sy)) + (ty >> sy);
}

__global__ __launch_bounds__(T) void k(float4* __restrict__ out, const int* __restrict__ tab,
                                       long long per_wg, const long long* __restrict__ base,
                                       int nbins, int sx, int sy) {
    extern __shared__ int cur[];
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    for (int t = threadIdx.x; t < nbins; t += T) cur[t] = (int)base[(long long)b * nbins + t];
    __syncthreads();
    for (long long j0 = 0; j0 < per_wg; j0 += T * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long j = j0 + u * T + threadIdx.x;
            const int t = tab[hash32((unsigned)(b * per_wg + j)) & (TABN - 1)];
            const int bn = bin_of(t, sx, sy);
            const int slot = j < per_wg ? atomicAdd(&cur[bn], 1) : -1;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int src = half * 32 + (lane >> 1);
                const int s = __shfl(slot, src);
                const float4 val = (lane & 1) ? make_float4(3.f, 0.f, 0.f, 0.f)
                                              : make_float4((float)__shfl((int)j, src), 1.f, 2.f, 3.f);
                if (s >= 0) out[2 * (long long)s + (lane & 1)] = val;
            }
        }
    }
}

int main() {
    // Plummer surface density (1 + R^2)^-2 over [-4, 4]^2, 64 x 64 tiles
    std::vector<double> w(4096);
    double sum = 0.0;
    for (int tx = 0; tx < 64; ++tx)
        for (int ty = 0; ty < 64; ++ty) {
            double x = -4.0 + (tx + 0.5) * 0.125, y = -4.0 + (ty + 0.5) * 0.125;
            double r2 = x * x + y * y;
            w[tx * 64 + ty] = 1.0 / ((1.0 + r2) * (1.0 + r2));
            sum += w[tx * 64 + ty];
        }
    std::vector<int> tab(TABN);
    {
        double acc = 0.0;
        int t = 0;
        double edge = w[0];
        for (int i = 0; i < TABN; ++i) {
            double q = (i + 0.5) / TABN * sum;
            while (q > edge && t < 4095) edge += w[++t];
            tab[i] = t;
        }
        (void)acc;
    }
    int* dtab;
    hipMalloc(&dtab, TABN * sizeof(int));
    hipMemcpy(dtab, tab.data(), TABN * sizeof(int), hipMemcpyHostToDevice);
    const long long per_wg = NREC / NB;
    float4* out;
    hipMalloc(&out, (size_t)NREC * 32 + (1 << 20));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int cfg[4][2] = {{0, 0}, {1, 0}, {1, 1}, {2, 2}};
    long long* dbase[4];
    auto h32 = [](unsigned x) {
        x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
        return x;
    };
    std::vector<int> tile_of_rec((size_t)NB * per_wg);  // the hash stream's tiles, once
    for (int b = 0; b < NB; ++b)
        for (long long j = 0; j < per_wg; ++j)
            tile_of_rec[(size_t)b * per_wg + j] = tab[h32((unsigned)(b * per_wg + j)) & (TABN - 1)];
    for (int c = 0; c < 4; ++c) {  // exact run bases per (workgroup, bin), bin-major
        const int sx = cfg[c][0], sy = cfg[c][1], nbins = (64 >> sx) * (64 >> sy);
        std::vector<long long> cnt((size_t)NB * nbins, 0), base((size_t)NB * nbins);
        for (int b = 0; b < NB; ++b)
            for (long long j = 0; j < per_wg; ++j)
                ++cnt[(size_t)b * nbins + bin_of(tile_of_rec[(size_t)b * per_wg + j], sx, sy)];
        long long o = 0;
        for (int bn = 0; bn < nbins; ++bn)
            for (int b = 0; b < NB; ++b) {
                base[(size_t)b * nbins + bn] = o;
                o += cnt[(size_t)b * nbins + bn];
            }
        hipMalloc(&dbase[c], base.size() * sizeof(long long));
        hipMemcpy(dbase[c], base.data(), base.size() * sizeof(long long), hipMemcpyHostToDevice);
    }
    for (int rep = 0; rep < 3; ++rep)
        for (int c = 0; c < 4; ++c) {
            const int sx = cfg[c][0], sy = cfg[c][1], nbins = (64 >> sx) * (64 >> sy);
            hipLaunchKernelGGL(k, dim3(NB), dim3(T), nbins * 4, 0, out, dtab, per_wg, dbase[c], nbins, sx, sy);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(NB), dim3(T), nbins * 4, 0, out, dtab, per_wg, dbase[c], nbins, sx, sy);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("rep %d  bins %4d (%dx%d tiles)  %.3f ms\n", rep, nbins, 1 << sx, 1 << sy, ms);
            fflush(stdout);
        }
    return 0;
}
