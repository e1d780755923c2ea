// Microbenchmark (round 5, verdict r04 item 4): can a segmented reduction beat the
// deposit's fp64 LDS atomics on gfx950?  One 64x64 tile per workgroup, two maps, batches of
// 512 random 3x3-pixel boxes (one per thread, 9 pairs each -- the pixel-scale-h deposit's
// shape), NB batches per workgroup, 512 workgroups (2 per CU).
//   A  atomics:   every pair -> two ds_add_f64 into the padded 64x65 fp64 tiles (k_deposit)
//   S  segmented: per batch, a counting sort of the pairs by pixel in LDS -- count
//                 (ds_add_u32), block scan of the 4096 counters (8 per thread), place
//                 (ds_add_rtn_u32 on the offsets + one ds_write_b64 of the (t0, t1) pair),
//                 then every thread sums the segments of ITS 8 pixels in fp64 registers (no
//                 atomics at all on the accumulators); 4 block barriers per batch
//   S1 segmented without the final reads (the sort alone)
// Prints ms and pairs/ns; both produce the same sums (checked).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_seg tools/microbench/segred.hip && /tmp/mb_seg
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int T = 512;        // threads per workgroup
constexpr int NPIX = 4096;    // 64 x 64
constexpr int ROW = 65;       // padded LDS row (k_deposit's layout)
constexpr int CAP = T * 9;    // pairs per batch

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// record r of batch b: box origin (0..61)^2, two coefficients
__device__ __forceinline__ void record(unsigned seed, int& x0, int& y0, float& c0, float& c1) {
    unsigned h = hash32(seed);
    x0 = (int)(h % 62u);
    y0 = (int)((h >> 8) % 62u);
    c0 = 1.0f + (float)(h >> 24) * (1.0f / 256.0f);
    c1 = 0.5f + (float)((h >> 16) & 255u) * (1.0f / 512.0f);
}

__device__ __forceinline__ float wgt(int i, int j) { return 1.0f / (1.0f + (float)(i * 3 + j)); }

__global__ __launch_bounds__(T) void kA(int nb, double* out) {
    extern __shared__ double acc[];  // 2 x 64 x 65
    for (int i = threadIdx.x; i < 2 * 64 * ROW; i += T) acc[i] = 0.0;
    __syncthreads();
    for (int b = 0; b < nb; ++b) {
        int x0, y0;
        float c0, c1;
        record((blockIdx.x * nb + b) * T + threadIdx.x, x0, y0, c0, c1);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int w = (x0 + i) * ROW + y0 + j;
                const float wt = wgt(i, j);
                atomicAdd(&acc[w], (double)(c0 * wt));
                atomicAdd(&acc[64 * ROW + w], (double)(c1 * wt));
            }
    }
    __syncthreads();
    double s = 0.0;
    for (int k = threadIdx.x; k < NPIX; k += T) {
        const int w = (k >> 6) * ROW + (k & 63);
        s += acc[w] + 2.0 * acc[64 * ROW + w];
    }
    atomicAdd(&out[blockIdx.x], s);
}

template <bool READ>
__global__ __launch_bounds__(T) void kS(int nb, double* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned smem[];
    unsigned* cnt = smem;                          // 4096 counters -> offsets
    float2* buf = (float2*)(smem + NPIX);          // CAP pairs
    unsigned* wsum = (unsigned*)(buf + CAP);       // 8 wave totals
    for (int i = threadIdx.x; i < NPIX; i += T) cnt[i] = 0u;
    double a0[8], a1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = a1[i] = 0.0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    for (int b = 0; b < nb; ++b) {
        int x0, y0;
        float c0, c1;
        record((blockIdx.x * nb + b) * T + threadIdx.x, x0, y0, c0, c1);
        // 1. count
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) atomicAdd(&cnt[(x0 + i) * 64 + y0 + j], 1u);
        __syncthreads();
        // 2. scan: thread t owns counters 8t .. 8t + 7
        uint4 qa = *(uint4*)&cnt[8 * threadIdx.x], qb = *(uint4*)&cnt[8 * threadIdx.x + 4];
        unsigned c[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        unsigned tot = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) tot += c[i];
        unsigned inc = tot;  // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            unsigned v = __shfl_up(inc, d);
            if (lane >= d) inc += v;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        unsigned base = inc - tot;
        for (int w = 0; w < wv; ++w) base += wsum[w];
        unsigned off[9];
        off[0] = base;
#pragma unroll
        for (int i = 0; i < 8; ++i) off[i + 1] = off[i] + c[i];
        *(uint4*)&cnt[8 * threadIdx.x] = make_uint4(off[0], off[1], off[2], off[3]);
        *(uint4*)&cnt[8 * threadIdx.x + 4] = make_uint4(off[4], off[5], off[6], off[7]);
        __syncthreads();
        // 3. place
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const unsigned pos = atomicAdd(&cnt[(x0 + i) * 64 + y0 + j], 1u);
                const float wt = wgt(i, j);
                buf[pos] = make_float2(c0 * wt, c1 * wt);
            }
        __syncthreads();
        // 4. owners sum their segments; counters zeroed for the next batch
        if (READ) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                for (unsigned q = off[i]; q < off[i + 1]; ++q) {
                    const float2 t = buf[q];
                    a0[i] += (double)t.x;
                    a1[i] += (double)t.y;
                }
        }
        *(uint4*)&cnt[8 * threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
        *(uint4*)&cnt[8 * threadIdx.x + 4] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a0[i] + 2.0 * a1[i];
    atomicAdd(&out[blockIdx.x], s);
}

int main() {
    const int blocks = 512, nb = 400;
    double* d;
    hipMalloc(&d, blocks * sizeof(double));
    const size_t ldsA = 2 * 64 * ROW * sizeof(double);
    const size_t ldsS = NPIX * 4 + CAP * 8 + 64;
    hipFuncSetAttribute((const void*)kA, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsA);
    hipFuncSetAttribute((const void*)kS<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsS);
    hipFuncSetAttribute((const void*)kS<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsS);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<double> ha(blocks), hs(blocks);
    const double pairs = (double)blocks * nb * T * 9;
    for (int rep = 0; rep < 3; ++rep) {
        float ms[3];
        for (int v = 0; v < 3; ++v) {
            hipMemset(d, 0, blocks * sizeof(double));
            hipEventRecord(e0);
            if (v == 0) hipLaunchKernelGGL(kA, dim3(blocks), dim3(T), ldsA, 0, nb, d);
            else if (v == 1) hipLaunchKernelGGL(kS<true>, dim3(blocks), dim3(T), ldsS, 0, nb, d);
            else hipLaunchKernelGGL(kS<false>, dim3(blocks), dim3(T), ldsS, 0, nb, d);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms[v], e0, e1);
            if (v < 2) hipMemcpy(v == 0 ? ha.data() : hs.data(), d, blocks * sizeof(double),
                                 hipMemcpyDeviceToHost);
        }
        double dev = 0.0;
        for (int i = 0; i < blocks; ++i) dev = std::max(dev, std::abs(ha[i] - hs[i]) / std::abs(ha[i]));
        printf("rep %d  A atomics %.3f ms (%.1f pairs/ns)  S segmented %.3f ms (%.1f)  S1 sort only %.3f ms  max rel diff %.2e\n",
               rep, ms[0], pairs / ms[0] / 1e6, ms[1], pairs / ms[1] / 1e6, ms[2], dev);
    }
    return 0;
}
