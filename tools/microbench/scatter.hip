// Microbenchmark: the record-scatter store pattern of k_scatter on gfx950.
// B workgroups x 1024 threads write ~1e8 32-B records into K tile segments; every
// (workgroup, tile) pair owns a contiguous run (the production layout), and records arrive
// in pseudo-random tile order.  Measures how the store cost depends on K (open lines per
// workgroup) and on the record layout.  Build & run:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mbs tools/microbench/scatter.hip && /tmp/mbs
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int T = 1024;

// MODE 0: tile-major segments, workgroup runs inside (production)
// MODE 1: coalesced destinations (same bytes)
// MODE 2: no stores
// MODE 3: tile-major, workgroup runs ordered by (b % 8, b / 8) (XCD classes adjacent)
// MODE 4: records as two planes (16-B {u,v,h,a0} plane + 4-B a1 plane), production order
// MODE 5: XCD-affine regions: workgroup b only writes the K/8 tiles of region b % 8 (blocks
//         b, b + 8, ... share an XCD), production layout
// MODE 6: pass-1 shape: each wave's records grouped by 8 regions, 8 consecutive slots per
//         region and wave (region-major layout, workgroup runs inside)
// MODE 7: LDS-staged full lines: every 8 lanes write one whole 128-B line (4 records) of a
//         tile of region b % 8 (K/8 tiles per region)
// MODE 8: as 7 over all K tiles
template <int MODE>
__global__ __launch_bounds__(T) void k(float4* __restrict__ recs, float* __restrict__ plane1,
                                       int K, int kshift, long long R, int B) {
    const long long cap = (100000000LL + (1LL << 24)) * 2;  // float4 slots allocated
    const int lane = threadIdx.x & 63;
    const long long nb = R * K;  // records per workgroup
    const int b = blockIdx.x;
    const int bpos = MODE == 3 ? (b % 8) * (B / 8) + b / 8 : b;
    const long long nj = (MODE == 7 || MODE == 8) ? 2 * nb : nb;  // 16-B pieces there
    for (long long j0 = 0; j0 < nj; j0 += T) {
        long long j = j0 + threadIdx.x;
        long long c = j >> kshift;                               // chunk: each tile once
        int t = (int)(((j & (K - 1)) * 2654435761u + c * 40503u) & (K - 1));
        long long TS = (long long)B * R + 61;  // tile stride: no power-of-two alignment
        long long slot = (long long)t * TS + (long long)bpos * R + c;
        if (MODE == 1) slot = (long long)b * nb + j;
        if (MODE == 5) {  // K/8 tiles per workgroup, each (B/8 workgroups) x (8R records)
            const int K8 = K >> 3;
            long long c8 = j >> (kshift - 3);
            int t8 = (int)(((j & (K8 - 1)) * 2654435761u + c8 * 40503u) & (K8 - 1));
            t = (b & 7) * K8 + t8;
            slot = (long long)t * TS + (long long)(b >> 3) * (8 * R + 1) + c8;
        }
        if (MODE == 6) {  // 8 regions; wave w, lane l: region l >> 3 ... records 2 per lane below
            long long RR = nb / 8 + 64;       // records per (workgroup, region)
            long long wi = j0 / T;            // iteration
            int w = threadIdx.x >> 6;
            int reg = (lane >> 3);
            slot = (long long)reg * B * RR + (long long)b * RR + ((wi * (T / 64) + w) * 8 + (lane & 7)) % RR;
        }
        if (MODE == 7 || MODE == 8) {   // line granularity: slot is a LINE index (4 records)
            const int KT = MODE == 7 ? (K >> 3) : K;
            const int ks = MODE == 7 ? kshift - 3 : kshift;
            long long line = j >> 3;      // 8 lanes per line
            long long cl = line >> ks;
            int tt = (int)(((line & (KT - 1)) * 2654435761u + cl * 40503u) & (KT - 1));
            int tile = MODE == 7 ? (b & 7) * KT + tt : tt;
            int nbk = MODE == 7 ? B / 8 : B;
            int bb = MODE == 7 ? b >> 3 : b;
            long long RLn = (nj / 8) / KT + 1;  // lines per (workgroup, tile)
            long long ln = (long long)tile * ((long long)nbk * RLn + 3) + (long long)bb * RLn + cl % RLn;
            if (ln * 8 + 8 <= cap) recs[ln * 8 + (lane & 7)] = make_float4((float)j, 1.f, 2.f, 3.f);
            continue;
        }
        float4 v0 = make_float4((float)j, (float)t, 1.f, 2.f);
        if constexpr (MODE == 2) {
            asm volatile("" ::"v"(v0.x), "v"((int)slot));
        } else if constexpr (MODE == 4) {
            if (slot < cap / 2) {
                recs[slot] = v0;
                plane1[slot] = 3.f;
            }
        } else {
            // paired store: lanes 2i, 2i+1 write the halves of record i (32 lines / instr)
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                int src = half * 32 + (lane >> 1);
                long long s = __shfl(slot, src);
                float4 val = (lane & 1) ? make_float4(3.f, 0.f, 0.f, 0.f)
                                        : make_float4(__shfl(v0.x, src), __shfl(v0.y, src), 1.f, 2.f);
                if (2 * s + 2 <= cap) recs[2 * s + (lane & 1)] = val;
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
    if (hipMalloc(&d, (size_t)(N + (1 << 24)) * 32) != hipSuccess) return 1;
    if (hipMalloc(&p1, (size_t)(N + (1 << 24)) * 4) != hipSuccess) return 1;
    printf("K     B     recs      prod   coal   none   xcdord planes xcdreg pass1  line8r line8 (ms)\n");
    for (int B : {256, 512, 1024}) {
        for (int K : {1024, 2048, 4096, 8192}) {
            long long R = (N / B + K - 1) / K;
            float t0 = run<0>(d, p1, K, R, B);
            float t1 = run<1>(d, p1, K, R, B);
            float t2 = run<2>(d, p1, K, R, B);
            float t3 = run<3>(d, p1, K, R, B);
            float t4 = run<4>(d, p1, K, R, B);
            float t5 = run<5>(d, p1, K, R, B);
            float t6 = run<6>(d, p1, K, R, B);
            float t7 = run<7>(d, p1, K, R, B);
            float t8 = run<8>(d, p1, K, R, B);
            printf("%-5d %-5d %-9lld %6.3f %6.3f %6.3f %6.3f %6.3f %6.3f %6.3f %6.3f %6.3f\n", K, B, R * K * B, t0, t1, t2, t3, t4, t5, t6, t7, t8);
        }
    }
    return 0;
}
