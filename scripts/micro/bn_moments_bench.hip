// Micro-benchmark: BatchNorm-backward moments pass variants on the dec4 / dec3 shapes (bf16 [R][C]).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../hybrid-language-music-clustering-vae_amd/csrc bn_moments_bench.hip
// A: f64 accumulators + shuffle/LDS tail (as in kernels.hip)  B: f32 accumulators  C: f64, no math (loads + tail)
// D: f64, one partial row per thread group without shuffles (old LDS tail)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "common.hpp"
using namespace hlmc;

template <int V, typename Acc>
__device__ __forceinline__ void tail_shfl(Acc (&a)[V], int tpr, int C, Acc* lds, Acc* out) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int slot, cg, nslot; bool valid;
    if (tpr < 64) {
        for (int o = tpr; o < 64; o <<= 1)
#pragma unroll
            for (int v = 0; v < V; ++v) a[v] += __shfl_xor(a[v], o, 64);
        slot = w; cg = lane; valid = lane < tpr; nslot = 4;
    } else { slot = tid / tpr; cg = tid % tpr; valid = true; nslot = 256 / tpr; }
    if (valid)
#pragma unroll
        for (int v = 0; v < V; ++v) lds[slot * C + cg * V + v] = a[v];
    __syncthreads();
    for (int c = tid; c < C; c += 256) { Acc x = 0; for (int k = 0; k < nslot; ++k) x += lds[k * C + c]; out[c] = x; }
}
template <int V, typename Acc>
__device__ __forceinline__ void tail_lds(Acc (&a)[V], int tpr, int C, Acc* lds, Acc* out) {
    const int tid = threadIdx.x, cg = tid % tpr, rr = tid / tpr, rpp = 256 / tpr;
#pragma unroll
    for (int v = 0; v < V; ++v) lds[rr * C + cg * V + v] = a[v];
    __syncthreads();
    for (int c = tid; c < C; c += 256) { Acc x = 0; for (int k = 0; k < rpp; ++k) x += lds[k * C + c]; out[c] = x; }
}

template <typename Acc, int MODE>  // MODE 0 normal, 1 no math, 2 LDS tail
__global__ __launch_bounds__(256) void moments(const bf16* __restrict__ da, const bf16* __restrict__ y, int64_t R, int C,
                                               const float* __restrict__ mean, const float* __restrict__ invstd,
                                               int64_t rpb, Acc* __restrict__ part) {
    constexpr int V = 8, kUb = 4;
    __shared__ Acc s1[2048], s2[2048];
    const int tpr = C / V, rpp = 256 / tpr;
    const int tid = threadIdx.x, cg = tid % tpr, rr = tid / tpr, c0 = cg * V;
    const int64_t r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
    float mu[V], is[V];
    for (int v = 0; v < V; ++v) { mu[v] = mean[c0 + v]; is[v] = invstd[c0 + v]; }
    Acc a[V], b[V];
    for (int v = 0; v < V; ++v) a[v] = b[v] = 0;
    uint4 nx[kUb], ng[kUb];
    auto fetch = [&](int64_t rb) {
#pragma unroll
        for (int u = 0; u < kUb; ++u) {
            const int64_t rc = min(rb + u * rpp, r1 - 1);
            nx[u] = load16_raw(y + rc * C + c0);
            ng[u] = load16_raw(da + rc * C + c0);
        }
    };
    if (r0 + rr < r1) fetch(r0 + rr);
    for (int64_t r = r0 + rr; r < r1; r += kUb * rpp) {
        uint4 rx[kUb], rg[kUb];
#pragma unroll
        for (int u = 0; u < kUb; ++u) { rx[u] = nx[u]; rg[u] = ng[u]; }
        if (r + kUb * rpp < r1) fetch(r + kUb * rpp);
#pragma unroll
        for (int u = 0; u < kUb; ++u) {
            if (r + u * rpp >= r1) break;
            float x[V], g[V];
            cvt16_f32<bf16>(rx[u], x);
            cvt16_f32<bf16>(rg[u], g);
            if constexpr (MODE == 1) {
#pragma unroll
                for (int v = 0; v < V; ++v) { a[v] += x[v]; b[v] += g[v]; }
            } else {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    float xh = (x[v] - mu[v]) * is[v];
                    float dz = g[v] * (xh > 0.f ? 1.f : 0.01f);
                    a[v] += dz;
                    b[v] += (Acc)dz * xh;
                }
            }
        }
    }
    if constexpr (MODE == 2) {
        tail_lds<V, Acc>(a, tpr, C, s1, part + (int64_t)blockIdx.x * 2 * C);
        tail_lds<V, Acc>(b, tpr, C, s2, part + (int64_t)blockIdx.x * 2 * C + C);
    } else {
        tail_shfl<V, Acc>(a, tpr, C, s1, part + (int64_t)blockIdx.x * 2 * C);
        tail_shfl<V, Acc>(b, tpr, C, s2, part + (int64_t)blockIdx.x * 2 * C + C);
    }
}

template <typename Acc, int MODE>
float run(const bf16* da, const bf16* y, int64_t R, int C, const float* m, const float* is, void* part, int nblk_target) {
    int64_t step = 8192 / C, want = (R + nblk_target - 1) / nblk_target;
    int64_t rpb = (want + step - 1) / step * step;
    int nblk = (int)((R + rpb - 1) / rpb);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) moments<Acc, MODE><<<nblk, 256>>>(da, y, R, C, m, is, rpb, (Acc*)part);
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) moments<Acc, MODE><<<nblk, 256>>>(da, y, R, C, m, is, rpb, (Acc*)part);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 20 * 1e3f;
}

int main() {
    const int64_t maxe = 256LL * 64 * 64 * 32;
    bf16 *da, *y; float *m, *is; void* part;
    hipMalloc(&da, maxe * 2); hipMalloc(&y, maxe * 2); hipMalloc(&m, 4096); hipMalloc(&is, 4096); hipMalloc(&part, 64 << 20);
    hipMemset(da, 0x3c, maxe * 2); hipMemset(y, 0x3c, maxe * 2); hipMemset(m, 0, 4096); hipMemset(is, 0, 4096);
    struct S { int64_t R; int C; } shapes[] = {{256LL * 64 * 64, 32}, {256LL * 32 * 32, 64}, {256LL * 16 * 16, 128}, {256LL * 8 * 8, 256}};
    for (auto sh : shapes) {
        const double mb = sh.R * sh.C * 4.0 / 1e6;
        for (int nb : {1024, 4096}) {
            float tA = run<double, 0>(da, y, sh.R, sh.C, m, is, part, nb);
            float tB = run<float, 0>(da, y, sh.R, sh.C, m, is, part, nb);
            float tC = run<double, 1>(da, y, sh.R, sh.C, m, is, part, nb);
            float tD = run<double, 2>(da, y, sh.R, sh.C, m, is, part, nb);
            printf("R=%lld C=%d nblk~%d  MB=%.0f  A f64 %.1f us (%.0f GB/s)  B f32 %.1f  C nomath %.1f  D ldstail %.1f\n",
                   (long long)sh.R, sh.C, nb, mb, tA, mb * 1e3 / tA, tB, tC, tD);
        }
    }
    return 0;
}
