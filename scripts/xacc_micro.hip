// Micro-benchmark: per-block column statistics delivered as (a) f64 partial rows (today's layout, folded by a
// later pass) or (b) exact fixed-point words added with no-return int64 atomics into S shards (no fold pass).
// Also times the consumer-side fold of S shards by NB blocks.  hipcc --offload-arch=gfx950 -O3 xacc_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ void split3(double v, long long& a, long long& b, long long& c) {
    const double f = floor(v);
    a = (long long)f;
    const double r1 = (v - f) * 4294967296.0;
    const double g = floor(r1);
    b = (long long)g;
    c = (long long)floor((r1 - g) * 4294967296.0);
}

// each block: a little streaming work (to space the blocks like a producer), then 2C column values
__global__ void prod_rows(const float* x, int64_t n_per_blk, int C2, double* part) {
    float acc = 0.f;
    for (int64_t i = threadIdx.x; i < n_per_blk; i += 256) acc += x[blockIdx.x * n_per_blk + i];
    for (int c = threadIdx.x; c < C2; c += 256) part[(int64_t)blockIdx.x * C2 + c] = (double)acc + c;
}
__global__ void prod_atom(const float* x, int64_t n_per_blk, int C2, int S, unsigned long long* acc3) {
    float acc = 0.f;
    for (int64_t i = threadIdx.x; i < n_per_blk; i += 256) acc += x[blockIdx.x * n_per_blk + i];
    unsigned long long* base = acc3 + (size_t)(blockIdx.x % S) * 3 * C2;
    for (int c = threadIdx.x; c < C2; c += 256) {
        long long a, b, d;
        split3((double)acc + c * 1.37, a, b, d);
        atomicAdd(base + c, (unsigned long long)a);
        atomicAdd(base + C2 + c, (unsigned long long)b);
        atomicAdd(base + 2 * C2 + c, (unsigned long long)d);
    }
}
__global__ void fold_rows(const double* part, int rows, int C2, float* out) {
    __shared__ double red[1024];
    for (int c = threadIdx.x; c < C2; c += 256) {
        double s = 0;
        for (int r = 0; r < rows; ++r) s += part[(int64_t)r * C2 + c];
        red[c & 1023] = s;
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < C2) out[threadIdx.x] = (float)red[threadIdx.x];
}
__global__ void fold_atom(const unsigned long long* acc3, int S, int C2, float* out) {
    __shared__ double red[1024];
    for (int c = threadIdx.x; c < C2; c += 256) {
        long long a = 0, b = 0, d = 0;
        for (int s = 0; s < S; ++s) {
            a += (long long)acc3[(size_t)s * 3 * C2 + c];
            b += (long long)acc3[(size_t)s * 3 * C2 + C2 + c];
            d += (long long)acc3[(size_t)s * 3 * C2 + 2 * C2 + c];
        }
        red[c & 1023] = (double)a + (double)b * 0x1p-32 + (double)d * 0x1p-64;
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < C2) out[threadIdx.x] = (float)red[threadIdx.x];
}

int main() {
    const int64_t NX = 64 << 20;
    float* x;
    double* part;
    unsigned long long* acc;
    float* out;
    CK(hipMalloc(&x, NX * 4));
    CK(hipMemset(x, 0, NX * 4));
    CK(hipMalloc(&part, 4096 * 1024 * 8));
    CK(hipMalloc(&acc, 64 * 3 * 1024 * 8));
    CK(hipMalloc(&out, 4096 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](auto launch) -> float {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(e0, 0);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        return ms * 1000.f / 20;
    };
    printf("producer: G blocks, 2C columns; rows = f64 partial rows; atom S = int64 x3 atomics into S shards (us)\n");
    for (int G : {256, 1024, 4096}) {
        const int64_t npb = (16 << 20) / G;  // 64 MB of x streamed in all
        for (int C : {32, 64, 256, 512}) {
            const int C2 = 2 * C;
            float tr = timed([&] { prod_rows<<<G, 256>>>(x, npb, C2, part); });
            printf("G %4d C %3d: rows %6.1f", G, C, tr);
            for (int S : {1, 4, 8, 16, 32}) {
                float ta = timed([&] { prod_atom<<<G, 256>>>(x, npb, C2, S, acc); });
                printf("  S%-2d %6.1f", S, ta);
            }
            printf("\n");
        }
    }
    printf("consumer fold: NB blocks each folding the table (us)\n");
    for (int NB : {256, 1024, 4096}) {
        for (int C : {32, 64, 256, 512}) {
            const int C2 = 2 * C;
            const int rows = 8 * (C <= 256 ? 256 / C : 1);
            float tr = timed([&] { fold_rows<<<NB, 256>>>(part, rows, C2, out); });
            printf("NB %4d C %3d: rows(%3d) %6.1f", NB, C, rows, tr);
            for (int S : {1, 4, 8, 16, 32}) {
                float ta = timed([&] { fold_atom<<<NB, 256>>>(acc, S, C2, out); });
                printf("  S%-2d %6.1f", S, ta);
            }
            printf("\n");
        }
    }
    printf("empty launch: %6.1f us\n", timed([&] { fold_atom<<<1, 64>>>(acc, 0, 2, out); }));
    return 0;
}
