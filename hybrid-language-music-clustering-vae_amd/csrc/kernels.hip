// Memory-bound kernels of the VAE hot path: BatchNorm (train/eval) + activation fwd/bwd, the
// single-channel edge convolutions, layout changes, reparameterisation, loss, Adam, weight packing.
// Reductions are deterministic: fixed-size block partials in float64, summed in block order.
#include "ops.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <vector>
#include <atomic>

namespace hlmc {
namespace {

constexpr int kThreads = 256;
constexpr int kC1FusedBlocks = 1024;  // grid of the statistics-fused edge conv (accumulator contributions)
constexpr int kC1BwdBlocks = 768;     // the same as the output convT's data gradient with the BN-backward moments

inline int grid_for(int64_t n, int per_block = kThreads, int cap = 8192) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(cap, (n + per_block - 1) / per_block));
}

// Row-chunking shared by the [R][C] BatchNorm column reductions: each block streams one contiguous range of
// 8192 / C rows (16 KB of bf16, every thread's rows in flight at once) and emits one partial row.  (Measured:
// the former 1024-block cap left the wide-channel layers with 16-64 blocks, latency-bound at 5-20% of HBM.)
// <= 1024 blocks (about 4 per CU); each range is a multiple of 8192 / C rows (one 4-row-per-thread step for bf16)
// and the backward kernels prefetch the next step's rows into registers while reducing the current one.
// (round 3: 2048 / 512 within noise of 1024)
constexpr int kBnBlockTarget = 1024;
// block target of the wide-channel layers (C >= 128: each block's partial row costs 2C x 3 accumulator atomics and
// each apply block folds the shards of 2C columns, for 16-64 KB of rows per block at 1024 blocks).  Measured (3
// alternating rounds): 256 blocks 127.85k clips/s vs 126.76k at 1024, 127.1k at 512, 126.8k at 128, 127.6k at 384;
// the same target from C >= 64 127.4k, from C >= 256 127.4k
constexpr int kBnBlockTargetWide = 256;
inline int64_t bn_rows_per_blk(int64_t R, int C) {
    const int64_t step = std::max(1, 8192 / C);
    const int64_t tb = C >= 128 ? kBnBlockTargetWide : kBnBlockTarget;
    const int64_t want = std::max<int64_t>(1, (R + tb - 1) / tb);
    return (want + step - 1) / step * step;
}
inline int bn_blocks(int64_t R, int C) { return (int)((R + bn_rows_per_blk(R, C) - 1) / bn_rows_per_blk(R, C)); }

__device__ __forceinline__ float act_fwd(float z, int act) {
    if (act == 0) return z > 0.f ? z : 0.01f * z;
    if (act == 1) return z > 0.f ? z : 0.f;
    return z;
}
__device__ __forceinline__ float act_grad(float z, int act) {
    if (act == 0) return z > 0.f ? 1.f : 0.01f;
    if (act == 1) return z > 0.f ? 1.f : 0.f;
    return 1.f;
}
// ACT >= 0: the activation fixed at compile time (0 = LeakyReLU 0.01, the conv layers'), else the runtime `act`
template <int ACT>
__device__ __forceinline__ float act_grad_t(float z, int act) { return act_grad(z, ACT >= 0 ? ACT : act); }


// Column sums of per-thread V-channel accumulators across a 256-thread block whose thread t covers row
// rr = t / tpr, channel group cg = t % tpr (tpr = C / V, a power of two dividing 256).  Fixed order:
// xor-shuffle tree inside each wavefront over the lanes sharing cg, then the (<= 4) wave / row slots in LDS.
// The block's column totals go to the exact accumulator acc, columns coff + c (c < C).  lds: >= 256 * V doubles.
template <int V>
__device__ __forceinline__ void block_colsum(double (&a)[V], int tpr, int C, double* lds, const XAcc& acc, int coff) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int slot, cg, nslot;
    bool valid;
    if (tpr < 64) {
        for (int o = tpr; o < 64; o <<= 1)
#pragma unroll
            for (int v = 0; v < V; ++v) a[v] += __shfl_xor(a[v], o, 64);
        slot = w; cg = lane; valid = lane < tpr; nslot = 4;
    } else {
        slot = tid / tpr; cg = tid % tpr; valid = true; nslot = 256 / tpr;
    }
    if (valid)
#pragma unroll
        for (int v = 0; v < V; ++v) lds[slot * C + cg * V + v] = a[v];
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        double x = 0.0;
        for (int k = 0; k < nslot; ++k) x += lds[k * C + c];
        xacc_add(acc, coff + c, x);
    }
}

// Deterministic block reduction of per-block partials: part[k * stride + col] for k < nblk.
// Thread t sums k = t, t+256, ... in order; the 256 thread sums are combined by a fixed tree.
__device__ __forceinline__ double block_sum_partials(const double* __restrict__ part, int nblk, int64_t stride,
                                                     int64_t col, double* sh) {
    double s = 0.0;
    for (int k = threadIdx.x; k < nblk; k += blockDim.x) s += part[(int64_t)k * stride + col];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    double r = sh[0];
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------- BN statistics
// Column sums into the exact accumulator acc (2C columns): [0..C) = sum y, [C..2C) = sum y^2.
// Column-streaming kernels over a row-major [R][C] map: thread = (row lane rr, column group cg of V channels);
// a block pass covers rpp = 256 / (C/V) consecutive rows (one contiguous 4 KB span); each thread keeps its
// V channels' parameters in registers and has kU rows in flight.
constexpr int kU = 4;   // rows in flight, forward streaming kernels
constexpr int kUb = 2;  // backward (two operands per row, the next step's rows prefetched as well; 4 measured -0.6%)

template <typename T>
__global__ __launch_bounds__(256) void col_moments_kernel(const T* __restrict__ y, int64_t R, int C, int64_t rows_per_blk,
                                                          XAcc acc) {
    constexpr int V = Vec16<T>::N;
    __shared__ double s1[2048], s2[2048];
    const int tpr = C / V;                 // threads per row
    const int rpp = kThreads / tpr;        // rows per pass
    const int tid = threadIdx.x, cg = tid % tpr, rr = tid / tpr;
    const int64_t r0 = blockIdx.x * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
    double a[V], b[V];
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = b[v] = 0.0;
    const T* yp = y + cg * V;
    for (int64_t r = r0 + rr; r < r1; r += kU * rpp) {
        // every row load issued before any use: clamped (always in-bounds) rows, skipped below
        uint4 raw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) raw[u] = load16_raw(yp + min(r + u * rpp, r1 - 1) * C);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (r + u * rpp >= r1) break;
            float x[V];
            cvt16_f32<T>(raw[u], x);
#pragma unroll
            for (int v = 0; v < V; ++v) { a[v] += x[v]; b[v] += (double)x[v] * x[v]; }
        }
    }
    block_colsum<V>(a, tpr, C, s1, acc, 0);
    block_colsum<V>(b, tpr, C, s2, acc, C);
}

// ---------------------------------------------------------------- statistics finalize
// mean / invstd / running statistics from the exact accumulator (2C columns: sum | sum of squares); one thread per
// channel, grid ceil(C / 64) x 64 (the C > 512 layers, whose consumers do not finalize themselves)
__global__ __launch_bounds__(64) void bn_finalize_kernel(XAcc acc, int C, int64_t R, float* mean, float* invstd,
                                                         float* rmean, float* rvar, int64_t* nbt, float momentum,
                                                         float eps) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= C) return;
    // xacc_column masks the sticky non-finite flag (common.hpp kXAccBad): a diverged column comes out NaN
    const double s = xacc_column(acc, c), q = xacc_column(acc, C + c);
    if (c == 0 && nbt) nbt[0] += 1;
    const double m = s / (double)R;
    double var = q / (double)R - m * m;
    if (var < 0.0) var = 0.0;
    mean[c] = (float)m;
    invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (rmean) {
        const double unb = R > 1 ? var * (double)R / (double)(R - 1) : var;
        rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * m);
        rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
    }
}

__global__ void bn_eval_kernel(const float* rmean, const float* rvar, int C, float eps, float* mean, float* invstd) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    mean[c] = rmean[c];
    invstd[c] = 1.f / sqrtf(rvar[c] + eps);
}

// Consumer-side BatchNorm finalize: the streaming kernel that needs the per-channel statistics (bn_act: mean /
// invstd; bn_bwd_apply: sum dz / sum dz*xhat) reads the totals from the producer's exact accumulator itself
// (xacc_fold: shards x 6C int64 words) -- no finalize launch (every one costs >= 5 us on the critical path).
// Every block computes the same values; block 0 also stores the ones later kernels read (mean / invstd and the
// running statistics; dgamma / dbeta).
constexpr int kFinMaxC = 512;  // channels a consumer finalizes itself (LDS: 2 x 512 floats + 2 x 512 doubles)
struct BnFin {
    XAcc acc;                      // 2C columns
    int64_t R = 0;                 // rows of the normalised map (forward)
    float *mean = nullptr, *invstd = nullptr, *rmean = nullptr, *rvar = nullptr;  // forward outputs (block 0)
    int64_t* nbt = nullptr;
    float momentum = 0.f, eps = 0.f;
    float *dgamma = nullptr, *dbeta = nullptr;  // backward outputs (block 0)
};
// The per-channel values from the totals tot (LDS, 2C doubles): fwd mean / invstd, bwd sum dz / sum dz*xhat
template <bool kFwd>
__device__ __forceinline__ void bn_fin_values(const BnFin& f, const double* tot, int C, int c, float& x0, float& x1,
                                              double* var_out = nullptr) {
    const double s = tot[c], q = tot[C + c];
    if constexpr (kFwd) {
        const double m = s / (double)f.R;
        double var = q / (double)f.R - m * m;
        if (var < 0.0) var = 0.0;
        x0 = (float)m;
        x1 = (float)(1.0 / sqrt(var + (double)f.eps));
        if (var_out) *var_out = var;
    } else {
        x0 = (float)s;
        x1 = (float)q;
    }
}
// x0[c] / x1[c] (LDS floats, c < C) <- the per-channel values from the accumulator's totals (tot: LDS >= 2C
// doubles; red: LDS >= 3 * 256 int64, may not overlap tot); block 0 stores the finalized per-channel outputs.
// Ends with a barrier.
template <bool kFwd>
__device__ __forceinline__ void bn_fin_prologue(const BnFin& f, int C, double* tot, long long* red, float* x0s,
                                                float* x1s) {
    xacc_fold(f.acc, tot, red);
    for (int c = threadIdx.x; c < C; c += kThreads) {
        float x0, x1;
        double var = 0.0;
        bn_fin_values<kFwd>(f, tot, C, c, x0, x1, &var);
        x0s[c] = x0;
        x1s[c] = x1;
        if (blockIdx.x == 0) {
            if constexpr (kFwd) {
                f.mean[c] = x0;
                f.invstd[c] = x1;
                if (f.rmean) {
                    const double m = tot[c] / (double)f.R;
                    const double unb = f.R > 1 ? var * (double)f.R / (double)(f.R - 1) : var;
                    f.rmean[c] = (float)((1.0 - f.momentum) * f.rmean[c] + f.momentum * m);
                    f.rvar[c] = (float)((1.0 - f.momentum) * f.rvar[c] + f.momentum * unb);
                }
                if (c == 0 && f.nbt) f.nbt[0] += 1;
            } else {
                f.dbeta[c] = x0;
                f.dgamma[c] = x1;
            }
        }
    }
    __syncthreads();
}

struct BnChan {  // one thread's V channels of BatchNorm parameters
    template <int V>
    __device__ static void load(const float* __restrict__ src, int c0, float (&dst)[V]) {
#pragma unroll
        for (int v = 0; v < V; ++v) dst[v] = src[c0 + v];
    }
};

// a = act(gamma*(y-mean)*invstd + beta) [* mask * mscale]; grid-stride over row passes.
// kFin: train mode, mean / invstd folded here from the partial table (bn_fin_prologue).
template <typename T, bool kMask, bool kFin>
__global__ __launch_bounds__(256) void bn_act_kernel(const T* __restrict__ y, int64_t R, int C,
                                                     const float* __restrict__ mean, const float* __restrict__ invstd,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     int act, const uint8_t* __restrict__ mask, float mscale,
                                                     T* __restrict__ a, int lda, BnFin fin) {
    constexpr int V = Vec16<T>::N;
    __shared__ double fin_sh[kFin ? 2 * kFinMaxC + 3 * kThreads : 1];  // totals | fold scratch
    __shared__ float fin_x[kFin ? 2 * kFinMaxC : 1];                     // mean | invstd
    const int tpr = C / V, rpp = kThreads / tpr;
    const int tid = threadIdx.x, cg = tid % tpr, rr = tid / tpr;
    const int c0 = cg * V;
    const int64_t step = (int64_t)gridDim.x * rpp;
    const int64_t rfirst = (int64_t)blockIdx.x * rpp + rr;
    uint4 raw[kU];
    auto load_rows = [&](int64_t r) {
#pragma unroll
        for (int u = 0; u < kU; ++u) raw[u] = load16_raw(y + min(r + u * step, R - 1) * C + c0);
    };
    if (rfirst < R) load_rows(rfirst);  // the first pass's rows are in flight during the finalize prologue
    float mu[V], is[V], ga[V], be[V];
    if constexpr (kFin) {
        bn_fin_prologue<true>(fin, C, fin_sh, reinterpret_cast<long long*>(fin_sh + 2 * kFinMaxC), fin_x,
                              fin_x + kFinMaxC);
        BnChan::load(fin_x, c0, mu);
        BnChan::load(fin_x + kFinMaxC, c0, is);
    } else {
        BnChan::load(mean, c0, mu);
        BnChan::load(invstd, c0, is);
    }
    BnChan::load(gamma, c0, ga);
    BnChan::load(beta, c0, be);
    for (int64_t r = rfirst; r < R; r += kU * step) {
        if (r != rfirst) load_rows(r);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t ru = r + u * step;
            if (ru >= R) break;
            float x[V], o[V];
            cvt16_f32<T>(raw[u], x);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                float z = (x[v] - mu[v]) * is[v] * ga[v] + be[v];
                float t = act_fwd(z, act);
                if constexpr (kMask) t = mask[ru * C + c0 + v] ? t * mscale : 0.f;
                o[v] = t;
            }
            store16_f32(a + ru * lda + c0, o);
        }
    }
}

// backward partial sums: part[blk][0..C) = sum dz, [C..2C) = sum dz*xhat
// Rows past the block's range are clamped (always-valid addresses) and masked out of the sums, so every load is
// unconditional: a conditional prefetch leaves hipcc unable to count the loads younger than the ones it waits for
// at the top of the next step, and it waits for all of them (measured in the halo and GEMM loops).
template <typename T, bool kMask, int ACT = -1>
__global__ __launch_bounds__(256) void bn_bwd_moments_kernel(const T* __restrict__ da, int lda, const T* __restrict__ y,
                                                             int64_t R, int C, const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int act,
                                                             const uint8_t* __restrict__ mask, float mscale,
                                                             int64_t rows_per_blk, XAcc acc) {
    constexpr int V = Vec16<T>::N;
    __shared__ double s1[2048];
    const int tpr = C / V, rpp = kThreads / tpr;
    const int tid = threadIdx.x, cg = tid % tpr, rr = tid / tpr;
    const int c0 = cg * V;
    const int64_t r0 = blockIdx.x * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
    float mu[V], is[V], ga[V], be[V];
    BnChan::load(mean, c0, mu);
    BnChan::load(invstd, c0, is);
    BnChan::load(gamma, c0, ga);
    BnChan::load(beta, c0, be);
    // f32 per thread (rows_per_blk / rpp rows: 16 at the bench shapes, <= 128 at 128 x 1024 mel), f64 across
    // the block's threads and the blocks:
    // the lean register / LDS footprint lets more blocks share a CU with the weight-gradient GEMMs
    float a[V], b[V];
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = b[v] = 0.f;
    uint4 nx[kUb], ng[kUb];  // next step's rows (clamped, always in-bounds)
    auto fetch = [&](int64_t rb) {
#pragma unroll
        for (int u = 0; u < kUb; ++u) {
            const int64_t rc = min(rb + u * rpp, r1 - 1);
            nx[u] = load16_raw(y + rc * C + c0);
            ng[u] = load16_raw(da + rc * lda + c0);
        }
    };
    fetch(r0 + rr);
    for (int64_t r = r0 + rr; r < r1; r += kUb * rpp) {
        uint4 rx[kUb], rg[kUb];
#pragma unroll
        for (int u = 0; u < kUb; ++u) { rx[u] = nx[u]; rg[u] = ng[u]; }
        fetch(r + kUb * rpp);
#pragma unroll
        for (int u = 0; u < kUb; ++u) {
            const int64_t ru = r + u * rpp;
            const bool valid = ru < r1;
            float x[1][V], g[1][V];
            cvt16_f32<T>(rx[u], x[0]);
            cvt16_f32<T>(rg[u], g[0]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                float xh = (x[0][v] - mu[v]) * is[v];
                float z = xh * ga[v] + be[v];
                float dz = g[0][v] * act_grad_t<ACT>(z, act);
                if constexpr (kMask) dz = (valid && mask[ru * C + c0 + v]) ? dz * mscale : 0.f;
                dz = valid ? dz : 0.f;
                a[v] += dz;
                b[v] = fmaf(dz, xh, b[v]);
            }
        }
    }
    double da_[V], db_[V];
#pragma unroll
    for (int v = 0; v < V; ++v) { da_[v] = a[v]; db_[v] = b[v]; }
    block_colsum<V>(da_, tpr, C, s1, acc, 0);
    __syncthreads();   // s1 reused
    block_colsum<V>(db_, tpr, C, s1, acc, C);
}

// backward moments (2C columns): sum dz (-> dbeta), sum dz*xhat (-> dgamma); grid ceil(C / 64) x 64 (C > 512)
__global__ __launch_bounds__(64) void bn_bwd_finalize_kernel(XAcc acc, int C, float* dgamma, float* dbeta, float* sums_f) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= C) return;
    const double s = xacc_column(acc, c), q = xacc_column(acc, C + c);
    dbeta[c] = (float)s;
    dgamma[c] = (float)q;
    sums_f[c] = (float)s;
    sums_f[C + c] = (float)q;
}

// dy = gamma*invstd*(dz - sum_dz/R - xhat*sum_dzxh/R); also column partial sums of dy (bias grad)
// kFin: sum dz / sum dz*xhat folded here from the moments' partial table (bn_fin_prologue; block 0 stores
// dgamma / dbeta) instead of read from `sums`
// (unconditional clamped loads and stores: bn_bwd_moments_kernel; a clamped row's store rewrites the same value)
template <typename T, bool kMask, bool kFin, int ACT = -1>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ da, int lda, const T* __restrict__ y,
                                                           int64_t R, int C, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int act,
                                                           const uint8_t* __restrict__ mask, float mscale,
                                                           const float* __restrict__ sums, T* __restrict__ dy,
                                                           int64_t rows_per_blk, XAcc bias_acc, BnFin fin) {
    constexpr int V = Vec16<T>::N;
    __shared__ double s1[2048];
    const int tpr = C / V, rpp = kThreads / tpr;
    const int tid = threadIdx.x, cg = tid % tpr, rr = tid / tpr;
    const int c0 = cg * V;
    const int64_t r0 = blockIdx.x * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
    const float invR = 1.f / (float)R;
    float mu[V], is[V], ga[V], be[V], s0[V], sx[V];
    BnChan::load(mean, c0, mu);
    BnChan::load(invstd, c0, is);
    BnChan::load(gamma, c0, ga);
    BnChan::load(beta, c0, be);
    float a[V];   // f32 per thread, f64 across threads and blocks (see bn_bwd_moments_kernel)
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = 0.f;
    uint4 nx[kUb], ng[kUb];  // next step's rows (clamped, always in-bounds)
    auto fetch = [&](int64_t rb) {
#pragma unroll
        for (int u = 0; u < kUb; ++u) {
            const int64_t rc = min(rb + u * rpp, r1 - 1);
            nx[u] = load16_raw(y + rc * C + c0);
            ng[u] = load16_raw(da + rc * lda + c0);
        }
    };
    fetch(r0 + rr);  // in flight during the finalize prologue
    if constexpr (kFin) {
        // s1 is free until the closing block_colsum: totals in [0, 2C), the 2C sums as floats from 1024 (C
        // doubles), fold scratch after them (only used when 2C < 256: ends below 1024 + 64 + 768)
        float* xs = reinterpret_cast<float*>(s1 + 2 * kFinMaxC);
        bn_fin_prologue<false>(fin, C, s1, reinterpret_cast<long long*>(s1 + 2 * kFinMaxC + C), xs, xs + C);
        BnChan::load(xs, c0, s0);
        BnChan::load(xs + C, c0, sx);
        __syncthreads();  // every thread has its sums before block_colsum reuses s1
    } else {
        BnChan::load(sums, c0, s0);
        BnChan::load(sums + C, c0, sx);
    }
    for (int64_t r = r0 + rr; r < r1; r += kUb * rpp) {
        uint4 rx[kUb], rg[kUb];
#pragma unroll
        for (int u = 0; u < kUb; ++u) { rx[u] = nx[u]; rg[u] = ng[u]; }
        fetch(r + kUb * rpp);
#pragma unroll
        for (int u = 0; u < kUb; ++u) {
            const int64_t ru = r + u * rpp;
            const bool valid = ru < r1;
            const int64_t rc = valid ? ru : r1 - 1;  // the row whose inputs rx / rg hold (fetch clamps the same way)
            float x[1][V], g[1][V];
            cvt16_f32<T>(rx[u], x[0]);
            cvt16_f32<T>(rg[u], g[0]);
            float o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                float xh = (x[0][v] - mu[v]) * is[v];
                float z = xh * ga[v] + be[v];
                float dz = g[0][v] * act_grad_t<ACT>(z, act);
                if constexpr (kMask) dz = mask[rc * C + c0 + v] ? dz * mscale : 0.f;
                o[v] = ga[v] * is[v] * (dz - s0[v] * invR - xh * sx[v] * invR);
            }
            store16_f32(dy + rc * C + c0, o);
            // the bias grad is the sum of the dy actually stored (rounded to T), each row once
#pragma unroll
            for (int v = 0; v < V; ++v) a[v] += valid ? to_f32<T>(from_f32<T>(o[v])) : 0.f;
        }
    }
    if (bias_acc.on()) {
        double ad[V];
#pragma unroll
        for (int v = 0; v < V; ++v) ad[v] = a[v];
        block_colsum<V>(ad, tpr, C, s1, bias_acc, 0);
    }
}

// The whole BatchNorm backward of a SMALL layer (R <= 256 * kSmallRpt rows: the 4 x 4 / 2 x 2 conv maps and the
// BatchNorm1d layers) in one launch: block b owns the V channels c0 = b V of every row, each of its 256 threads
// holds its rows (r = t, t + 256, ...; <= kSmallRpt) of y and da in registers, so the moments are a block reduction
// (f32 per thread, f64 xor-tree over the wave, then the 4 waves in order) and the apply pass reuses the held rows:
// no accumulator atomics, no shard fold, no second read, one launch instead of two.  dgamma / dbeta written
// directly; the conv-bias column sums of the stored dy go into the exact accumulator (one add per column).
constexpr int kSmallRpt = 4;   // R <= 1024 (the 2 x 2 maps, BatchNorm1d at B <= 1024); at 16 rows per thread (4 x 4 maps) it lost to the two passes (34.8 vs 28.7 us)
template <int V>
__device__ __forceinline__ void block_sum_v(double (&x)[V], double (*lds)[V]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x[v] += __shfl_xor(x[v], o, 64);
    if (lane == 0)
#pragma unroll
        for (int v = 0; v < V; ++v) lds[w][v] = x[v];
    __syncthreads();
#pragma unroll
    for (int v = 0; v < V; ++v) x[v] = (lds[0][v] + lds[1][v]) + (lds[2][v] + lds[3][v]);
    __syncthreads();
}
template <typename T, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_small_kernel(const T* __restrict__ da, int lda, const T* __restrict__ y,
                                                           int R, int C, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int act, T* __restrict__ dy,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           XAcc bias_acc) {
    constexpr int V = Vec16<T>::N;
    __shared__ double red[4][V];
    const int c0 = blockIdx.x * V, t = threadIdx.x;
    float mu[V], is[V], ga[V], be[V];
    BnChan::load(mean, c0, mu);
    BnChan::load(invstd, c0, is);
    BnChan::load(gamma, c0, ga);
    BnChan::load(beta, c0, be);
    uint4 ry[kSmallRpt], rg[kSmallRpt];
#pragma unroll
    for (int i = 0; i < kSmallRpt; ++i) {  // every load issued up front (clamped rows, masked below)
        const int r = min(t + 256 * i, R - 1);
        ry[i] = load16_raw(y + (int64_t)r * C + c0);
        rg[i] = load16_raw(da + (int64_t)r * lda + c0);
    }
    float a[V], b[V];
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = b[v] = 0.f;
#pragma unroll
    for (int i = 0; i < kSmallRpt; ++i) {
        const bool ok = t + 256 * i < R;
        float x[V], g[V];
        cvt16_f32<T>(ry[i], x);
        cvt16_f32<T>(rg[i], g);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float xh = (x[v] - mu[v]) * is[v];
            const float dz = ok ? g[v] * act_grad_t<ACT>(xh * ga[v] + be[v], act) : 0.f;
            a[v] += dz;
            b[v] = fmaf(dz, xh, b[v]);
        }
    }
    double sa[V], sb[V];
#pragma unroll
    for (int v = 0; v < V; ++v) { sa[v] = a[v]; sb[v] = b[v]; }
    block_sum_v<V>(sa, red);
    block_sum_v<V>(sb, red);
    float s0[V], sx[V];
#pragma unroll
    for (int v = 0; v < V; ++v) { s0[v] = (float)sa[v]; sx[v] = (float)sb[v]; }
    if (t < V) {
        dbeta[c0 + t] = s0[t];
        dgamma[c0 + t] = sx[t];
    }
    const float invR = 1.f / (float)R;
    float bs[V];
#pragma unroll
    for (int v = 0; v < V; ++v) bs[v] = 0.f;
#pragma unroll
    for (int i = 0; i < kSmallRpt; ++i) {
        const int r = t + 256 * i;
        if (r >= R) break;
        float x[V], g[V], o[V];
        cvt16_f32<T>(ry[i], x);
        cvt16_f32<T>(rg[i], g);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float xh = (x[v] - mu[v]) * is[v];
            const float dz = g[v] * act_grad_t<ACT>(xh * ga[v] + be[v], act);
            o[v] = ga[v] * is[v] * (dz - s0[v] * invR - xh * sx[v] * invR);
        }
        store16_f32(dy + (int64_t)r * C + c0, o);
#pragma unroll
        for (int v = 0; v < V; ++v) bs[v] += to_f32<T>(from_f32<T>(o[v]));   // the stored dy, rounded to T
    }
    if (bias_acc.on()) {
        double sbias[V];
#pragma unroll
        for (int v = 0; v < V; ++v) sbias[v] = bs[v];
        block_sum_v<V>(sbias, red);
        if (t < V) xacc_add_shard(bias_acc, 0, c0 + t, sbias[t]);
    }
}

// The whole BatchNorm backward of a MID-SIZE layer (the 8 x 8 and 4 x 4 conv maps: R = 4 k - 16 k rows, C = 256 /
// 512; R * C <= kBnFusedMaxElems) in one launch with one grid-wide arrival count between the moments and the apply.  The two-pass form reads y
// and da twice over two launches whose blocks each fold the full 2C-column accumulator (6C x shards words) before
// their first row; here every block owns a channel slab (8 V channels: one 128-byte segment of each row) and kNR x 32
// rows, holds its rows of y and da in registers across the count, and adds / folds only its slab's 2 x 8V columns.
// Grid = slabs x row blocks, all co-resident (checked by the launcher against the occupancy query, with half of the
// chip left to grids co-running on the weight-gradient / comm streams), so every block reaches the count.  The spin
// is bounded (spin_max polls) so that a grid that could not become resident ends instead of hanging, and a block whose
// spin ran out is LOUD: its folded totals are replaced by NaN (its dgamma / dbeta / dy come out NaN, and so does every
// gradient below it) and it raises bit kDevBnCountTimeout of the library's device status word, which the next C-ABI
// backward call reports as HLMC_EDEVICE (hlmc_device_status).
// The arrival counter is the zeroed tail word of the moments accumulator (bn_acc_bytes).  Visibility follows the
// write-through hand-off form of the CDNA guide's Guideline 16 (every payload word written and read at the memory
// side, no L2 write-back fence): the payload is the accumulator's agent-scope atomic adds; every thread drains them
// (s_waitcnt vmcnt(0) with a memory clobber, so the compiler cannot sink an add below it) before the block's barrier
// and its one arrival add; one lane polls the counter relaxed; after the poll a wavefront-scope acquire fence keeps
// the fold's loads below it, and EVERY fold load is an agent-scope atomic load (sc1), never a plain load that could
// hit a stale L1 line.  (A per-block agent release + acquire, buffer_wbl2 + buffer_inv, measured 3.9x slower for
// the same kind of hand-off in round 2)
constexpr int kBnSpinMax = 1 << 22;   // polls of ~64 sleep cycles + one memory round trip each: ~2-4 s
constexpr int kBnFusedShards = 8;  // accumulator copies the fold reads (xacc_shards(C) <= 8 for C >= 128; checked)
template <typename T, int kNR, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_fused_kernel(const T* __restrict__ da, int lda, const T* __restrict__ y,
                                                           int R, int C, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int act, T* __restrict__ dy,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           XAcc mom, XAcc bias_acc, int nslab, int spin_max,
                                                           unsigned* status) {
    constexpr int V = Vec16<T>::N, SW = 8 * V;   // 8 threads x V channels per slab row segment
    __shared__ double red[4][2][SW];
    __shared__ double tot[2 * SW];
    __shared__ int timed_out;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, cg = t & 7, rr = t >> 3;
    const int slab = blockIdx.x % nslab, rb = blockIdx.x / nslab;
    const int c0 = slab * SW + cg * V;
    const int r0 = rb * (32 * kNR) + rr;
    uint4 hy[kNR], hg[kNR];
#pragma unroll
    for (int i = 0; i < kNR; ++i) {  // every row issued up front (clamped, masked below)
        const int r = min(r0 + 32 * i, R - 1);
        hy[i] = load16_raw(y + (int64_t)r * C + c0);
        hg[i] = load16_raw(da + (int64_t)r * lda + c0);
    }
    float mu[V], is[V], ga[V], be[V];
    BnChan::load(mean, c0, mu);
    BnChan::load(invstd, c0, is);
    BnChan::load(gamma, c0, ga);
    BnChan::load(beta, c0, be);
    float a[V], b[V];
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = b[v] = 0.f;
#pragma unroll
    for (int i = 0; i < kNR; ++i) {
        const bool ok = r0 + 32 * i < R;
        float x[V], g[V];
        cvt16_f32<T>(hy[i], x);
        cvt16_f32<T>(hg[i], g);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float xh = (x[v] - mu[v]) * is[v];
            float dz = g[v] * act_grad_t<ACT>(xh * ga[v] + be[v], act);
            dz = ok ? dz : 0.f;
            a[v] += dz;
            b[v] = fmaf(dz, xh, b[v]);
        }
    }
    // the apply pass recomputes x-hat / dz from the held raw rows: without this barrier to value propagation hipcc
    // keeps the 2 x V x kNR unpacked floats live across the count (232 VGPRs at kNR = 8)
#pragma unroll
    for (int i = 0; i < kNR; ++i) {
        asm volatile("" : "+v"(hy[i].x), "+v"(hy[i].y), "+v"(hy[i].z), "+v"(hy[i].w));
        asm volatile("" : "+v"(hg[i].x), "+v"(hg[i].y), "+v"(hg[i].z), "+v"(hg[i].w));
    }
    // block column sums (f32 per thread, f64 across): lanes sharing cg (xor 8, 16, 32), then the 4 waves in order
    auto slab_sums = [&](const float (&p)[V], const float (&q)[V], bool two) {
        double sp[V], sq[V];
#pragma unroll
        for (int v = 0; v < V; ++v) { sp[v] = p[v]; sq[v] = two ? q[v] : 0.0; }
#pragma unroll
        for (int o = 8; o < 64; o <<= 1)
#pragma unroll
            for (int v = 0; v < V; ++v) {
                sp[v] += __shfl_xor(sp[v], o, 64);
                if (two) sq[v] += __shfl_xor(sq[v], o, 64);
            }
        if (lane < 8)
#pragma unroll
            for (int v = 0; v < V; ++v) {
                red[w][0][lane * V + v] = sp[v];
                red[w][1][lane * V + v] = sq[v];
            }
        __syncthreads();
    };
    slab_sums(a, b, true);
    const int shard = rb % mom.shards;
    if (t < 2 * SW) {
        const int k = t / SW, j = t % SW;
        const double s = (red[0][k][j] + red[1][k][j]) + (red[2][k][j] + red[3][k][j]);
        xacc_add_shard(mom, shard, k * C + slab * SW + j, s);
    }
    // arrival: this thread's adds complete (drained), then one count per block; wait for all blocks of the grid
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* arrive = reinterpret_cast<unsigned*>(mom.p + (size_t)mom.shards * 3 * mom.ncols);
    if (t == 0) {
        __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned nblk = gridDim.x;
        int late = 1;
        for (int spin = 0; spin < spin_max; ++spin) {
            if (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nblk) {
                late = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (late && __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nblk) late = 0;
        if (late) __hip_atomic_store(status, kDevBnCountTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = late;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    const bool lost = timed_out != 0;
    // fold this slab's 2 x SW columns over the shards (agent-scope loads: the other XCDs' adds)
    if (t < 2 * SW) {
        const int k = t / SW, j = t % SW;
        const int col = k * C + slab * SW + j;
        // every shard's three words in flight at once (clamped shard index, masked adds): a shard loop waits one
        // memory-side round trip per shard
        unsigned long long w0[kBnFusedShards], w1[kBnFusedShards], w2[kBnFusedShards];
#pragma unroll
        for (int sh = 0; sh < kBnFusedShards; ++sh) {
            unsigned long long* q = mom.p + (size_t)min(sh, mom.shards - 1) * 3 * mom.ncols + col;
            w0[sh] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w1[sh] = __hip_atomic_load(q + mom.ncols, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w2[sh] = __hip_atomic_load(q + 2 * mom.ncols, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        long long s0w = 0, s1w = 0, s2w = 0;
        unsigned long long bad = 0;
#pragma unroll
        for (int sh = 0; sh < kBnFusedShards; ++sh)
            if (sh < mom.shards) {
                s0w += (long long)w0[sh];
                s1w += (long long)w1[sh];
                bad |= w2[sh] & kXAccBad;
                s2w += (long long)(w2[sh] & ~kXAccBad);
            }
        const double v = (bad || lost) ? __builtin_nan("") : xacc_value(s0w, s1w, s2w);
        tot[t] = v;
        if (rb == 0) (k == 0 ? dbeta : dgamma)[slab * SW + j] = (float)v;
    }
    __syncthreads();
    float s0[V], sx[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        s0[v] = (float)tot[cg * V + v];
        sx[v] = (float)tot[SW + cg * V + v];
    }
    const float invR = 1.f / (float)R;
    float bs[V];
#pragma unroll
    for (int v = 0; v < V; ++v) bs[v] = 0.f;
#pragma unroll
    for (int i = 0; i < kNR; ++i) {
        const int r = r0 + 32 * i;
        if (r >= R) break;
        float x[V], g[V], o[V];
        cvt16_f32<T>(hy[i], x);
        cvt16_f32<T>(hg[i], g);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float xh = (x[v] - mu[v]) * is[v];
            const float dz = g[v] * act_grad_t<ACT>(xh * ga[v] + be[v], act);
            o[v] = ga[v] * is[v] * (dz - s0[v] * invR - xh * sx[v] * invR);
        }
        store16_f32(dy + (int64_t)r * C + c0, o);
#pragma unroll
        for (int v = 0; v < V; ++v) bs[v] += to_f32<T>(from_f32<T>(o[v]));   // the stored dy, rounded to T
    }
    if (bias_acc.on()) {
        slab_sums(bs, bs, false);
        if (t < SW) {
            const double s = (red[0][0][t] + red[1][0][t]) + (red[2][0][t] + red[3][0][t]);
            xacc_add_shard(bias_acc, rb % bias_acc.shards, slab * SW + t, s);
        }
    }
}

// out[c] = column c of an exact accumulator (bias gradients); grid ceil(C / 64) x 64
__global__ __launch_bounds__(64) void xacc_to_f32_kernel(XAcc acc, int C, float* out) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c < C) out[c] = (float)xacc_column(acc, c);
}
__global__ __launch_bounds__(64) void xacc_to_f64_kernel(XAcc acc, int C, double* out) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c < C) out[c] = xacc_column(acc, c);
}

// sum over rows of column col of a [nrows][stride] table: 16 waves x 4 accumulators, LDS combine (1024 threads)
__device__ __forceinline__ double fold_column(const double* __restrict__ p, int nrows, int64_t stride, int col, bool ok,
                                              double (*sh)[64]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (ok) {
        int r = w;
        for (; r + 48 < nrows; r += 64) {
            a0 += p[(int64_t)r * stride + col];
            a1 += p[(int64_t)(r + 16) * stride + col];
            a2 += p[(int64_t)(r + 32) * stride + col];
            a3 += p[(int64_t)(r + 48) * stride + col];
        }
        for (; r < nrows; r += 16) a0 += p[(int64_t)r * stride + col];
    }
    sh[w][lane] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    double x = 0.0;
    for (int k = 0; k < 16; ++k) x += sh[k][lane];
    __syncthreads();
    return x;
}
// out[c] = sum_k part[k][c] over [nblk][C] partials (the generic colsum); grid ceil(C / 64) x 1024
__global__ __launch_bounds__(1024) void colsum_finalize_kernel(const double* __restrict__ part, int nblk, int C,
                                                               float* out) {
    __shared__ double sh[16][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const bool ok = c < C;
    const double s = fold_column(part, nblk, C, c, ok, sh);
    if (threadIdx.x < 64 && ok) out[c] = (float)s;
}

// Live-probe site of one BatchNorm-family launch (kind kBn, HBM-bound): algorithmic bytes = tensor bytes it
// must read + write (flops reported as 0)
#define HLMC_BN_PROBED(s, bytes, launch)                  \
    do {                                                  \
        probe::site(probe::kBn, 0.0, (double)(bytes));    \
        HLMC_PROBE_BEGIN(s);                              \
        launch;                                           \
        HLMC_PROBE_END(s);                                \
    } while (0)

inline unsigned fin_grid(int C) { return (unsigned)cdiv(C, 64); }

// generic column sum for arbitrary ld/cols (bias grads): block = (row chunk, 64-column slab);
// 4 waves split the chunk's rows, lanes own columns; fixed-order combine in LDS.
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ x, int ld, int rows, int cols,
                                                             int rows_per_blk, double* __restrict__ part) {
    __shared__ double red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y * 64 + lane;
    const int r0 = blockIdx.x * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
    double s = 0.0;
    if (c < cols)
        for (int r = r0 + w; r < r1; r += 4) s += to_f32<T>(x[(int64_t)r * ld + c]);
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && c < cols) part[(int64_t)blockIdx.x * cols + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// ---------------------------------------------------------------- edge convs (one channel side)
// y[b,oh,ow,co] = bias[co] + sum_{kh,kw} x[b, 2oh-1+kh, 2ow-1+kw] * w[co*9 + kh*3+kw]
// y[b, oh, ow, co] = bias[co] + sum_taps x[b, 2oh-1+kh, 2ow-1+kw] * w[co*9 + tap]  (1 input channel, CO = 32)
// Four threads per output pixel, each computing 8 channels (one 16-byte store): a wave's store instruction
// writes 1 KB contiguous; the 9 input taps are re-read by the 4 threads from L1.
// MODE 1 (encoder input conv): also the BatchNorm statistics of the stored outputs, [sum | sum of squares] into an
// exact accumulator (the col_moments pass it replaces).  MODE 2 (data gradient of the decoder's output
// convT, which writes the gradient of the last BatchNorm layer's output): also that layer's backward moments
// [sum dz | sum dz * xhat] (what bn_bwd_moments_kernel accumulates), with ybn / mean / invstd / gamma / beta of
// the layer (LeakyReLU 0.01).  Both: per-thread accumulators over the grid-stride pixels, block_colsum per block.
struct C1Fuse {
    XAcc acc;  // 2 CO columns
    const void* ybn = nullptr;
    const float *mean = nullptr, *invstd = nullptr, *gamma = nullptr, *beta = nullptr;
};
// Weights in LDS as [tap][CO] (each tap's 8 channels of a thread: two float4 reads), U = 2 pixels' tap loads in flight
// per step; launch bounds keep >= 4 waves per SIMD (the per-pixel register set is small: no weights in registers).
template <typename T, int CO, int MODE>
__global__ __launch_bounds__(256, MODE == 2 ? 3 : 4) void conv_c1_s2_kernel(const float* __restrict__ x, int B, int Hi, int Wi,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            T* __restrict__ y, FastDiv dWo, FastDiv dHo, C1Fuse fz) {
    constexpr int V = Vec16<T>::N, G = CO / V;  // threads per pixel
    constexpr int U = 2;                        // pixels per thread per step
    __shared__ __attribute__((aligned(16))) float wsh[9 * CO];
    __shared__ __attribute__((aligned(16))) float bsh[CO];
    __shared__ double fred[MODE ? 4 * CO : 1];
    for (int i = threadIdx.x; i < 9 * CO; i += blockDim.x) {
        const int tap = i / CO, c = i - tap * CO;
        wsh[i] = w[c * 9 + tap];
    }
    for (int i = threadIdx.x; i < CO; i += blockDim.x) bsh[i] = bias ? bias[i] : 0.f;
    // a thread's channel group is fixed (the grid stride is a multiple of G)
    const int c0 = (int)((blockIdx.x * blockDim.x + threadIdx.x) % G) * V;
    float fa[V], fb[V];  // per-thread statistics (a handful of pixels) in f32, widened once for the block tree
    float bmu[V], bis[V], bga[V], bbe[V];
#pragma unroll
    for (int v = 0; v < V; ++v) fa[v] = fb[v] = 0.f;
    if constexpr (MODE == 2) {
        BnChan::load(fz.mean, c0, bmu);
        BnChan::load(fz.invstd, c0, bis);
        BnChan::load(fz.gamma, c0, bga);
        BnChan::load(fz.beta, c0, bbe);
    }
    __syncthreads();
    const int Ho = Hi / 2, Wo = Wi / 2;
    const int nthr = B * Ho * Wo * G;  // < 2^31 (checked by the launcher)
    const int stride = gridDim.x * blockDim.x;
    for (int tb = blockIdx.x * blockDim.x + threadIdx.x; tb < nthr; tb += U * stride) {
        float in[U][9];
        int pix[U];
        uint4 yraw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every load of the U pixels issued before any use
            const int t0 = tb + u * stride;
            const bool ok = t0 < nthr;
            const int p = ok ? t0 / G : 0;
            pix[u] = ok ? p : -1;
            const int t = (int)dWo.div((uint32_t)p), ow = p - t * Wo;
            const int b = (int)dHo.div((uint32_t)t), oh = t - b * Ho;
            const float* xr = x + ((int64_t)b * Hi + 2 * oh - 1) * Wi + 2 * ow - 1;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
                    in[u][kh * 3 + kw] = (2 * oh - 1 + kh >= 0 && 2 * ow - 1 + kw >= 0) ? xr[kh * Wi + kw] : 0.f;
            if constexpr (MODE == 2) yraw[u] = load16_raw(static_cast<const T*>(fz.ybn) + (int64_t)p * CO + c0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (pix[u] < 0) break;
            float o[V];
#pragma unroll
            for (int v = 0; v < V; v += 4) {
                const float4 bq = *reinterpret_cast<const float4*>(bsh + c0 + v);
                o[v] = bq.x; o[v + 1] = bq.y; o[v + 2] = bq.z; o[v + 3] = bq.w;
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) {
#pragma unroll
                for (int v = 0; v < V; v += 4) {
                    const float4 wq = *reinterpret_cast<const float4*>(wsh + k * CO + c0 + v);
                    o[v] = fmaf(in[u][k], wq.x, o[v]);
                    o[v + 1] = fmaf(in[u][k], wq.y, o[v + 1]);
                    o[v + 2] = fmaf(in[u][k], wq.z, o[v + 2]);
                    o[v + 3] = fmaf(in[u][k], wq.w, o[v + 3]);
                }
            }
            store16_f32(y + (int64_t)pix[u] * CO + c0, o);
            if constexpr (MODE == 1) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const float q = to_f32<T>(from_f32<T>(o[v]));  // statistics of the stored values
                    fa[v] += q;
                    fb[v] = fmaf(q, q, fb[v]);
                }
            } else if constexpr (MODE == 2) {
                float xb[V];
                cvt16_f32<T>(yraw[u], xb);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const float g = to_f32<T>(from_f32<T>(o[v]));  // the stored gradient
                    const float xh = (xb[v] - bmu[v]) * bis[v];
                    const float dz = g * (xh * bga[v] + bbe[v] > 0.f ? 1.f : 0.01f);
                    fa[v] += dz;
                    fb[v] = fmaf(dz, xh, fb[v]);
                }
            }
        }
    }
    if constexpr (MODE != 0) {
        double da_[V], db_[V];
#pragma unroll
        for (int v = 0; v < V; ++v) { da_[v] = fa[v]; db_[v] = fb[v]; }
        block_colsum<V>(da_, G, CO, fred, fz.acc, 0);
        __syncthreads();
        block_colsum<V>(db_, G, CO, fred, fz.acc, CO);
    }
}

// y[b, oh, ow] = bias + sum_ci sum_taps x[b, ih, iw, ci] * w[ci*9 + kh*3 + kw]  (transposed, 1 output channel).
// One thread per LOW-RES pixel (r, c) computes its 2 x 2 output block (2r + py, 2c + px): the block reads exactly
// the 2 x 2 low-res neighbourhood (r..r+1, c..c+1; zero past the image), all of it loaded up front (16 16-byte
// loads for bf16), and uses each of the 9 taps once: (py, px; dy, dx) -> (kh, kw) with kh = 1 for py = 0, else
// 0 (dy = 1) / 2 (dy = 0); kw likewise.  Weights sit in LDS as [tap][ci] and are read as float4 broadcasts; each
// output keeps two accumulators (even / odd channel chunks) to halve its FMA chain.  Stores: two float2 rows.
// (Supersedes one thread per output pixel, whose per-tap loads waited one round trip each: 47 us at B = 256.)
// (launch bounds: >= 4 waves per SIMD; unbounded, hipcc hoisted every LDS weight read out of the pixel loop into
// 450 registers -> one wave per SIMD)
template <typename T, int CI>
__global__ __launch_bounds__(256, 4) void convT_c1_kernel(const T* __restrict__ x, int B, int Hi, int Wi,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       float* __restrict__ y, FastDiv dWi, FastDiv dHi) {
    constexpr int V = Vec16<T>::N, NC = CI / V;  // 16-byte chunks per pixel
    __shared__ __attribute__((aligned(16))) float wt[9 * CI];
    for (int i = threadIdx.x; i < 9 * CI; i += blockDim.x) {
        const int tap = i / CI, ci = i - tap * CI;
        wt[i] = w[ci * 9 + tap];
    }
    __syncthreads();
    const float b0 = bias ? bias[0] : 0.f;
    const int Ho = 2 * Hi, Wo = 2 * Wi;
    const int nlow = B * Hi * Wi;  // < 2^31 (checked by the launcher)
    // (out = py * 2 + px, neighbour n = dy * 2 + dx, tap) for the 9 contributions of a 2 x 2 block
    constexpr int kOut[9] = {0, 1, 1, 2, 2, 3, 3, 3, 3};
    constexpr int kNb[9] = {0, 0, 1, 0, 2, 0, 1, 2, 3};
    constexpr int kTap[9] = {4, 5, 3, 7, 1, 8, 6, 2, 0};
    // one low-res pixel per thread, no grid-stride loop: nothing is loop-invariant for hipcc to hoist into registers
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nlow) {
        const int t = (int)dWi.div((uint32_t)q), c = q - t * Wi;
        const int b = (int)dHi.div((uint32_t)t), r = t - b * Hi;
        const bool okr = r + 1 < Hi, okc = c + 1 < Wi;
        const T* p00 = x + (int64_t)q * CI;
        const T* nbp[4] = {p00, okc ? p00 + CI : p00, okr ? p00 + (int64_t)Wi * CI : p00,
                           (okr && okc) ? p00 + (int64_t)(Wi + 1) * CI : p00};
        const bool nbok[4] = {true, okc, okr, okr && okc};
        uint4 raw[4][NC];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < NC; ++j) raw[n][j] = load16_raw(nbp[n] + j * V);
        float acc[4][2];
#pragma unroll
        for (int o = 0; o < 4; ++o) { acc[o][0] = b0; acc[o][1] = 0.f; }
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            float v[4][V];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                cvt16_f32<T>(raw[n][j], v[n]);
#pragma unroll
                for (int e = 0; e < V; ++e) v[n][e] = nbok[n] ? v[n][e] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const float4* wp = reinterpret_cast<const float4*>(wt + kTap[k] * CI + j * V);
#pragma unroll
                for (int e4 = 0; e4 < V / 4; ++e4) {
                    const float4 wq = wp[e4];
                    float& a = acc[kOut[k]][j & 1];
                    a = fmaf(v[kNb[k]][4 * e4 + 0], wq.x, a);
                    a = fmaf(v[kNb[k]][4 * e4 + 1], wq.y, a);
                    a = fmaf(v[kNb[k]][4 * e4 + 2], wq.z, a);
                    a = fmaf(v[kNb[k]][4 * e4 + 3], wq.w, a);
                }
            }
        }
        float* o0 = y + ((int64_t)b * Ho + 2 * r) * Wo + 2 * c;
        *reinterpret_cast<float2*>(o0) = make_float2(acc[0][0] + acc[0][1], acc[1][0] + acc[1][1]);
        *reinterpret_cast<float2*>(o0 + Wo) = make_float2(acc[2][0] + acc[2][1], acc[3][0] + acc[3][1]);
    }
}

// dW[m*9+tap] partials: block = chunk of low-res rows (b,r,c); Xh single-channel high-res [B, 2Hl, 2Wl].
// Thread (row group rg = tid / 8, channel group cg = tid % 8) accumulates a 4 (m) x 9 (tap) register block over
// rows k0 + rg, k0 + rg + 32, ... straight from global memory: per row 4 channels of L (8 bytes for bf16; a wave
// reads 8 whole 64-byte rows) and the row's 9 high-res taps (L1-shared by the 8 channel groups), U rows' loads
// in flight per step.  The 32 row groups are combined in LDS in a fixed order.  (Supersedes 256-row LDS stages
// with a barrier each: 45 us at B = 256.)
template <typename T, int M>
__global__ __launch_bounds__(256, 4) void wgrad_c1_kernel(const T* __restrict__ L, int B, int Hl, int Wl,
                                                       const float* __restrict__ Xh, int rows_per_blk,
                                                       float* __restrict__ part, FastDiv dWl, FastDiv dHl) {
    static_assert(M == 32, "8 channel groups of 4");
    constexpr int U = 4;
    __shared__ float red[32][M * 9 + 1];
    const int64_t K = (int64_t)B * Hl * Wl;
    const int64_t k0 = (int64_t)blockIdx.x * rows_per_blk, k1 = min(K, k0 + rows_per_blk);
    const int Hh = 2 * Hl, Wh = 2 * Wl;
    const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
    float acc[4][9];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) acc[i][j] = 0.f;
    for (int64_t kb = k0 + rg; kb < k1; kb += 32 * U) {
        float l[U][4], h[U][9];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every load of the U rows issued before any use
            const int64_t k = kb + 32 * u;
            const bool ok = k < k1;
            const int kk = ok ? (int)k : (int)k0;
            if constexpr (sizeof(T) == 2) {
                const uint2 raw = *reinterpret_cast<const uint2*>(L + (int64_t)kk * M + 4 * cg);
                l[u][0] = __uint_as_float(raw.x << 16);
                l[u][1] = __uint_as_float(raw.x & 0xffff0000u);
                l[u][2] = __uint_as_float(raw.y << 16);
                l[u][3] = __uint_as_float(raw.y & 0xffff0000u);
            } else {
                const float4 raw = *reinterpret_cast<const float4*>(L + (int64_t)kk * M + 4 * cg);
                l[u][0] = raw.x; l[u][1] = raw.y; l[u][2] = raw.z; l[u][3] = raw.w;
            }
            const int t = (int)dWl.div((uint32_t)kk), c = kk - t * Wl;
            const int b = (int)dHl.div((uint32_t)t), r = t - b * Hl;
            const float* xr = Xh + ((int64_t)b * Hh + 2 * r - 1) * Wh + 2 * c - 1;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int kh = tap / 3, kw = tap % 3;
                h[u][tap] = (ok && 2 * r - 1 + kh >= 0 && 2 * c - 1 + kw >= 0) ? xr[kh * Wh + kw] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 9; ++j) acc[i][j] = fmaf(l[u][i], h[u][j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) red[rg][(4 * cg + i) * 9 + j] = acc[i][j];
    __syncthreads();
    for (int o = threadIdx.x; o < M * 9; o += blockDim.x) {
        float v = 0.f;
        for (int g = 0; g < 32; ++g) v += red[g][o];
        part[(int64_t)blockIdx.x * (M * 9) + o] = v;
    }
}

// The same weight gradient for the 64-wide layers (every use in the model), streamed by low-res ROWS: thread
// (pixel c = tid / 4, channel group cg = tid % 4) of a block takes U rows per step with every load of the U rows
// issued up front -- its 8 channels of L (one 16-byte load) and its 3 x 3 high-res taps as 6 float2 loads (columns
// 2c-2 .. 2c+1 of rows 2r-1 .. 2r+1; the 4 channel groups of a pixel share the lines in L1) -- so a block keeps
// U rows of loads in flight with no barrier in the loop.  acc[8 channels][9 taps] per thread; at the end lanes of
// equal cg are summed with xor shuffles over the wave's 16 pixels, then the 4 waves in LDS, in a fixed order ->
// part[block][co * 9 + tap] (sum_partials_f32_kernel adds the blocks).
template <typename T>
__global__ __launch_bounds__(256, 2) void wgrad_c1_rows_kernel(const T* __restrict__ L, int rows, int Hl,
                                                             const float* __restrict__ Xh, float* __restrict__ part) {
    constexpr int WL = 64, WH = 128, M = 32, U = 4;
    __shared__ float red[4][4][8 * 9];
    const int tid = threadIdx.x, c = tid >> 2, cg = tid & 3, lane = tid & 63, wave = tid >> 6;
    float acc[8][9];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) acc[i][j] = 0.f;
    const int stride = gridDim.x;
    for (int r0 = blockIdx.x; r0 < rows; r0 += U * stride) {
        float lv[U][8], xv[U][3][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every load of the U rows issued before any use (rows past the end: row 0)
            const int row = r0 + u * stride < rows ? r0 + u * stride : 0;
            const T* lp = L + ((int64_t)row * WL + c) * M + 8 * cg;
            if constexpr (sizeof(T) == 2) {
                cvt16_f32<T>(*reinterpret_cast<const uint4*>(lp), lv[u]);
            } else {
                const float4 a = *reinterpret_cast<const float4*>(lp), b = *reinterpret_cast<const float4*>(lp + 4);
                lv[u][0] = a.x; lv[u][1] = a.y; lv[u][2] = a.z; lv[u][3] = a.w;
                lv[u][4] = b.x; lv[u][5] = b.y; lv[u][6] = b.z; lv[u][7] = b.w;
            }
            const int b = row / Hl, r = row - b * Hl;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                const int ih = 2 * r - 1 + kh;
                const float* xr = Xh + ((int64_t)b * 2 * Hl + (ih < 0 ? 0 : ih)) * WH + 2 * c;
                const float2 lo = *reinterpret_cast<const float2*>(xr - (c > 0 ? 2 : 0));   // columns 2c-2, 2c-1
                const float2 hi = *reinterpret_cast<const float2*>(xr);                     // columns 2c, 2c+1
                const bool okr = ih >= 0;
                xv[u][kh][0] = (okr && c > 0) ? lo.y : 0.f;   // column 2c - 1 (left padding at c = 0)
                xv[u][kh][1] = okr ? hi.x : 0.f;
                xv[u][kh][2] = okr ? hi.y : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float m = r0 + u * stride < rows ? 1.f : 0.f;   // rows past the end add zero
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float l = lv[u][i] * m;
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) acc[i][kh * 3 + kw] = fmaf(l, xv[u][kh][kw], acc[i][kh * 3 + kw]);
            }
        }
    }
    // lanes 4 p + cg of a wave: sum over the 16 pixels p (xor over lane bits 2..5), fixed order
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            float v = acc[i][j];
#pragma unroll
            for (int o = 4; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
            acc[i][j] = v;
        }
    if (lane < 4) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 9; ++j) red[wave][lane][i * 9 + j] = acc[i][j];
    }
    __syncthreads();
    for (int o = tid; o < M * 9; o += 256) {
        const int co = o / 9, tap = o - co * 9, g = co >> 3, i = co & 7;
        const float v = (red[0][g][i * 9 + tap] + red[1][g][i * 9 + tap]) + (red[2][g][i * 9 + tap] + red[3][g][i * 9 + tap]);
        part[(int64_t)blockIdx.x * (M * 9) + o] = v;
    }
}

__global__ __launch_bounds__(256) void sum_partials_f32_kernel(const float* __restrict__ part, int nblk, int n,
                                                               float* out) {
    __shared__ double sh[256];
    const int i = blockIdx.x;
    double s = 0.0;
    for (int k = threadIdx.x; k < nblk; k += blockDim.x) s += part[(int64_t)k * n + i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[i] = (float)sh[0];
}

// ---------------------------------------------------------------- layout / elementwise
template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = from_f32<TO>(to_f32<TI>(x[i]));
}
template <typename TI, typename TO>
__global__ void cast2d_kernel(const TI* __restrict__ x, int ldx, TO* __restrict__ y, int ldy, int rows, int cols) {
    int64_t n = (int64_t)rows * cols;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int r = (int)(i / cols), c = (int)(i % cols);
        y[(int64_t)r * ldy + c] = from_f32<TO>(to_f32<TI>(x[(int64_t)r * ldx + c]));
    }
}
template <typename T>
__global__ void nhwc_to_flat_kernel(const T* __restrict__ x, int B, int h, int w, int C, T* __restrict__ y, int ldy,
                                    const T* __restrict__ relu_ref) {
    const int F = C * h * w;
    int64_t n = (int64_t)B * F;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int b = (int)(i / F), f = (int)(i % F);
        int c = f / (h * w), hw = f % (h * w);
        const int64_t o = (int64_t)b * ldy + f;
        T v = x[((int64_t)b * h * w + hw) * C + c];
        if (relu_ref && !(to_f32<T>(relu_ref[o]) > 0.f)) v = from_f32<T>(0.f);
        y[o] = v;
    }
}
template <typename T>
__global__ void flat_to_nhwc_kernel(const T* __restrict__ x, int ldx, int B, int h, int w, int C, T* __restrict__ y) {
    const int F = C * h * w;
    int64_t n = (int64_t)B * F;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int b = (int)(i / F), rem = (int)(i % F);
        int hw = rem / C, c = rem % C;  // i enumerates the NHWC output
        y[i] = x[(int64_t)b * ldx + (int64_t)c * h * w + hw];
    }
}
// optional copies a reparameterisation launch also writes: the caller's mu / logvar outputs and (host-supplied eps)
// the eps the backward keeps -- one launch instead of a copy launch plus the reparameterisation
struct LatentOut {
    float* mu = nullptr;
    float* lv = nullptr;
    float* eps = nullptr;
};
template <typename T>
__global__ void reparam_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                   const float* __restrict__ eps, int n_rows, int L, T* __restrict__ z, int ldz,
                                   LatentOut lo) {
    int64_t n = (int64_t)n_rows * L;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int r = (int)(i / L), c = (int)(i % L);
        const float m = mu[i], l = lv[i], e = eps[i];
        float sd = expf(0.5f * l);
        z[(int64_t)r * ldz + c] = from_f32<T>(m + e * sd);
        if (lo.mu) lo.mu[i] = m;
        if (lo.lv) lo.lv[i] = l;
        if (lo.eps) lo.eps[i] = e;
    }
}
// ---------------------------------------------------------------- reparameterisation noise (Philox4x32-10)
// eps ~ N(0, 1) drawn on the device instead of a host/torch launch: element g = offset + i of the (seed) stream is
// component g % 4 of Philox4x32-10(counter = {g / 4 (64 bits), 0, 0}, key = seed) (Salmon et al., SC'11: 10 rounds,
// multipliers 0xD2511F53 / 0xCD9E8D57, key bumps 0x9E3779B9 / 0xBB67AE85), the 4 words mapped to 2 Box-Muller
// pairs: u1 = (w0 + 1) 2^-32 in (0, 1], u2 = w1 2^-32, n0 = sqrt(-2 ln u1) cos(2 pi u2), n1 = ... sin(2 pi u2).
// Counter-based, so any element is computed independently (no generator state on the device).
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
__device__ __forceinline__ void philox_normal4(uint64_t seed, uint64_t q, float (&n)[4]) {
    const uint4 w = philox4x32_10(make_uint4((uint32_t)q, (uint32_t)(q >> 32), 0u, 0u), (uint32_t)seed,
                                  (uint32_t)(seed >> 32));
    const float k = 2.3283064365386963e-10f;  // 2^-32
    const float r0 = sqrtf(-2.f * logf(((float)w.x + 1.f) * k)), a0 = 6.283185307179586f * ((float)w.y * k);
    const float r1 = sqrtf(-2.f * logf(((float)w.z + 1.f) * k)), a1 = 6.283185307179586f * ((float)w.w * k);
    n[0] = r0 * cosf(a0);
    n[1] = r0 * sinf(a0);
    n[2] = r1 * cosf(a1);
    n[3] = r1 * sinf(a1);
}
// out[i] = element offset + i of the stream (offset % 4 == 0): one thread per group of 4
__global__ void randn_kernel(float* __restrict__ out, int64_t n, uint64_t seed, uint64_t offset) {
    const int64_t groups = (n + 3) / 4;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < groups; t += (int64_t)gridDim.x * blockDim.x) {
        float v[4];
        philox_normal4(seed, offset / 4 + t, v);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * t + j < n) out[4 * t + j] = v[j];
    }
}
// z = mu + eps * exp(0.5 lv) with eps drawn here (element i of the [n_rows][L] block = stream element offset + i)
// and stored to eps_out for the backward pass
template <typename T>
__global__ void reparam_rng_kernel(const float* __restrict__ mu, const float* __restrict__ lv, uint64_t seed,
                                   uint64_t offset, int n_rows, int L, float* __restrict__ eps_out, T* __restrict__ z,
                                   int ldz, LatentOut lo) {
    const int64_t n = (int64_t)n_rows * L, groups = (n + 3) / 4;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < groups; t += (int64_t)gridDim.x * blockDim.x) {
        float v[4];
        philox_normal4(seed, offset / 4 + t, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t i = 4 * t + j;
            if (i >= n) break;
            const int r = (int)(i / L), c = (int)(i - (int64_t)r * L);
            const float m = mu[i], l = lv[i];
            eps_out[i] = v[j];
            z[(int64_t)r * ldz + c] = from_f32<T>(m + v[j] * expf(0.5f * l));
            if (lo.mu) lo.mu[i] = m;
            if (lo.lv) lo.lv[i] = l;
        }
    }
}

template <typename T>
__global__ void reparam_bwd_kernel(const T* __restrict__ dz, int lddz, const float* __restrict__ lv,
                                   const float* __restrict__ eps, const float* __restrict__ d_mu,
                                   const float* __restrict__ d_lv, int n_rows, int L, T* __restrict__ gmu,
                                   T* __restrict__ glv) {
    int64_t n = (int64_t)n_rows * L;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int r = (int)(i / L), c = (int)(i % L);
        float g = to_f32<T>(dz[(int64_t)r * lddz + c]);
        float sd = expf(0.5f * lv[i]);
        gmu[i] = from_f32<T>((d_mu ? d_mu[i] : 0.f) + g);
        glv[i] = from_f32<T>((d_lv ? d_lv[i] : 0.f) + g * eps[i] * sd * 0.5f);
    }
}

// ---------------------------------------------------------------- loss
__global__ __launch_bounds__(256) void vae_sums_kernel(const float* __restrict__ ra, const float* __restrict__ a,
                                                       int64_t na, const float* __restrict__ rt,
                                                       const float* __restrict__ t, int64_t nt,
                                                       const float* __restrict__ mu, const float* __restrict__ lv,
                                                       int64_t nl, double* __restrict__ part) {
    __shared__ double red[3][4];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < na; i += stride) { float d = ra[i] - a[i]; s0 += (double)d * d; }
    for (int64_t i = i0; i < nt; i += stride) { float d = rt[i] - t[i]; s1 += (double)d * d; }
    for (int64_t i = i0; i < nl; i += stride) s2 += (double)(1.f + lv[i] - mu[i] * mu[i] - expf(lv[i]));
    s0 = wave_sum(s0); s1 = wave_sum(s1); s2 = wave_sum(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = s0; red[1][w] = s1; red[2][w] = s2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double s = 0.0;
        for (int k = 0; k < 4; ++k) s += red[threadIdx.x][k];
        part[blockIdx.x * 3 + threadIdx.x] = s;
    }
}
// loss sums and their gradient in one pass over (ra, a), (rt, t), (mu, lv): vae_sums_kernel's partial rows plus
// vae_bwd_kernel's outputs (the gradient does not depend on the sums: d ra = ca (ra - a), ...)
__global__ __launch_bounds__(256) void vae_sums_bwd_kernel(const float* __restrict__ ra, const float* __restrict__ a,
                                                           int64_t na, float* __restrict__ dra,
                                                           const float* __restrict__ rt, const float* __restrict__ t,
                                                           int64_t nt, float* __restrict__ drt,
                                                           const float* __restrict__ mu, const float* __restrict__ lv,
                                                           int64_t nl, const float* __restrict__ coef,
                                                           float* __restrict__ dmu, float* __restrict__ dlv,
                                                           double* __restrict__ part) {
    __shared__ double red[3][4];
    const float ca = coef[0], ct = coef[1], ck = coef[2];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < na; i += stride) {
        const float d = ra[i] - a[i];
        s0 += (double)d * d;
        dra[i] = ca * d;
    }
    for (int64_t i = i0; i < nt; i += stride) {
        const float d = rt[i] - t[i];
        s1 += (double)d * d;
        drt[i] = ct * d;
    }
    for (int64_t i = i0; i < nl; i += stride) {
        const float e = expf(lv[i]);
        s2 += (double)(1.f + lv[i] - mu[i] * mu[i] - e);
        dmu[i] = ck * mu[i];
        dlv[i] = -0.5f * ck * (1.f - e);
    }
    s0 = wave_sum(s0); s1 = wave_sum(s1); s2 = wave_sum(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = s0; red[1][w] = s1; red[2][w] = s2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double s = 0.0;
        for (int k = 0; k < 4; ++k) s += red[threadIdx.x][k];
        part[blockIdx.x * 3 + threadIdx.x] = s;
    }
}
__global__ __launch_bounds__(256) void vae_sums_finalize_kernel(const double* __restrict__ part, int nblk, double* out) {
    __shared__ double sh[256];
    const int j = blockIdx.x;
    const double s = block_sum_partials(part, nblk, 3, j, sh);
    if (threadIdx.x == 0) out[j] = s;
}
__global__ void vae_bwd_kernel(const float* __restrict__ ra, const float* __restrict__ a, int64_t na,
                               float* __restrict__ dra, const float* __restrict__ rt, const float* __restrict__ t,
                               int64_t nt, float* __restrict__ drt, const float* __restrict__ mu,
                               const float* __restrict__ lv, int64_t nl, const float* __restrict__ coef,
                               float* __restrict__ dmu, float* __restrict__ dlv) {
    const float ca = coef[0], ct = coef[1], ck = coef[2];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < na; i += stride) dra[i] = ca * (ra[i] - a[i]);
    for (int64_t i = i0; i < nt; i += stride) drt[i] = ct * (rt[i] - t[i]);
    for (int64_t i = i0; i < nl; i += stride) {
        dmu[i] = ck * mu[i];
        dlv[i] = -0.5f * ck * (1.f - expf(lv[i]));
    }
}

// ---------------------------------------------------------------- Adam (torch.optim.Adam single-tensor math)
constexpr int kAdamMax = 32;
struct AdamBatch {
    float* p[kAdamMax];
    const float* g[kAdamMax];
    float* m[kAdamMax];
    float* v[kAdamMax];
    int64_t n[kAdamMax];
    int blk0[kAdamMax + 1];
    int count;
};
struct AdamCoef {
    float b1, b2, eps, wd, step_size, bc2_sqrt;
};
// one element of torch.optim.Adam (foreach=False, amsgrad=False, maximize=False) on values: p, m, v updated
__device__ __forceinline__ void adam_val(float& p, float g, float& m, float& v, const AdamCoef& c) {
#pragma clang fp contract(off)  // identical rounding in every kernel that inlines this (no FMA contraction)
    float gi = g;
    const float pi = p;
    if (c.wd != 0.f) gi = gi + c.wd * pi;
    float mi = m;
    mi = mi + (gi - mi) * (1.f - c.b1);
    const float vi = v * c.b2 + (1.f - c.b2) * gi * gi;
    m = mi;
    v = vi;
    const float denom = sqrtf(vi) / c.bc2_sqrt + c.eps;
    p = pi - c.step_size * (mi / denom);
}
// the same on element i of the arrays; returns the new parameter
__device__ __forceinline__ float adam_elem(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                           float* __restrict__ v, int64_t i, const AdamCoef& c) {
    float pi = p[i], mi = m[i], vi = v[i];
    adam_val(pi, g[i], mi, vi, c);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    return pi;
}
__global__ __launch_bounds__(256) void adam_kernel(AdamBatch bt, AdamCoef c) {
    int t = 0;
    while (t + 1 < bt.count && (int)blockIdx.x >= bt.blk0[t + 1]) ++t;
    const int64_t base = (int64_t)(blockIdx.x - bt.blk0[t]) * 1024;
    const int64_t n = bt.n[t];
    for (int64_t i = base + threadIdx.x; i < min(n, base + 1024); i += blockDim.x) adam_elem(bt.p[t], bt.g[t], bt.m[t], bt.v[t], i, c);
}

// ---------------------------------------------------------------- Adam + GEMM weight packing, one launch
// W [d0][d1][taps] f32 -> P0 [d0][taps][ld0] and P1 [d1][taps][ld1] (T).  A block owns one 32 x 32 (i0, i1)
// tile of one weight: it streams the tile's p/g/m/v rows (n1*taps contiguous floats per i0) through the
// Adam update, keeps the new values in LDS (row stride 32*taps+1: conflict-free for both read-outs) and
// writes each (i0, tap) segment of P0 and each (i1, tap) segment of P1 as 32 consecutive elements.
// Unpacked tensors (BatchNorm affine, biases) are 4096-element chunks of the same launch.
// Tile edge of a packed job: conv weights (taps 9) 32 x 32 x 9, linear weights (taps 1) 64 x 64 (4096 elements:
// 16 per thread, every float4 of p / g / m / v in flight at once; 128-byte pack segments)
__host__ __device__ inline int adam_tile_edge(int taps) { return taps == 1 ? 64 : 32; }
// the tile's P0 [d0][taps][ld0] and P1 [d1][taps][ld1] segments from the updated values in LDS (row stride RS)
template <typename T>
__device__ __forceinline__ void pack_tile_out(const ops::AdamJob& jb, const float* tile, int RS, int TS, int t0, int t1,
                                              int n0, int n1) {
    const int taps = jb.taps, sh = TS == 64 ? 6 : 5;
    T* p0 = (T*)jb.p0;
    T* p1 = (T*)jb.p1;
    if (p0)
        for (int e = threadIdx.x; e < n0 * taps * TS; e += 256) {
            const int q = e & (TS - 1), at = e >> sh, a = at / taps, tap = at - a * taps;
            if (q < n1) p0[((int64_t)(t0 + a) * taps + tap) * jb.ld0 + t1 + q] = from_f32<T>(tile[a * RS + q * taps + tap]);
        }
    if (p1)
        for (int e = threadIdx.x; e < n1 * taps * TS; e += 256) {
            const int q = e & (TS - 1), ct = e >> sh, cc = ct / taps, tap = ct - cc * taps;
            if (q < n0) p1[((int64_t)(t1 + cc) * taps + tap) * jb.ld1 + t0 + q] = from_f32<T>(tile[q * RS + cc * taps + tap]);
        }
}
template <typename T>
// cdev (nullable): coefficients read from device memory (graph replays: the host refreshes them per step)
// tile_base: first tile of this launch (a launch may cover a contiguous tile range of the job list)
__global__ __launch_bounds__(256) void adam_pack_kernel(const ops::AdamJob* __restrict__ jobs, int njobs, AdamCoef cv,
                                                        const AdamCoef* __restrict__ cdev, int tile_base) {
    const AdamCoef c = cdev ? *cdev : cv;
    const int bid = blockIdx.x + tile_base;
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].tile0 <= bid) lo = mid; else hi = mid - 1;
    }
    const ops::AdamJob jb = jobs[lo];
    const int tl = bid - jb.tile0;
    if (jb.taps == 0) {
        const int64_t base = (int64_t)tl * 4096, end = min(jb.n, base + 4096);
        for (int64_t i = base + threadIdx.x; i < end; i += 256) adam_elem(jb.p, jb.g, jb.m, jb.v, i, c);
        return;
    }
    const int taps = jb.taps, TS = adam_tile_edge(taps);
    const int tt0 = tl / jb.nt1, tt1 = tl - tt0 * jb.nt1;
    const int t0 = tt0 * TS, t1 = tt1 * TS;
    const int n0 = min(TS, jb.d0 - t0), n1 = min(TS, jb.d1 - t1);
    const int RS = TS * taps + 1;
    __shared__ float tile[32 * (32 * 9 + 1)];  // >= 64 x 65 as well
    const int rowlen = n1 * taps;
    const int64_t row0 = ((int64_t)t0 * jb.d1 + t1) * taps;  // element offset of the tile's first row
    const auto al16 = [&](const float* q) { return ((reinterpret_cast<uintptr_t>(q + row0)) & 15) == 0; };
    if ((rowlen & 3) == 0 && ((jb.d1 * taps) & 3) == 0 && al16(jb.p) && al16(jb.g) && al16(jb.m) && al16(jb.v)) {
        // 16-byte rows: every thread has U float4 of each of p / g / m / v in flight before the updates
        // (the per-element path below waits on each element's four loads in turn: 3.7 TB/s for the whole step)
        constexpr int U = 4;
        const int rl4 = rowlen >> 2, total4 = n0 * rl4;
        for (int e0 = threadIdx.x; e0 < total4; e0 += 256 * U) {
            float4 pp[U], gg[U], mm[U], vv[U];
            int64_t gi[U];
            int li[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = min(e0 + u * 256, total4 - 1);  // clamped: always in-bounds, skipped below
                const int a = e / rl4, r4 = e - a * rl4;
                gi[u] = row0 + (int64_t)a * jb.d1 * taps + 4 * r4;
                li[u] = a * RS + 4 * r4;
                pp[u] = *reinterpret_cast<const float4*>(jb.p + gi[u]);
                gg[u] = *reinterpret_cast<const float4*>(jb.g + gi[u]);
                mm[u] = *reinterpret_cast<const float4*>(jb.m + gi[u]);
                vv[u] = *reinterpret_cast<const float4*>(jb.v + gi[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (e0 + u * 256 >= total4) break;
                adam_val(pp[u].x, gg[u].x, mm[u].x, vv[u].x, c);
                adam_val(pp[u].y, gg[u].y, mm[u].y, vv[u].y, c);
                adam_val(pp[u].z, gg[u].z, mm[u].z, vv[u].z, c);
                adam_val(pp[u].w, gg[u].w, mm[u].w, vv[u].w, c);
                *reinterpret_cast<float4*>(jb.p + gi[u]) = pp[u];
                *reinterpret_cast<float4*>(jb.m + gi[u]) = mm[u];
                *reinterpret_cast<float4*>(jb.v + gi[u]) = vv[u];
                tile[li[u]] = pp[u].x;
                tile[li[u] + 1] = pp[u].y;
                tile[li[u] + 2] = pp[u].z;
                tile[li[u] + 3] = pp[u].w;
            }
        }
    } else {
        int a = 0, r = threadIdx.x;
        while (r >= rowlen) { r -= rowlen; ++a; }
        for (; a < n0;) {
            const int64_t idx = ((int64_t)(t0 + a) * jb.d1 + t1) * taps + r;
            tile[a * RS + r] = adam_elem(jb.p, jb.g, jb.m, jb.v, idx, c);
            r += 256;
            while (r >= rowlen) { r -= rowlen; ++a; }
        }
    }
    __syncthreads();
    pack_tile_out<T>(jb, tile, RS, TS, t0, t1, n0, n1);
}

// packing alone (forward of a model whose weights were changed outside the engine)
template <typename T>
__global__ __launch_bounds__(256) void pack_kernel(const ops::AdamJob* __restrict__ jobs, int njobs) {
    const int bid = blockIdx.x;
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].tile0 <= bid) lo = mid; else hi = mid - 1;
    }
    const ops::AdamJob jb = jobs[lo];
    if (jb.taps == 0) return;
    const int tl = bid - jb.tile0;
    const int taps = jb.taps, TS = adam_tile_edge(taps);
    const int tt0 = tl / jb.nt1, tt1 = tl - tt0 * jb.nt1;
    const int t0 = tt0 * TS, t1 = tt1 * TS;
    const int n0 = min(TS, jb.d0 - t0), n1 = min(TS, jb.d1 - t1);
    const int RS = TS * taps + 1;
    __shared__ float tile[32 * (32 * 9 + 1)];
    const int rowlen = n1 * taps;
    {
        int a = 0, r = threadIdx.x;
        while (r >= rowlen) { r -= rowlen; ++a; }
        for (; a < n0;) {
            tile[a * RS + r] = jb.p[((int64_t)(t0 + a) * jb.d1 + t1) * taps + r];
            r += 256;
            while (r >= rowlen) { r -= rowlen; ++a; }
        }
    }
    __syncthreads();
    pack_tile_out<T>(jb, tile, RS, TS, t0, t1, n0, n1);
}

}  // namespace

// ============================================================================ launchers
namespace ops {

// the accumulator a layer's statistics use (xacc_shards(C) copies of 2C columns)
size_t bn_acc_bytes(int C) { return XAcc::bytes(xacc_shards(C), 2 * C) + 64; }  // + bn_bwd_fused_kernel's arrival count
size_t bias_acc_bytes(int C) { return XAcc::bytes(xacc_shards(C), C); }

template <typename T>
static int check_bn_shape(int C) {
    constexpr int V = Vec16<T>::N;
    HLMC_CHECK_ARG(C % V == 0 && C / V <= 256 && 256 % (C / V) == 0, "BatchNorm channel count unsupported");
    return HLMC_OK;
}
static int check_acc(const XAcc& a, int ncols) {
    HLMC_CHECK_ARG(a.p && a.ncols == ncols && a.shards >= 1 && a.shards <= kXAccMaxShards, "statistics accumulator");
    return HLMC_OK;
}

template <typename T>
int bn_stats(hipStream_t s, const T* y, int64_t R, int C, float* mean, float* invstd, float* run_mean, float* run_var,
             int64_t* nbt, float momentum, float eps, XAcc acc) {
    HLMC_TRY(check_bn_shape<T>(C));
    HLMC_TRY(check_acc(acc, 2 * C));
    const int nblk = bn_blocks(R, C);
    HLMC_BN_PROBED(s, (double)sizeof(T) * R * C,
                   (col_moments_kernel<T><<<nblk, kThreads, 0, s>>>(y, R, C, bn_rows_per_blk(R, C), acc)));
    HLMC_LAUNCHED();
    bn_finalize_kernel<<<fin_grid(C), 64, 0, s>>>(acc, C, R, mean, invstd, run_mean, run_var, nbt, momentum, eps);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int bn_moments(hipStream_t s, const T* y, int64_t R, int C, XAcc acc) {
    HLMC_TRY(check_bn_shape<T>(C));
    HLMC_TRY(check_acc(acc, 2 * C));
    HLMC_BN_PROBED(s, (double)sizeof(T) * R * C,
                   (col_moments_kernel<T><<<bn_blocks(R, C), kThreads, 0, s>>>(y, R, C, bn_rows_per_blk(R, C), acc)));
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int bn_eval_stats(hipStream_t s, const float* run_mean, const float* run_var, int C, float eps, float* mean, float* invstd) {
    bn_eval_kernel<<<cdiv(C, 256), 256, 0, s>>>(run_mean, run_var, C, eps, mean, invstd);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int bn_act(hipStream_t s, const T* y, int64_t R, int C, const float* mean, const float* invstd, const float* gamma,
           const float* beta, int act, const uint8_t* mask, float mscale, T* a, int lda) {
    HLMC_TRY(check_bn_shape<T>(C));
    HLMC_CHECK_ARG(lda % Vec16<T>::N == 0, "bn_act: output row stride must be a multiple of 16 bytes");
    const int rpp = kThreads / (C / Vec16<T>::N);
    const unsigned g = grid_for(R, rpp * kU);
    const double by = 2.0 * sizeof(T) * R * C;
    if (mask)
        HLMC_BN_PROBED(s, by, (bn_act_kernel<T, true, false><<<g, kThreads, 0, s>>>(y, R, C, mean, invstd, gamma, beta, act,
                                                                                   mask, mscale, a, lda, BnFin{})));
    else
        HLMC_BN_PROBED(s, by, (bn_act_kernel<T, false, false><<<g, kThreads, 0, s>>>(y, R, C, mean, invstd, gamma, beta,
                                                                                    act, mask, mscale, a, lda, BnFin{})));
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int bn_act_train(hipStream_t s, const T* y, int64_t R, int C, XAcc acc, bool have_stats, float* mean, float* invstd,
                 float* run_mean, float* run_var, int64_t* nbt, float momentum, float eps, const float* gamma,
                 const float* beta, int act, const uint8_t* mask, float mscale, T* a, int lda) {
    HLMC_TRY(check_bn_shape<T>(C));
    HLMC_TRY(check_acc(acc, 2 * C));
    HLMC_CHECK_ARG(lda % Vec16<T>::N == 0, "bn_act: output row stride must be a multiple of 16 bytes");
    if (!have_stats) {  // no statistics from the producer: a moments pass into the (zeroed) accumulator first
        HLMC_BN_PROBED(s, (double)sizeof(T) * R * C,
                       (col_moments_kernel<T><<<bn_blocks(R, C), kThreads, 0, s>>>(y, R, C, bn_rows_per_blk(R, C), acc)));
        HLMC_LAUNCHED();
    }
    if (C > kFinMaxC) {  // wide channels: a separate finalize
        bn_finalize_kernel<<<fin_grid(C), 64, 0, s>>>(acc, C, R, mean, invstd, run_mean, run_var, nbt, momentum, eps);
        HLMC_LAUNCHED();
        return bn_act<T>(s, y, R, C, mean, invstd, gamma, beta, act, mask, mscale, a, lda);
    }
    BnFin fin;
    fin.acc = acc; fin.R = R;
    fin.mean = mean; fin.invstd = invstd; fin.rmean = run_mean; fin.rvar = run_var; fin.nbt = nbt;
    fin.momentum = momentum; fin.eps = eps;
    const int rpp = kThreads / (C / Vec16<T>::N);
    const unsigned g = grid_for(R, rpp * kU);
    const double by = 2.0 * sizeof(T) * R * C;
    if (mask)
        HLMC_BN_PROBED(s, by, (bn_act_kernel<T, true, true><<<g, kThreads, 0, s>>>(y, R, C, mean, invstd, gamma, beta, act,
                                                                                  mask, mscale, a, lda, fin)));
    else
        HLMC_BN_PROBED(s, by, (bn_act_kernel<T, false, true><<<g, kThreads, 0, s>>>(y, R, C, mean, invstd, gamma, beta,
                                                                                   act, mask, mscale, a, lda, fin)));
    HLMC_LAUNCHED();
    return HLMC_OK;
}

// bn_bwd_fused_kernel instances: rows per thread kNR (8, or 4 where 8 leaves fewer than 256 blocks), activation
template <typename T>
static void bn_bwd_fused_kernel_ptr(int nr, int act, void (*&k)(const T*, int, const T*, int, int, const float*,
                                                                const float*, const float*, const float*, int, T*,
                                                                float*, float*, XAcc, XAcc, int, int, unsigned*)) {
    k = nr == 8 ? (act == 0 ? bn_bwd_fused_kernel<T, 8, 0> : bn_bwd_fused_kernel<T, 8, -1>)
                : (act == 0 ? bn_bwd_fused_kernel<T, 4, 0> : bn_bwd_fused_kernel<T, 4, -1>);
}
// Which layers take the fused form: R * C <= kBnFusedMaxElems, C a multiple of the slab width, and the whole grid
// co-resident (occupancy query x CUs) -- the kernel's arrival count needs every block running at once.  Measured
// (scripts/bench_bn.py under rocprofv3, bf16 B = 256): 4 x 4 x 512 14.4 us vs 21.3 us for the two passes, 8 x 8 x 256
// 15.4 vs 21.3, 16 x 16 x 128 30.8 vs 21.3 (512 blocks: the count waits for the slowest of two blocks per CU; 26.6 vs
// 26.6 us per op call with 16 rows per thread on 256 blocks, yet the step 136.1k vs 138.1k); the step with 2^22:
// 138.6k vs 137.9k clips/s (3 rounds; 2^21: 138.3k, 2^23: 133.7k).  The test hook hlmc_test_bn_fused overrides the
// limit (0: every layer on the two passes; the parity test compares the forms) and the spin bound.
constexpr int64_t kBnFusedMaxElems = (int64_t)1 << 22;
static std::atomic<int64_t> g_bn_fused_lim{kBnFusedMaxElems};
static std::atomic<int> g_bn_spin_max{kBnSpinMax};

void test_bn_fused(int64_t max_elems, int spin_max) {
    g_bn_fused_lim.store(max_elems < 0 ? kBnFusedMaxElems : max_elems);
    g_bn_spin_max.store(spin_max < 0 ? kBnSpinMax : spin_max);
}

// The library's device status word: pinned, mapped host memory that kernels write with system-scope stores when they
// detect a fault they must not hang on or hide (bn_bwd_fused_kernel's spin running out).  The host reads it without
// synchronising; the C-ABI backward entry points report a raised bit as HLMC_EDEVICE.
static unsigned* g_dev_status = nullptr;
static std::mutex g_dev_status_mu;
unsigned* dev_status_word() {
    std::lock_guard<std::mutex> lk(g_dev_status_mu);
    if (!g_dev_status) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
            return nullptr;
        std::memset(p, 0, 64);
        g_dev_status = static_cast<unsigned*>(p);
    }
    return g_dev_status;
}
unsigned dev_status_take(bool clear) {
    unsigned* w = dev_status_word();
    if (!w) return 0;
    return clear ? __atomic_exchange_n(w, 0u, __ATOMIC_SEQ_CST) : __atomic_load_n(w, __ATOMIC_SEQ_CST);
}

// Residency of a bn_bwd_fused_kernel instance on one device (blocks per CU x CUs), computed once per (device, kNR,
// activation): the arrival count needs every block of the grid running at once.
static int bn_fused_resident(int nr, int act, bool bf) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, bool>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(dev, nr, act, bf);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    const void* k = nullptr;
    if (bf) {
        void (*kp)(const bf16*, int, const bf16*, int, int, const float*, const float*, const float*, const float*, int,
                   bf16*, float*, float*, XAcc, XAcc, int, int, unsigned*);
        bn_bwd_fused_kernel_ptr<bf16>(nr, act, kp);
        k = reinterpret_cast<const void*>(kp);
    } else {
        void (*kp)(const float*, int, const float*, int, int, const float*, const float*, const float*, const float*,
                   int, float*, float*, float*, XAcc, XAcc, int, int, unsigned*);
        bn_bwd_fused_kernel_ptr<float>(nr, act, kp);
        k = reinterpret_cast<const void*>(kp);
    }
    int cus = 0, occ = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kThreads, 0) != hipSuccess) occ = 0;
    const int res = cus * occ > 0 ? cus * occ : -1;
    cache[key] = res;
    return res;
}
template <typename T>
static bool bn_fused_plan(int64_t R, int C, int act, int& nr, int& nslab, unsigned& grid) {
    constexpr int SW = 8 * Vec16<T>::N;
    const int64_t lim = g_bn_fused_lim.load(std::memory_order_relaxed);
    if (C % SW != 0 || R * C > lim || R >= ((int64_t)1 << 31) || xacc_shards(C) > kBnFusedShards) return false;
    nslab = C / SW;
    nr = (int64_t)nslab * ((R + 255) / 256) >= 256 ? 8 : 4;
    const int64_t G = (int64_t)nslab * ((R + 32 * nr - 1) / (32 * nr));
    // at most HALF the device's resident capacity: the other half stays free for the grids that co-run on the
    // weight-gradient stream and, under data parallelism, RCCL's kernels on the comm stream, so the count's blocks
    // never wait for CUs those grids hold (the B = 256 layers: G = 256 against 2 blocks per CU x 256 CUs)
    const int res = bn_fused_resident(nr, act, std::is_same<T, bf16>::value);
    if (res < 0 || 2 * G > res || !dev_status_word()) return false;
    grid = (unsigned)G;
    return true;
}
template <typename T>
static void bn_fused_launch(hipStream_t s, int nr, int act, unsigned g, const T* da, int lda, const T* y, int R,
                                  int C, const float* mean, const float* invstd, const float* gamma, const float* beta,
                                  T* dy, float* dgamma, float* dbeta, XAcc mom, XAcc bias_acc, int nslab) {
    void (*k)(const T*, int, const T*, int, int, const float*, const float*, const float*, const float*, int, T*, float*,
              float*, XAcc, XAcc, int, int, unsigned*);
    bn_bwd_fused_kernel_ptr<T>(nr, act, k);
    k<<<g, kThreads, 0, s>>>(da, lda, y, R, C, mean, invstd, gamma, beta, act, dy, dgamma, dbeta, mom, bias_acc, nslab,
                             g_bn_spin_max.load(std::memory_order_relaxed), dev_status_word());
}

template <typename T>
int bn_act_bwd(hipStream_t s, const T* da, int lda, const T* y, int64_t R, int C, const float* mean, const float* invstd,
               const float* gamma, const float* beta, int act, const uint8_t* mask, float mscale, T* dy, float* dgamma,
               float* dbeta, XAcc mom, const BnBwdFuse* fused, XAcc bias_acc, float* dbias, float* sums) {
    HLMC_TRY(check_bn_shape<T>(C));
    HLMC_TRY(check_acc(mom, 2 * C));
    if (bias_acc.on()) HLMC_TRY(check_acc(bias_acc, C));
    HLMC_CHECK_ARG(!dbias || bias_acc.on(), "bn_act_bwd: dbias needs its accumulator");
    HLMC_CHECK_ARG(lda % Vec16<T>::N == 0, "bn_act_bwd: grad row stride must be a multiple of 16 bytes");
    if (!mask && !(fused && fused->done) && R <= 256 * kSmallRpt) {  // small layer: one launch (bn_bwd_small_kernel)
        auto k = act == 0 ? bn_bwd_small_kernel<T, 0> : bn_bwd_small_kernel<T, -1>;
        HLMC_BN_PROBED(s, 3.0 * sizeof(T) * R * C,
                       (k<<<C / Vec16<T>::N, kThreads, 0, s>>>(da, lda, y, (int)R, C, mean, invstd, gamma, beta, act, dy,
                                                              dgamma, dbeta, bias_acc)));
        HLMC_LAUNCHED();
        if (dbias) return colsum_finalize(s, bias_acc, C, dbias);
        return HLMC_OK;
    }
    if (!mask && !(fused && fused->done)) {  // mid-size layer: one launch with a grid-wide count (bn_bwd_fused_kernel)
        int nr = 0, nslab = 0;
        unsigned g = 0;
        if (bn_fused_plan<T>(R, C, act, nr, nslab, g)) {
            HLMC_BN_PROBED(s, 3.0 * sizeof(T) * R * C, bn_fused_launch<T>(s, nr, act, g, da, lda, y, (int)R, C, mean,
                                                                       invstd, gamma, beta, dy, dgamma, dbeta, mom,
                                                                       bias_acc, nslab));
            HLMC_LAUNCHED();
            if (dbias) return colsum_finalize(s, bias_acc, C, dbias);
            return HLMC_OK;
        }
    }
    const int nblk = bn_blocks(R, C);
    const int64_t rpb = bn_rows_per_blk(R, C);
    if (fused && fused->done) {  // moments came with the producer of da
        HLMC_CHECK_ARG(fused->acc.p == mom.p && lda == C && !mask && act == 0,
                       "bn_act_bwd: fused moments need a dense lrelu layer and its accumulator");
    } else {
        auto k = mask ? bn_bwd_moments_kernel<T, true> : act == 0 ? bn_bwd_moments_kernel<T, false, 0>
                                                                  : bn_bwd_moments_kernel<T, false>;
        HLMC_BN_PROBED(s, 2.0 * sizeof(T) * R * C,
                       (k<<<nblk, kThreads, 0, s>>>(da, lda, y, R, C, mean, invstd, gamma, beta, act, mask, mscale, rpb,
                                                    mom)));
        HLMC_LAUNCHED();
    }
    const bool fin_here = C <= kFinMaxC;  // the apply kernel finalizes the moments itself: no finalize launch
    BnFin bf;
    if (fin_here) {
        bf.acc = mom; bf.dgamma = dgamma; bf.dbeta = dbeta;
    } else {
        HLMC_CHECK_ARG(sums, "bn_act_bwd: C > 512 needs 2C floats of sums scratch");
        bn_bwd_finalize_kernel<<<fin_grid(C), 64, 0, s>>>(mom, C, dgamma, dbeta, sums);
        HLMC_LAUNCHED();
    }
    auto ka = mask ? (fin_here ? bn_bwd_apply_kernel<T, true, true> : bn_bwd_apply_kernel<T, true, false>)
              : act == 0 ? (fin_here ? bn_bwd_apply_kernel<T, false, true, 0> : bn_bwd_apply_kernel<T, false, false, 0>)
                         : (fin_here ? bn_bwd_apply_kernel<T, false, true> : bn_bwd_apply_kernel<T, false, false>);
    HLMC_BN_PROBED(s, 3.0 * sizeof(T) * R * C,
                   (ka<<<nblk, kThreads, 0, s>>>(da, lda, y, R, C, mean, invstd, gamma, beta, act, mask, mscale, sums,
                                                 dy, rpb, bias_acc, bf)));
    HLMC_LAUNCHED();
    if (dbias) return colsum_finalize(s, bias_acc, C, dbias);
    return HLMC_OK;
}
int colsum_to_f64(hipStream_t s, XAcc acc, int C, double* out) {
    HLMC_CHECK_ARG(out && C > 0, "colsum_to_f64: bad arguments");
    HLMC_TRY(check_acc(acc, C));
    xacc_to_f64_kernel<<<fin_grid(C), 64, 0, s>>>(acc, C, out);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
int colsum_finalize(hipStream_t s, XAcc acc, int C, float* out) {
    HLMC_CHECK_ARG(out && C > 0, "colsum_finalize: bad arguments");
    HLMC_TRY(check_acc(acc, C));
    HLMC_BN_PROBED(s, 24.0 * acc.shards * C, (xacc_to_f32_kernel<<<fin_grid(C), 64, 0, s>>>(acc, C, out)));
    HLMC_LAUNCHED();
    return HLMC_OK;
}


template <typename T>
int conv_c1_s2(hipStream_t s, const float* x, int B, int Hi, int Wi, const float* w, const float* bias, int Co, T* y,
               ColStats* st, BnBwdFuse* bf) {
    HLMC_CHECK_ARG(Co == 32 && Hi % 2 == 0 && Wi % 2 == 0, "conv_c1_s2: only Co == 32, even H/W");
    int64_t nthr = (int64_t)B * (Hi / 2) * (Wi / 2) * (32 / Vec16<T>::N);
    HLMC_CHECK_ARG(nthr < (int64_t)1 << 31, "conv_c1_s2: too many pixels");
    const FastDiv dW((uint32_t)(Wi / 2)), dH((uint32_t)(Hi / 2));
    C1Fuse fz;
    if (st) st->done = false;
    if (bf) bf->done = false;
    if (st && st->acc.on()) {
        // fewer, longer-running blocks: one accumulator contribution each
        HLMC_TRY(check_acc(st->acc, 2 * Co));
        const int g = grid_for(nthr, kThreads, kC1FusedBlocks);
        fz.acc = st->acc;
        conv_c1_s2_kernel<T, 32, 1><<<g, kThreads, 0, s>>>(x, B, Hi, Wi, w, bias, y, dW, dH, fz);
        st->done = true;
    } else if (bf && bf->acc.on()) {
        HLMC_TRY(check_acc(bf->acc, 2 * Co));
        // one full wave of blocks at this mode's 3 blocks per CU (launch bounds): 132.3k vs 131.9k clips/s with
        // 1024 blocks (1.33 waves; 512: 132.3k; the forward mode's 4 per CU keep 1024: 768 there 132.0k)
        const int g = grid_for(nthr, kThreads, kC1BwdBlocks);
        fz.acc = bf->acc;
        fz.ybn = bf->y; fz.mean = bf->mean; fz.invstd = bf->invstd; fz.gamma = bf->gamma; fz.beta = bf->beta;
        conv_c1_s2_kernel<T, 32, 2><<<g, kThreads, 0, s>>>(x, B, Hi, Wi, w, bias, y, dW, dH, fz);
        bf->done = true;
    } else {
        conv_c1_s2_kernel<T, 32, 0><<<grid_for(nthr, kThreads, 16384), kThreads, 0, s>>>(x, B, Hi, Wi, w, bias, y, dW, dH,
                                                                                        fz);
    }
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int convT_c1(hipStream_t s, const T* x, int B, int Hi, int Wi, int Ci, const float* w, const float* bias, float* y) {
    HLMC_CHECK_ARG(Ci == 32, "convT_c1: only Ci == 32");
    int64_t npix = (int64_t)B * 4 * Hi * Wi;
    HLMC_CHECK_ARG(npix < (int64_t)1 << 31, "convT_c1: too many pixels");
    HLMC_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0, "convT_c1: alignment");
    const FastDiv dW((uint32_t)Wi), dH((uint32_t)Hi);
    convT_c1_kernel<T, 32><<<(unsigned)((npix / 4 + kThreads - 1) / kThreads), kThreads, 0, s>>>(x, B, Hi, Wi, w, bias, y,
                                                                                              dW, dH);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

static int wgrad_c1_blocks(int64_t K) { return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (K + 1023) / 1024)); }
static int wgrad_c1_row_blocks(int64_t rows);
size_t wgrad_c1_ws(int B, int Hl, int Wl, int M) {
    return (size_t)std::max(wgrad_c1_blocks((int64_t)B * Hl * Wl), wgrad_c1_row_blocks((int64_t)B * Hl)) * M * 9 *
           sizeof(float);
}

// 64-wide layers (every use in the model): the row-staged kernel on <= 512 blocks (two per CU)
static int wgrad_c1_row_blocks(int64_t rows) { return (int)std::max<int64_t>(1, std::min<int64_t>(512, rows)); }

template <typename T>
int wgrad_c1(hipStream_t s, const T* L, int B, int Hl, int Wl, int M, const float* Xh, float* dW, Ws ws) {
    HLMC_CHECK_ARG(M == 32, "wgrad_c1: only M == 32");
    if (Wl == 64 && ((uintptr_t)L & 15) == 0 && ((uintptr_t)Xh & 15) == 0) {
        const int64_t rows = (int64_t)B * Hl;
        HLMC_CHECK_ARG(rows < (int64_t)1 << 31, "wgrad_c1: too many rows");
        const int nb = wgrad_c1_row_blocks(rows);
        HLMC_CHECK_ARG(ws.bytes >= (size_t)nb * M * 9 * sizeof(float), "wgrad_c1 workspace");
        wgrad_c1_rows_kernel<T><<<nb, kThreads, 0, s>>>(L, (int)rows, Hl, Xh, ws.p);
        HLMC_LAUNCHED();
        sum_partials_f32_kernel<<<M * 9, 256, 0, s>>>(ws.p, nb, M * 9, dW);
        HLMC_LAUNCHED();
        return HLMC_OK;
    }
    int64_t K = (int64_t)B * Hl * Wl;
    int nblk = wgrad_c1_blocks(K);
    HLMC_CHECK_ARG(ws.bytes >= wgrad_c1_ws(B, Hl, Wl, M), "wgrad_c1 workspace");
    int rpb = (int)((K + nblk - 1) / nblk);
    HLMC_CHECK_ARG(K < (int64_t)1 << 31, "wgrad_c1: too many rows");
    wgrad_c1_kernel<T, 32><<<nblk, kThreads, 0, s>>>(L, B, Hl, Wl, Xh, rpb, ws.p, FastDiv((uint32_t)Wl),
                                                     FastDiv((uint32_t)Hl));
    HLMC_LAUNCHED();
    sum_partials_f32_kernel<<<M * 9, 256, 0, s>>>(ws.p, nblk, M * 9, dW);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int cast_from_f32(hipStream_t s, const float* x, T* y, int64_t n) {
    cast_kernel<float, T><<<grid_for(n), kThreads, 0, s>>>(x, y, n);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int cast_to_f32(hipStream_t s, const T* x, float* y, int64_t n) {
    cast_kernel<T, float><<<grid_for(n), kThreads, 0, s>>>(x, y, n);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int copy2d(hipStream_t s, const T* x, int ldx, T* y, int ldy, int rows, int cols) {
    cast2d_kernel<T, T><<<grid_for((int64_t)rows * cols), kThreads, 0, s>>>(x, ldx, y, ldy, rows, cols);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int cast2d_from_f32(hipStream_t s, const float* x, int ldx, T* y, int ldy, int rows, int cols) {
    cast2d_kernel<float, T><<<grid_for((int64_t)rows * cols), kThreads, 0, s>>>(x, ldx, y, ldy, rows, cols);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int nhwc_to_flat(hipStream_t s, const T* x, int B, int h, int w, int C, T* y, int ldy, const T* relu_ref) {
    nhwc_to_flat_kernel<T><<<grid_for((int64_t)B * C * h * w), kThreads, 0, s>>>(x, B, h, w, C, y, ldy, relu_ref);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int flat_to_nhwc(hipStream_t s, const T* x, int ldx, int B, int h, int w, int C, T* y) {
    flat_to_nhwc_kernel<T><<<grid_for((int64_t)B * C * h * w), kThreads, 0, s>>>(x, ldx, B, h, w, C, y);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
static int colsum_blocks(int rows) { return std::max(1, std::min(1024, rows / 256)); }
size_t colsum_ws(int rows, int cols) { return (size_t)colsum_blocks(rows) * cols * sizeof(double); }  // <= 1024 rows: no fold
template <typename T>
__global__ __launch_bounds__(256) void colsum_narrow_kernel(const T* __restrict__ x, int ld, int rows, int cols,
                                                            int rows_per_blk, double* __restrict__ part) {
    __shared__ double sh[256];
    const int r0 = blockIdx.x * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
    for (int c = 0; c < cols; ++c) {
        double s = 0.0;
        for (int r = r0 + threadIdx.x; r < r1; r += blockDim.x) s += to_f32<T>(x[(int64_t)r * ld + c]);
        sh[threadIdx.x] = s;
        __syncthreads();
        for (int w = blockDim.x / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) part[(int64_t)blockIdx.x * cols + c] = sh[0];
        __syncthreads();
    }
}

template <typename T>
int colsum(hipStream_t s, const T* dy, int ld, int rows, int cols, float* db, Ws ws) {
    int nblk = colsum_blocks(rows);
    if (cols < 16) {
        HLMC_CHECK_ARG(ws.bytes >= colsum_ws(rows, cols), "colsum workspace");
        const int rpb = (rows + nblk - 1) / nblk;
        double* part = reinterpret_cast<double*>(ws.p);
        colsum_narrow_kernel<T><<<nblk, 256, 0, s>>>(dy, ld, rows, cols, rpb, part);
        HLMC_LAUNCHED();
        colsum_finalize_kernel<<<fin_grid(cols), 1024, 0, s>>>(part, nblk, cols, db);
        HLMC_LAUNCHED();
        return HLMC_OK;
    }
    HLMC_CHECK_ARG(ws.bytes >= colsum_ws(rows, cols), "colsum workspace");
    int rpb = (rows + nblk - 1) / nblk;
    double* part = reinterpret_cast<double*>(ws.p);
    dim3 grid(nblk, cdiv(cols, 64));
    colsum_partial_kernel<T><<<grid, 256, 0, s>>>(dy, ld, rows, cols, rpb, part);
    HLMC_LAUNCHED();
    colsum_finalize_kernel<<<fin_grid(cols), 1024, 0, s>>>(part, nblk, cols, db);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
struct CopySegs4 {
    CopySeg seg[4];
    int64_t start[5];
};
__global__ __launch_bounds__(256) void copy_segments_kernel(CopySegs4 c) {
    const int64_t total = c.start[4];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int k = 0;
        while (k < 3 && i >= c.start[k + 1]) ++k;
        const int64_t j = i - c.start[k];
        c.seg[k].dst[j] = c.seg[k].src[j];
    }
}
int copy_segments(hipStream_t s, const CopySeg* segs, int nseg) {
    HLMC_CHECK_ARG(nseg >= 0 && nseg <= 4, "copy_segments: at most 4 segments");
    CopySegs4 c{};
    int k = 0;
    for (int i = 0; i < nseg; ++i)
        if (segs[i].dst && segs[i].src && segs[i].n > 0) c.seg[k++] = segs[i];
    if (k == 0) return HLMC_OK;
    c.start[0] = 0;
    for (int i = 0; i < 4; ++i) c.start[i + 1] = c.start[i] + (i < k ? c.seg[i].n : 0);
    copy_segments_kernel<<<grid_for(c.start[4]), kThreads, 0, s>>>(c);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int reparam_fwd(hipStream_t s, const float* mu, const float* lv, const float* eps, int n_rows, int L, T* z, int ldz,
                float* mu_out, float* lv_out, float* eps_keep) {
    LatentOut lo;
    lo.mu = mu_out; lo.lv = lv_out; lo.eps = eps_keep;
    reparam_fwd_kernel<T><<<grid_for((int64_t)n_rows * L), kThreads, 0, s>>>(mu, lv, eps, n_rows, L, z, ldz, lo);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
int randn(hipStream_t s, float* out, int64_t n, uint64_t seed, uint64_t offset) {
    HLMC_CHECK_ARG(out && n >= 0 && offset % 4 == 0, "randn: bad arguments (offset must be a multiple of 4)");
    if (n == 0) return HLMC_OK;
    randn_kernel<<<grid_for((n + 3) / 4), kThreads, 0, s>>>(out, n, seed, offset);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int reparam_rng(hipStream_t s, const float* mu, const float* lv, uint64_t seed, uint64_t offset, int n_rows, int L,
                float* eps_out, T* z, int ldz, float* mu_out, float* lv_out) {
    HLMC_CHECK_ARG(offset % 4 == 0, "reparam_rng: offset must be a multiple of 4");
    LatentOut lo;
    lo.mu = mu_out; lo.lv = lv_out;
    reparam_rng_kernel<T><<<grid_for(((int64_t)n_rows * L + 3) / 4), kThreads, 0, s>>>(mu, lv, seed, offset, n_rows, L,
                                                                                       eps_out, z, ldz, lo);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <typename T>
int reparam_bwd(hipStream_t s, const T* dz, int lddz, const float* lv, const float* eps, const float* d_mu,
                const float* d_lv, int n_rows, int L, T* gmu, T* glv) {
    reparam_bwd_kernel<T><<<grid_for((int64_t)n_rows * L), kThreads, 0, s>>>(dz, lddz, lv, eps, d_mu, d_lv, n_rows, L,
                                                                            gmu, glv);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

static int vae_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 2047) / 2048)); }
size_t vae_sums_ws(int64_t na, int64_t nt, int64_t nl) {
    return (size_t)vae_blocks(std::max(na, std::max(nt, nl))) * 3 * sizeof(double);
}
int vae_sums(hipStream_t s, const float* ra, const float* a, int64_t na, const float* rt, const float* t, int64_t nt,
             const float* mu, const float* lv, int64_t nl, double* out3, Ws ws) {
    int nblk = vae_blocks(std::max(na, std::max(nt, nl)));
    HLMC_CHECK_ARG(ws.bytes >= vae_sums_ws(na, nt, nl), "loss workspace");
    double* part = reinterpret_cast<double*>(ws.p);
    vae_sums_kernel<<<nblk, kThreads, 0, s>>>(ra, a, na, rt, t, nt, mu, lv, nl, part);
    HLMC_LAUNCHED();
    vae_sums_finalize_kernel<<<3, 256, 0, s>>>(part, nblk, out3);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
int vae_loss_bwd(hipStream_t s, const float* ra, const float* a, int64_t na, float* dra, const float* rt, const float* t,
                 int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl, const float* coef, float* dmu,
                 float* dlv) {
    int64_t n = std::max(na, std::max(nt, nl));
    vae_bwd_kernel<<<grid_for(n, kThreads, 4096), kThreads, 0, s>>>(ra, a, na, dra, rt, t, nt, drt, mu, lv, nl, coef,
                                                                     dmu, dlv);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int vae_sums_bwd(hipStream_t s, const float* ra, const float* a, int64_t na, float* dra, const float* rt, const float* t,
                 int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl, const float* coef, float* dmu,
                 float* dlv, double* out3, Ws ws) {
    int nblk = vae_blocks(std::max(na, std::max(nt, nl)));
    HLMC_CHECK_ARG(ws.bytes >= vae_sums_ws(na, nt, nl), "loss workspace");
    double* part = reinterpret_cast<double*>(ws.p);
    vae_sums_bwd_kernel<<<nblk, kThreads, 0, s>>>(ra, a, na, dra, rt, t, nt, drt, mu, lv, nl, coef, dmu, dlv, part);
    HLMC_LAUNCHED();
    vae_sums_finalize_kernel<<<3, 256, 0, s>>>(part, nblk, out3);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

static AdamCoef adam_coef(const AdamArgs& a) {
    const double bc1 = 1.0 - std::pow((double)a.beta1, (double)a.step);
    const double bc2 = 1.0 - std::pow((double)a.beta2, (double)a.step);
    return AdamCoef{a.beta1, a.beta2, a.eps, a.weight_decay, (float)(a.lr / bc1), (float)std::sqrt(bc2)};
}

int adam(hipStream_t s, int ntensors, float* const* p, const float* const* g, float* const* m, float* const* v,
         const int64_t* numel, AdamArgs a) {
    const AdamCoef c = adam_coef(a);
    for (int t0 = 0; t0 < ntensors; t0 += kAdamMax) {
        AdamBatch bt{};
        bt.count = std::min(kAdamMax, ntensors - t0);
        int blocks = 0;
        for (int i = 0; i < bt.count; ++i) {
            bt.p[i] = p[t0 + i]; bt.g[i] = g[t0 + i]; bt.m[i] = m[t0 + i]; bt.v[i] = v[t0 + i];
            bt.n[i] = numel[t0 + i];
            bt.blk0[i] = blocks;
            blocks += (int)((numel[t0 + i] + 1023) / 1024);
        }
        bt.blk0[bt.count] = blocks;
        if (blocks == 0) continue;
        adam_kernel<<<blocks, 256, 0, s>>>(bt, c);
        HLMC_LAUNCHED();
    }
    return HLMC_OK;
}

int adam_job_tiles(AdamJob& j) {
    if (j.taps == 0) {
        j.nt1 = 0;
        return (int)((j.n + 4095) / 4096);
    }
    const int TS = adam_tile_edge(j.taps);
    j.nt1 = (j.d1 + TS - 1) / TS;
    return ((j.d0 + TS - 1) / TS) * j.nt1;
}

void adam_coef_host(const AdamArgs& a, float* out6) {
    const AdamCoef c = adam_coef(a);
    static_assert(sizeof(AdamCoef) == 6 * sizeof(float), "AdamCoef layout");
    std::memcpy(out6, &c, sizeof(c));
}

template <typename T>
int adam_pack(hipStream_t s, const AdamJob* jobs_dev, int njobs, int total_tiles, AdamArgs a, const float* coef_dev,
              int tile_begin) {
    if (njobs == 0 || total_tiles <= tile_begin) return HLMC_OK;
    adam_pack_kernel<T><<<total_tiles - tile_begin, 256, 0, s>>>(jobs_dev, njobs, adam_coef(a),
                                                                 reinterpret_cast<const AdamCoef*>(coef_dev), tile_begin);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <typename T>
int pack(hipStream_t s, const AdamJob* jobs_dev, int njobs, int total_tiles) {
    if (njobs == 0 || total_tiles == 0) return HLMC_OK;
    pack_kernel<T><<<total_tiles, 256, 0, s>>>(jobs_dev, njobs);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

#define INST(T)                                                                                                      \
    template int bn_stats<T>(hipStream_t, const T*, int64_t, int, float*, float*, float*, float*, int64_t*, float,     \
                             float, XAcc);                                                                            \
    template int bn_moments<T>(hipStream_t, const T*, int64_t, int, XAcc);                                             \
    template int bn_act<T>(hipStream_t, const T*, int64_t, int, const float*, const float*, const float*, const float*, \
                           int, const uint8_t*, float, T*, int);                                                      \
    template int bn_act_train<T>(hipStream_t, const T*, int64_t, int, XAcc, bool, float*, float*, float*,            \
                                 float*, int64_t*, float, float, const float*, const float*, int, const uint8_t*, float, \
                                 T*, int);                                                                           \
    template int bn_act_bwd<T>(hipStream_t, const T*, int, const T*, int64_t, int, const float*, const float*,          \
                               const float*, const float*, int, const uint8_t*, float, T*, float*, float*, XAcc,      \
                               const BnBwdFuse*, XAcc, float*, float*);                                              \
    template int conv_c1_s2<T>(hipStream_t, const float*, int, int, int, const float*, const float*, int, T*,        \
                               ColStats*, BnBwdFuse*);                                                               \
    template int convT_c1<T>(hipStream_t, const T*, int, int, int, int, const float*, const float*, float*);         \
    template int wgrad_c1<T>(hipStream_t, const T*, int, int, int, int, const float*, float*, Ws);                    \
    template int cast_from_f32<T>(hipStream_t, const float*, T*, int64_t);                                           \
    template int cast_to_f32<T>(hipStream_t, const T*, float*, int64_t);                                             \
    template int copy2d<T>(hipStream_t, const T*, int, T*, int, int, int);                                           \
    template int cast2d_from_f32<T>(hipStream_t, const float*, int, T*, int, int, int);                              \
    template int nhwc_to_flat<T>(hipStream_t, const T*, int, int, int, int, T*, int, const T*);                      \
    template int flat_to_nhwc<T>(hipStream_t, const T*, int, int, int, int, int, T*);                                \
    template int colsum<T>(hipStream_t, const T*, int, int, int, float*, Ws);                                        \
    template int reparam_fwd<T>(hipStream_t, const float*, const float*, const float*, int, int, T*, int, float*,     \
                                float*, float*);                                                                     \
    template int reparam_rng<T>(hipStream_t, const float*, const float*, uint64_t, uint64_t, int, int, float*, T*, int, \
                                float*, float*);                                                                     \
    template int reparam_bwd<T>(hipStream_t, const T*, int, const float*, const float*, const float*, const float*,  \
                                int, int, T*, T*);                                                                  \
    template int pack<T>(hipStream_t, const AdamJob*, int, int);                                                     \
    template int adam_pack<T>(hipStream_t, const AdamJob*, int, int, AdamArgs, const float*, int);

INST(float)
INST(bf16)
#undef INST

}  // namespace ops
}  // namespace hlmc
