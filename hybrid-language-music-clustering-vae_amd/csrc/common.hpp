// Shared device/host helpers for libhlmc (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/hlmc.h"

namespace hlmc {

using bf16 = __hip_bfloat16;
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// ------------------------------------------------------------------ errors
void set_error(const std::string& msg);
const char* get_error();

#define HLMC_CHECK_ARG(cond, msg)                                          \
    do {                                                                   \
        if (!(cond)) {                                                     \
            ::hlmc::set_error(std::string(__func__) + ": " + (msg));       \
            return HLMC_EINVAL;                                            \
        }                                                                  \
    } while (0)

#define HLMC_HIP(...)                                                      \
    do {                                                                   \
        hipError_t e__ = (__VA_ARGS__);                                    \
        if (e__ != hipSuccess) {                                           \
            ::hlmc::set_error(std::string(#__VA_ARGS__) + ": " + hipGetErrorString(e__)); \
            return HLMC_EHIP;                                              \
        }                                                                  \
    } while (0)

#define HLMC_LAUNCHED()                                                    \
    do {                                                                   \
        hipError_t e__ = hipGetLastError();                                \
        if (e__ != hipSuccess) {                                           \
            ::hlmc::set_error(std::string(__func__) + ": launch: " + hipGetErrorString(e__)); \
            return HLMC_EHIP;                                              \
        }                                                                  \
    } while (0)

#define HLMC_TRY(...)                                                      \
    do {                                                                   \
        int s__ = (__VA_ARGS__);                                           \
        if (s__ != HLMC_OK) return s__;                                    \
    } while (0)

// ------------------------------------------------------------------ device status word
// Faults a kernel detects and reports instead of hanging or returning silently wrong values; the kernel writes the bit
// with a system-scope store into pinned, mapped host memory (dev_status_word), the host reads it without synchronising
// (dev_status_take, C ABI hlmc_device_status) and the backward entry points return HLMC_EDEVICE while a bit is raised.
constexpr unsigned kDevBnCountTimeout = 1u;   // bn_bwd_fused_kernel: a block's grid-wide arrival spin ran out
namespace ops {
unsigned* dev_status_word();
unsigned dev_status_take(bool clear);
void test_bn_fused(int64_t max_elems, int spin_max);
}  // namespace ops

// ------------------------------------------------------------------ live kernel timing (bench.py roofline)
// An op sets the site (its kind and ALGORITHMIC flops / HBM bytes) before its launcher runs; when the kind is
// in the armed mask (hlmc_probe_arm) the launcher brackets its main kernel with a HIP event pair on the launch
// stream.  Off (mask 0) it costs one branch per launch.
namespace probe {
enum : int { kConvS2 = 1, kSubpixel = 2, kWgradS2 = 4, kLinear = 8, kLinearWgrad = 16, kStftMel = 32, kBn = 64 };
struct Site {
    int kind;
    double flops, bytes;
};
extern int g_mask;
extern Site g_site;
void begin(hipStream_t s);
void end(hipStream_t s);
inline void site(int kind, double flops, double bytes) { g_site = Site{kind, flops, bytes}; }
}  // namespace probe
#define HLMC_PROBE_BEGIN(s) \
    do { if (::hlmc::probe::g_mask & ::hlmc::probe::g_site.kind) ::hlmc::probe::begin(s); } while (0)
#define HLMC_PROBE_END(s) \
    do { if (::hlmc::probe::g_mask & ::hlmc::probe::g_site.kind) ::hlmc::probe::end(s); ::hlmc::probe::g_site.kind = 0; } while (0)

// ------------------------------------------------------------------ scalar conversions
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16>(bf16 v) { return __bfloat162float(v); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return __float2bfloat16(v); }

// 16-byte vector of T: 8 bf16 or 4 f32
template <typename T> struct Vec16;
template <> struct Vec16<float> { static constexpr int N = 4; };
template <> struct Vec16<bf16> { static constexpr int N = 8; };

// 16 raw bytes -> f32 values (4 floats or 8 bf16)
template <typename T>
__device__ __forceinline__ void cvt16_f32(uint4 v, float* out) {
    if constexpr (sizeof(T) == 4) {
        out[0] = __uint_as_float(v.x); out[1] = __uint_as_float(v.y);
        out[2] = __uint_as_float(v.z); out[3] = __uint_as_float(v.w);
    } else {
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            out[2 * i] = __uint_as_float(w[i] << 16);
            out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    }
}
template <typename T>
__device__ __forceinline__ void load16_f32(const T* p, float* out) {
    cvt16_f32<T>(*reinterpret_cast<const uint4*>(p), out);
}
template <typename T>
__device__ __forceinline__ uint4 load16_raw(const T* p) { return *reinterpret_cast<const uint4*>(p); }

template <typename T>
__device__ __forceinline__ void store16_f32(T* p, const float* in) {
    if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<uint4*>(p) = make_uint4(__float_as_uint(in[0]), __float_as_uint(in[1]),
                                                  __float_as_uint(in[2]), __float_as_uint(in[3]));
    } else {
        unsigned w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bf16 lo = __float2bfloat16(in[2 * i]);
            bf16 hi = __float2bfloat16(in[2 * i + 1]);
            w[i] = (unsigned)(*reinterpret_cast<unsigned short*>(&lo)) |
                   ((unsigned)(*reinterpret_cast<unsigned short*>(&hi)) << 16);
        }
        *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : 0.01f * x; }

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Division by a runtime constant via a precomputed magic number (n < 2^31): q = (umulhi(n, mul) + n) >> sh
struct FastDiv {
    uint32_t d, mul, sh;
    FastDiv() = default;
    explicit FastDiv(uint32_t div) : d(div) {
        sh = 0;
        while ((1u << sh) < div) ++sh;
        mul = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << sh) - div)) / div + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, mul) + n) >> sh; }
};


// ------------------------------------------------------------------ exact column-sum accumulators
// Per-column sums that many blocks of one launch contribute to (BatchNorm batch statistics, backward moments, bias
// gradients), delivered straight from the producing blocks instead of as per-block f64 rows that a separate fold
// launch reduces.  Each block's f64 partial v is split into three integer words -- floor(v), the next 32 fraction
// bits, the 32 after those (bits below 2^-64 truncated; |v| clamped below 2^62) -- and added with no-return agent-scope
// int64 atomics (performed at the memory side, coherent across the XCDs).  Integer addition is associative, so the
// totals are bit-identical whatever order the blocks arrive in (deterministic), and exact: the only rounding is the
// consumer's single conversion back to f64.  Blocks spread their adds over `shards` copies (block id mod shards) so
// that no address sees more than a few dozen adders.  Layout: [shards][3 words][ncols] int64, zeroed before the
// producer runs (one memset per pass for all of a pass's accumulators); the consumer sums the shards' words.
struct XAcc {
    unsigned long long* p = nullptr;
    int shards = 0;
    int ncols = 0;
    __host__ __device__ bool on() const { return p != nullptr; }
    static size_t bytes(int shards, int ncols) { return (size_t)shards * 3 * ncols * 8; }
};
// shards for a BatchNorm pair table (2C columns): the consumer folds shards x 6C words per block, so fewer shards for
// wider layers (whose producers also have fewer blocks)
// accumulator copies per layer (block id mod shards): fewer atomics on one address vs more words for the consumers
// to fold (xacc_fold handles <= 8 shards when 2C >= 256 columns).  Round 4: 4 / 8 / 8 for C >= 512 / 256 / 128 (was
// 2 / 4 / 8) measured 133.9k vs 133.4k clips/s (4 rounds; 8 / 8 / 8: 133.3k)
inline int xacc_shards(int C) { return C >= 512 ? 4 : C >= 128 ? 8 : 16; }
constexpr int kXAccMaxShards = 16;

// A non-finite partial (NaN, inf, or beyond the +-4e18 range the integer word holds) sets bit 63 of the shard's
// third word instead (sticky: that word's adds total < 2^48, so no add reaches bit 63); the readers below return NaN
// for such a column, as torch's statistics of a diverged run would be, instead of finite garbage.
constexpr unsigned long long kXAccBad = 1ull << 63;
__device__ __forceinline__ void xacc_add_shard(const XAcc& x, int shard, int col, double v) {
    unsigned long long* b = x.p + (size_t)shard * 3 * x.ncols + col;
    if (!(fabs(v) <= 4.0e18)) {
        atomicOr(b + 2 * x.ncols, kXAccBad);
        return;
    }
    const double f = floor(v);
    const double r1 = (v - f) * 4294967296.0;  // exact: v - floor(v) and power-of-two scales
    const double g = floor(r1);
    const double r2 = (r1 - g) * 4294967296.0;
    atomicAdd(b, (unsigned long long)(long long)f);
    atomicAdd(b + x.ncols, (unsigned long long)(long long)g);
    atomicAdd(b + 2 * x.ncols, (unsigned long long)(long long)floor(r2));
}
__device__ __forceinline__ void xacc_add(const XAcc& x, int col, double v) {
    xacc_add_shard(x, (int)(blockIdx.x % (unsigned)x.shards), col, v);
}
__device__ __forceinline__ double xacc_value(long long a, long long b, long long c) {
    return (double)a + ((double)b * 0x1p-32 + (double)c * 0x1p-64);
}
// column c of an exact accumulator, summed over its shards (one thread)
__device__ __forceinline__ double xacc_column(const XAcc& acc, int c) {
    long long a = 0, b = 0, d = 0;
    unsigned long long bad = 0;
    for (int sh = 0; sh < acc.shards; ++sh) {
        const unsigned long long* q = acc.p + (size_t)sh * 3 * acc.ncols + c;
        a += (long long)q[0];
        b += (long long)q[acc.ncols];
        bad |= q[2 * acc.ncols] & kXAccBad;
        d += (long long)(q[2 * acc.ncols] & ~kXAccBad);
    }
    return bad ? __builtin_nan("") : xacc_value(a, b, d);
}
// out[c] (LDS, c < ncols) = the accumulator's column totals; every thread of the block calls it (blockDim.x == NT);
// red: LDS scratch of >= 3 * NT int64 (used when ncols < NT).  Thread (column c, shard group g) issues the loads of
// all its shards at once (<= 8 shards x 3 words in flight; clamped addresses, masked adds).  Ends with a barrier.
template <int NT = 256>
__device__ __forceinline__ void xacc_fold(const XAcc& x, double* out, long long* red) {
    constexpr int K = 8;  // shards per thread group (shards <= K * G, checked by the launchers via xacc_shards)
    const int tid = threadIdx.x, n = x.ncols, S = x.shards;
    const int G = n >= NT ? 1 : NT / n;
    // the third word's bad bit (xacc_add_shard) rides along as bit 63 of the group's d total: the d words' adds total
    // < 2^48, so the masked sum never reaches it and OR-ing the flags back in keeps it
    auto sum = [&](int c, int g, long long& a, long long& b, long long& d) {
        unsigned long long w0[K], w1[K], w2[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int sh = min(g + k * G, S - 1);
            const unsigned long long* q = x.p + (size_t)sh * 3 * n + c;
            w0[k] = q[0];
            w1[k] = q[n];
            w2[k] = q[2 * n];
        }
        a = b = d = 0;
        unsigned long long bad = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (g + k * G < S) {
                a += (long long)w0[k];
                b += (long long)w1[k];
                bad |= w2[k] & kXAccBad;
                d += (long long)(w2[k] & ~kXAccBad);
            }
        d = (long long)((unsigned long long)d | bad);
    };
    auto value = [](long long a, long long b, long long d) {
        return ((unsigned long long)d & kXAccBad) ? __builtin_nan("") : xacc_value(a, b, d);
    };
    if (n >= NT) {
        for (int c = tid; c < n; c += NT) {
            long long a, b, d;
            sum(c, 0, a, b, d);
            out[c] = value(a, b, d);
        }
    } else {
        const int c = tid % n, g = tid / n;
        long long a = 0, b = 0, d = 0;
        if (g < G) sum(c, g, a, b, d);
        red[tid] = a;
        red[NT + tid] = b;
        red[2 * NT + tid] = d;
        __syncthreads();
        if (tid < n) {
            unsigned long long bad = (unsigned long long)d & kXAccBad;
            d = (long long)((unsigned long long)d & ~kXAccBad);
            for (int k = 1; k < G; ++k) {
                a += red[k * n + tid];
                b += red[NT + k * n + tid];
                const unsigned long long dk = (unsigned long long)red[2 * NT + k * n + tid];
                bad |= dk & kXAccBad;
                d += (long long)(dk & ~kXAccBad);
            }
            out[tid] = bad ? __builtin_nan("") : xacc_value(a, b, d);
        }
    }
    __syncthreads();
}

// wave-level sums (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace hlmc
