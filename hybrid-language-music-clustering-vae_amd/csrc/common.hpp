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
