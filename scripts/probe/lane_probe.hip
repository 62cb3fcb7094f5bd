// Diagnostic: checks the lane-exchange primitives of the cross-lane FFT (features.hip lane_swap) and the
// buffer-load range check against their assumed semantics; prints PASS/FAIL per primitive.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename F> __device__ __forceinline__ F as_(int v) { return __builtin_bit_cast(F, v); }
__device__ __forceinline__ int bits_(float v) { return __builtin_bit_cast(int, v); }

template <int J>
__device__ __forceinline__ void lane_swap(float& x, float& y, bool lj) {
    if constexpr (J == 5) {
        const auto r = __builtin_amdgcn_permlane32_swap(bits_(x), bits_(y), false, false);
        x = as_<float>(r[0]); y = as_<float>(r[1]);
    } else if constexpr (J == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(bits_(x), bits_(y), false, false);
        x = as_<float>(r[0]); y = as_<float>(r[1]);
    } else if constexpr (J == 3 || J == 2) {
        constexpr int d = 1 << J, hi = J == 3 ? 0xC : 0xA, lo = J == 3 ? 0x3 : 0x5;
        const float nx = as_<float>(__builtin_amdgcn_update_dpp(bits_(x), bits_(y), 0x110 + d, 0xF, hi, false));
        const float ny = as_<float>(__builtin_amdgcn_update_dpp(bits_(y), bits_(x), 0x100 + d, 0xF, lo, false));
        x = nx; y = ny;
    } else {
        constexpr int qp = J == 1 ? 0x4E : 0xB1;
        const float ty = as_<float>(__builtin_amdgcn_mov_dpp(bits_(y), qp, 0xF, 0xF, false));
        const float tx = as_<float>(__builtin_amdgcn_mov_dpp(bits_(x), qp, 0xF, 0xF, false));
        x = lj ? ty : x;
        y = lj ? y : tx;
    }
}

template <int J>
__global__ void probe(float* out) {
    const int l = threadIdx.x;
    float x = l, y = 100 + l;
    lane_swap<J>(x, y, (l >> J) & 1);
    out[l] = x; out[64 + l] = y;
}
__global__ void probe_buf(const float* src, int n, float* out) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, n * 4, 0x00020000);
    const int l = threadIdx.x;
    const int i = l - 32;  // -32..31 over a 16-element buffer
    out[l] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * i, 0, 0));
    const float2 u = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, 4 * (2 * i), 0, 0));
    out[64 + l] = u.x;
    out[128 + l] = u.y;
}

template <int J>
bool run(float* d, float* h) {
    probe<J><<<1, 64>>>(d);
    hipMemcpy(h, d, 128 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const int dd = 1 << J, lj = (l >> J) & 1;
        const float ex = lj ? 100 + (l - dd) : l;
        const float ey = lj ? 100 + l : (l + dd);
        if (h[l] != ex || h[64 + l] != ey) ++bad;
    }
    printf("lane_swap<%d>: %s", J, bad ? "FAIL" : "PASS");
    if (bad) {
        printf("\n  x:");
        for (int l = 0; l < 64; ++l) printf(" %g", h[l]);
        printf("\n  y:");
        for (int l = 0; l < 64; ++l) printf(" %g", h[64 + l]);
    }
    printf("\n");
    return !bad;
}

int main() {
    float *d, h[192];
    hipMalloc(&d, 192 * 4);
    run<5>(d, h); run<4>(d, h); run<3>(d, h); run<2>(d, h); run<1>(d, h); run<0>(d, h);
    float src[16];
    for (int i = 0; i < 16; ++i) src[i] = 1 + i;
    float* ds;
    hipMalloc(&ds, 64 * 4);
    hipMemcpy(ds, src, 16 * 4, hipMemcpyHostToDevice);
    probe_buf<<<1, 64>>>(ds, 16, d);
    hipMemcpy(h, d, 192 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const int i = l - 32;
        const float e = (i >= 0 && i < 16) ? src[i] : 0.f;
        const float e0 = (2 * i >= 0 && 2 * i < 16) ? src[2 * i] : 0.f, e1 = (2 * i + 1 >= 0 && 2 * i + 1 < 16) ? src[2 * i + 1] : 0.f;
        if (h[l] != e || h[64 + l] != e0 || h[128 + l] != e1) ++bad;
    }
    printf("buffer range check: %s\n", bad ? "FAIL" : "PASS");
    if (bad) { for (int l = 0; l < 64; ++l) printf("%d:%g,%g,%g ", l - 32, h[l], h[64 + l], h[128 + l]); printf("\n"); }
    return 0;
}
