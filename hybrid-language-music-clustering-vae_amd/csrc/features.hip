// Audio features on gfx950: framed STFT -> |X|^2 -> Slaney mel -> dB (-> DCT-II MFCC), mean/std
// pooling and the StandardScaler fit/apply.  Replaces librosa / sklearn calls of
// src/1_preprocessing.py:48-70,115-121,305-311 and src/1_preprocessing_advanced.py:97-114,376-391.
//
// STFT kernel: one 256-thread workgroup per (clip, 16 frames), one wavefront per frame.  A 2048-point
// real frame is packed into a 1024-point complex sequence (even/odd samples), transformed with a
// register-resident radix-16/16/4 Stockham FFT, and split back into the 1025 real-FFT bins.  Window / twiddle tables are built on the host in double precision.  The Slaney filterbank is
// banded (each filter spans 4..53 bins) and stored as (first bin, count, weights) per mel band.
#include <algorithm>
#include <cmath>
#include <vector>

#include "features.hpp"

namespace hlmc {



namespace {

// ---------------------------------------------------------------- librosa.filters.mel (host, double)
double hz_to_mel(double f) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}
std::vector<float> slaney_filterbank(int sr, int n_fft, int n_mels, double fmin, double fmax) {
    const int nb = 1 + n_fft / 2;
    std::vector<float> w((size_t)n_mels * nb, 0.f);
    std::vector<double> fft(nb), melf(n_mels + 2);
    for (int i = 0; i < nb; ++i) fft[i] = (double)i * sr / n_fft;
    const double lo = hz_to_mel(fmin), hi = hz_to_mel(fmax);
    for (int i = 0; i < n_mels + 2; ++i) melf[i] = mel_to_hz(lo + (hi - lo) * i / (double)(n_mels + 1));
    for (int m = 0; m < n_mels; ++m) {
        const double d0 = melf[m + 1] - melf[m], d1 = melf[m + 2] - melf[m + 1];
        const float enorm = (float)(2.0 / (melf[m + 2] - melf[m]));
        for (int f = 0; f < nb; ++f) {
            const double lower = -(melf[m] - fft[f]) / d0;
            const double upper = (melf[m + 2] - fft[f]) / d1;
            const float v = (float)std::max(0.0, std::min(lower, upper));
            w[(size_t)m * nb + f] = v * enorm;  // float32 weights *= float32(enorm) as librosa does in place
        }
    }
    return w;
}

constexpr int kFFT = 1024;  // complex points (n_fft = 2048 real)

// complex product with two explicit fma (this file builds with -ffp-contract=off for the numpy-order dB / feature
// arithmetic, so the FFT's contractions are spelled out: 4 VALU ops instead of 6)
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}

// ---------------------------------------------------------------- STFT -> |X|^2 -> mel, one wavefront per frame
// A 2048-sample real frame is packed into z[n] = x[2n] w[2n] + i x[2n+1] w[2n+1] (n < 1024) and transformed
// as 1024 = 16 x 64 (four-step): lane p holds z[p + 64 r] (r < 16); a radix-16 DFT over r runs in registers,
// the twiddles W1024^{p k1} follow, and the 64-point DFTs over the lanes run as six radix-2 decimation-in-
// frequency stages whose exchanges never touch LDS.  Each stage swaps the lane bit it works on with a
// register bit (v_permlane32_swap / v_permlane16_swap for lane bits 5 and 4, DPP row shifts under bank masks
// for bits 3 and 2, quad permutes for bits 1 and 0), after which every lane holds both inputs of its
// butterflies.  The real-FFT split reads the conjugate partner with one ds_bpermute per word; the 1025 power
// bins go to a wave-private LDS row in natural order, and lane l accumulates the banded Slaney filters
// (l, n_mels-1-l).  Twiddles come from double-precision host tables.
constexpr int kWaves = 4;      // frames in flight per workgroup
constexpr int kFpw = 4;        // frames per wave
constexpr int kFpb = kWaves * kFpw;
constexpr int kPwRow = kFFT + 4;    // power row (floats, 16-byte aligned)
constexpr int kTwB = 15 * 64;       // W1024^{p k1}, k1 = 1..15
constexpr int kTwC = 5 * 64;        // radix-2 stage twiddles, lane bits 1..5
constexpr int kMelLanes = 64;  // band pairs (n_mels <= 128)
constexpr int kMaxWLds = 16384;     // filterbank bytes held in LDS (chunk-transposed); larger tables stay in global
constexpr int64_t kMaxStftSamples = int64_t(1) << 29;  // clip length: byte offsets of the buffer loads fit 31 bits

template <typename F>
__device__ __forceinline__ F as_(int v) { return __builtin_bit_cast(F, v); }
__device__ __forceinline__ int bits_(float v) { return __builtin_bit_cast(int, v); }

// Exchange lane bit J with the register bit that tells x (bit 0) from y (bit 1): afterwards x[l] holds the old
// (l_J ? y[l - 2^J] : x[l]) and y[l] the old (l_J ? y[l] : x[l + 2^J]).
template <int J>
__device__ __forceinline__ void lane_swap(float& x, float& y, bool lj) {
    if constexpr (J == 5) {
        const auto r = __builtin_amdgcn_permlane32_swap(bits_(x), bits_(y), false, false);
        x = as_<float>(r[0]); y = as_<float>(r[1]);
    } else if constexpr (J == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(bits_(x), bits_(y), false, false);
        x = as_<float>(r[0]); y = as_<float>(r[1]);
    } else if constexpr (J == 3 || J == 2) {
        // row_shr / row_shl by 2^J; bank_mask keeps the lanes whose bit J already matches
        constexpr int d = 1 << J, hi = J == 3 ? 0xC : 0xA, lo = J == 3 ? 0x3 : 0x5;
        const float nx = as_<float>(__builtin_amdgcn_update_dpp(bits_(x), bits_(y), 0x110 + d, 0xF, hi, false));
        const float ny = as_<float>(__builtin_amdgcn_update_dpp(bits_(y), bits_(x), 0x100 + d, 0xF, lo, false));
        x = nx; y = ny;
    } else {
        constexpr int qp = J == 1 ? 0x4E : 0xB1;  // quad_perm lane ^ 2 / lane ^ 1
        // (bound_ctrl set, all quad sources valid: lets the compiler fold the move into the select as its DPP source)
        const float ty = as_<float>(__builtin_amdgcn_mov_dpp(bits_(y), qp, 0xF, 0xF, true));
        const float tx = as_<float>(__builtin_amdgcn_mov_dpp(bits_(x), qp, 0xF, 0xF, true));
        x = lj ? ty : x;
        y = lj ? y : tx;
    }
}
// Lanes of one wavefront exchange data through LDS without a workgroup barrier: a wavefront-scope
// release/acquire pair around wave_barrier orders the exchange's writes before the other lanes' reads.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // -i * a

// y_k = sum_n a_n (-i)^{nk}
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = mul_mi(csub(a1, a3));
    a0 = cadd(s02, s13);
    a1 = cadd(d02, d13);
    a2 = csub(s02, s13);
    a3 = csub(d02, d13);
}
// 16-point DFT in place (output in slot order, see slot16): n = 4 n1 + n2, k = k1 + 4 k2
__device__ __forceinline__ void dft16(float2 (&a)[16]) {
    constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508977f, h = 0.70710678118654752f;
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(a[n2], a[4 + n2], a[8 + n2], a[12 + n2]);
    // twiddles W16^{n2 k1}: slot 4 k1 + n2 holds column n2, row k1
    // W^2 = h(1 - i) and W^6 = -h(1 + i): an add and a scale per component
    auto w2 = [&](float2 v) { return make_float2(h * (v.x + v.y), h * (v.y - v.x)); };
    auto w6 = [&](float2 v) { return make_float2(h * (v.y - v.x), -h * (v.x + v.y)); };
    a[5] = cmul(a[5], make_float2(c1, -s1));    // n2=1,k1=1: W^1
    a[9] = w2(a[9]);                            // n2=1,k1=2: W^2
    a[13] = cmul(a[13], make_float2(s1, -c1));  // n2=1,k1=3: W^3
    a[6] = w2(a[6]);                            // n2=2,k1=1: W^2
    a[10] = mul_mi(a[10]);                      // n2=2,k1=2: W^4
    a[14] = w6(a[14]);                          // n2=2,k1=3: W^6
    a[7] = cmul(a[7], make_float2(s1, -c1));    // n2=3,k1=1: W^3
    a[11] = w6(a[11]);                          // n2=3,k1=2: W^6
    a[15] = cmul(a[15], make_float2(-c1, s1));  // n2=3,k1=3: W^9
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) dft4(a[4 * k1], a[4 * k1 + 1], a[4 * k1 + 2], a[4 * k1 + 3]);
    // slot 4 k1 + k2 now holds X[k1 + 4 k2]; callers read X[r] from a[slot16(r)]
}
__device__ __forceinline__ constexpr int slot16(int r) { return 4 * (r & 3) + (r >> 2); }

// librosa.feature.spectral_centroid / spectral_bandwidth / spectral_rolloff of one frame from its power bins
// pw[0..1024] (wave-private LDS).  S_k = sqrt(pw_k) (power = 1), f_k = k sr / n_fft; librosa normalises
// S / sum(S) in float32 (left unnormalised when the sum is below float32 tiny) and sums freq * S_norm in
// float64.  Lane l owns bins 16 l .. 16 l + 15 (contiguous, for the rolloff prefix sum); lane 63 also owns
// the Nyquist bin 1024.  out[0], out[T], out[2T] <- centroid, bandwidth, rolloff (Hz).
__device__ __forceinline__ void spectral_shape(const float* pw, int ln, double bin_hz, double roll, double* out, int T) {
    const float4* pw4 = reinterpret_cast<const float4*>(pw);
    float m[17];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float4 v = pw4[4 * ln + c];
        m[4 * c] = sqrtf(v.x); m[4 * c + 1] = sqrtf(v.y); m[4 * c + 2] = sqrtf(v.z); m[4 * c + 3] = sqrtf(v.w);
    }
    m[16] = ln == 63 ? sqrtf(pw[kFFT]) : 0.f;
    double sl = 0.0;
#pragma unroll
    for (int j = 0; j < 17; ++j) sl += (double)m[j];
    const double total = wave_sum(sl);
    const float tot32 = (float)total;
    const float div = tot32 < 1.17549435e-38f ? 1.f : tot32;
    const int k0 = 16 * ln;
    auto fk = [&](int j) { return (double)(j < 16 ? k0 + j : kFFT) * bin_hz; };
    double cl = 0.0;
#pragma unroll
    for (int j = 0; j < 17; ++j) cl += (double)(m[j] / div) * fk(j);
    const double centroid = wave_sum(cl);
    double bl = 0.0;
#pragma unroll
    for (int j = 0; j < 17; ++j) {
        const double d = fk(j) - centroid;
        bl += (double)(m[j] / div) * (d * d);
    }
    const double bandwidth = sqrt(wave_sum(bl));
    // rolloff: first bin whose cumulative magnitude reaches roll * total (wave exclusive scan of lane sums)
    double inc = sl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double t = __shfl_up(inc, o, 64);
        if (ln >= o) inc += t;
    }
    const double thr = roll * total;
    double cum = inc - sl;
    int first = 1 << 30;
#pragma unroll
    for (int j = 0; j < 17; ++j) {
        cum += (double)m[j];
        const int k = j < 16 ? k0 + j : kFFT;
        if (cum >= thr && (j < 16 || ln == 63)) first = min(first, k);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
    if (ln == 0) {
        out[0] = centroid;
        out[T] = bandwidth;
        out[2 * T] = (double)first * bin_hz;
    }
}

// librosa.feature.zero_crossing_rate(frame_length, hop, center=True: edge padding, threshold 1e-10,
// zero_pos=True) and librosa.feature.rms(frame_length, hop, center=True: zero padding), one wavefront per frame.
// Lane l holds samples 4 (l + 64 r) + c (r < 8 for frame_length 2048): coalesced float4 loads.
constexpr int kZrFrame = 2048;
__global__ __launch_bounds__(256) void zcr_rms_kernel(const float* __restrict__ pcm, int64_t n, int T, int hop,
                                                      double* __restrict__ zcr, float* __restrict__ rms) {
    constexpr int R = kZrFrame / 256;  // float4 groups per lane
    const int b = blockIdx.y;
    const int wave = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const float* x = pcm + (int64_t)b * n;
    for (int t = blockIdx.x * 16 + wave; t < min(T, (int)blockIdx.x * 16 + 16); t += 4) {
        const int64_t start = (int64_t)t * hop - kZrFrame / 2;
        const bool interior = start >= 0 && start + kZrFrame <= n && ((reinterpret_cast<uintptr_t>(x + start) & 15) == 0);
        float4 e[R];  // edge-padded samples
        double sq = 0.0;
        if (interior) {
            const float4* xs = reinterpret_cast<const float4*>(x + start);
#pragma unroll
            for (int r = 0; r < R; ++r) e[r] = xs[ln + 64 * r];
#pragma unroll
            for (int r = 0; r < R; ++r)
                sq += (double)(e[r].x * e[r].x) + (double)(e[r].y * e[r].y) + (double)(e[r].z * e[r].z) + (double)(e[r].w * e[r].w);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float v[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int64_t i = start + 4 * (ln + 64 * r) + c;
                    const float xv = x[min(max(i, (int64_t)0), n - 1)];
                    v[c] = xv;
                    const float z = (i >= 0 && i < n) ? xv : 0.f;
                    sq += (double)(z * z);
                }
                e[r] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        // signbit after |y| <= 1e-10 -> +0
        auto neg = [](float v) -> int { return (fabsf(v) <= 1e-10f) ? 0 : (int)(__float_as_uint(v) >> 31); };
        int cnt = 0;
        int up_prev = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int s0 = neg(e[r].x), s1 = neg(e[r].y), s2 = neg(e[r].z), s3 = neg(e[r].w);
            cnt += (s0 != s1) + (s1 != s2) + (s2 != s3);
            const int up = __shfl(s3, (ln + 63) & 63, 64);  // last sign of the previous float4 group
            if (ln > 0) cnt += (up != s0);
            else if (r > 0) cnt += (up_prev != s0);     // lane 63 of group r - 1
            up_prev = up;
        }
        double c = (double)cnt;
        c = wave_sum(c);
        sq = wave_sum(sq);
        if (ln == 0) {
            zcr[(int64_t)b * T + t] = c / (double)kZrFrame;
            rms[(int64_t)b * T + t] = sqrtf((float)(sq / (double)kZrFrame));
        }
    }
}

// ---------------------------------------------------------------- chroma_stft (librosa.feature.chroma_stft)
// Pass A (stft_mel_kernel<2>): per frame, the power bins S (stored [b][t][kSRow] for pass C) and
// librosa.piptrack(S=S, fmin=150, fmax=4000, threshold=0.1): ref = 0.1 * max_k S_k; peaks are bins of the
// frequency mask where x = S * (S > ref) is a local maximum (x_k > x_{k-1}, x_k >= x_{k+1}); parabolic
// interpolation a = S_{k+1} + S_{k-1} - 2 S_k, b = (S_{k+1} - S_{k-1}) / 2, shift = |b| >= |a| ? 0 : -b / a
// (f64, stored f32), pitch = f32((k + shift) sr / n_fft), mag = S_k + 0.5 avg shift with avg = np.gradient(S).
// Peaks are compacted per frame (bin order) into cand[b][t][maxpk].
constexpr int kSRow = 1028;   // power row stride (floats, 16-byte aligned)
struct PipArgs {
    float* S;
    float2* cand;   // (pitch, mag)
    int* cnt;       // peaks per frame
    int kmin, kmax; // frequency mask [kmin, kmax)
    int maxpk;      // slots per frame: >= peaks per frame (at most every other masked bin)
    double sr;
    int n_fft;
};

__device__ __forceinline__ void piptrack_frame(const float* pw, int ln, const PipArgs& pa, int64_t row) {
    const float4* pw4 = reinterpret_cast<const float4*>(pw);
    float4* dst = reinterpret_cast<float4*>(pa.S + row * kSRow);
    for (int i = ln; i < 256; i += 64) dst[i] = pw4[i];
    if (ln == 0) dst[256] = make_float4(pw[kFFT], 0.f, 0.f, 0.f);
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) m = fmaxf(m, pw[16 * ln + j]);
    if (ln == 63) m = fmaxf(m, pw[kFFT]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const float ref = 0.1f * m;
    auto thr = [&](float v) { return v > ref ? v : 0.f; };
    auto is_peak = [&](int k) {
        if (k < pa.kmin || k >= pa.kmax) return false;
        const float x = thr(pw[k]);
        return x > thr(pw[k - 1]) && x >= thr(pw[k + 1]);
    };
    int n = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) n += is_peak(16 * ln + j) ? 1 : 0;
    int inc = n;  // inclusive scan of the per-lane counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (ln >= o) inc += t;
    }
    int slot = inc - n;
    float2* out = pa.cand + row * pa.maxpk;
    for (int j = 0; j < 16; ++j) {
        const int k = 16 * ln + j;
        if (!is_peak(k) || slot >= pa.maxpk) continue;
        const float s0 = pw[k], sl = pw[k - 1], sr = pw[k + 1];
        // librosa >= 0.10 numba stencil: f32 sums promoted to f64 by the integer constants
        const double a = (double)(sr + sl) - 2.0 * (double)s0;
        const double bb = (double)(sr - sl) / 2.0;
        const float shift = fabs(bb) >= fabs(a) ? 0.f : (float)(-bb / a);
        const float pitch = (float)(((double)k + (double)shift) * pa.sr / (double)pa.n_fft);
        const float avg = (sr - sl) / 2.f;  // np.gradient (float32)
        const float mag = s0 + (0.5f * avg) * shift;
        out[slot++] = make_float2(pitch, mag);
    }
    if (ln == 63) pa.cnt[row] = min(inc, pa.maxpk);
}

// Radix-2 decimation-in-frequency stage on lane bit J of the 64-point lane DFTs: swap lane bit J into register
// bit RB, then each lane forms both outputs of its butterflies in registers, (u + v) and (u - v) W.
template <int J, int RB>
__device__ __forceinline__ void lane_stage(float2 (&b)[16], float2 tw, bool lj) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (r & (1 << RB)) continue;
        float2& x = b[r];
        float2& y = b[r | (1 << RB)];
        lane_swap<J>(x.x, y.x, lj);
        lane_swap<J>(x.y, y.y, lj);
        const float2 s = cadd(x, y), d = csub(x, y);
        x = s;
        y = J == 0 ? d : cmul(d, tw);
    }
}
// After the six stages (lane bits 5,4,3,2,1,0 swapped with register bits 3,2,1,0,3,2) register r of lane l holds
// X[bin_lane(l) + 64 bin_reg(r)].
__device__ __forceinline__ constexpr int bin_reg(int r) { return ((r >> 1) & 1) | (r & 1) << 1 | ((r >> 3) & 1) << 2 | ((r >> 2) & 1) << 3; }
__device__ __forceinline__ int bin_lane(int l) { return (l >> 2) | ((l >> 1) & 1) << 4 | (l & 1) << 5; }
__device__ __forceinline__ int lane_of_bin(int g) { return ((g & 15) << 2) | ((g >> 4) & 1) << 1 | ((g >> 5) & 1); }

// kMode 0: banded mel (stored [b][m][t]) + per-clip max/min; kWL: filterbank staged in LDS.  kMode 1: spectral
// shape of |X| (power 1): centroid, bandwidth (p = 2) and rolloff per frame, stored f64 [b][3][t] (sout).
// kMode 2: piptrack (PipArgs).  Modes 1 and 2 leave the mel tables unused.
template <int kMode, bool kWL, bool kPairs>
__device__ __forceinline__ void stft_mel_body(const float* __restrict__ pcm, int nclips, int64_t n_samples, int T,
                                                       int hop, const float* __restrict__ window,
                                                       const float2* __restrict__ rtw, const float2* __restrict__ tw,
                                                       const int* __restrict__ band,
                                                       const int* __restrict__ woff, const float* __restrict__ wts,
                                                       int n_mels, int nnz, float* __restrict__ out,
                                                       unsigned* __restrict__ clip_max, unsigned* __restrict__ clip_min,
                                                       double bin_hz, double roll, double* __restrict__ sout,
                                                       PipArgs pa) {
    // LDS: FFT twiddles + one power row per wave (27 KB static); dynamic: band info, the chunk-transposed
    // filterbank (kWL, 16 KB at n_mels = 128) and the mel staging rows: 52 KB in all, 3 blocks per CU.
    __shared__ float2 stw[kTwB + kTwC];
    __shared__ __align__(16) float pwb[kWaves][kPwRow];
    extern __shared__ int4 sbl[];
    float4* swt = reinterpret_cast<float4*>(sbl + kMelLanes);
    float* smel = reinterpret_cast<float*>(swt + (kWL ? nnz / 4 : 0));
    const float4* __restrict__ gw4 = reinterpret_cast<const float4*>(wts);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // Persistent blocks over the (clip, 16-frame group) items.  Blocks are dispatched round-robin over the 8
    // XCDs; XCD k walks the contiguous item range [k n / 8, (k + 1) n / 8), so neighbouring groups of a clip (their
    // frames share 1536 samples) run on one L2.  The tables are staged once per block, and each wave prefetches its
    // first frame of the next item while it finishes the current one.
    const int ng = (T + kFpb - 1) / kFpb;
    const int nitems = nclips * ng;
    const int xcd = blockIdx.x & 7, per = gridDim.x >> 3;
    const int hi = (int)((int64_t)nitems * (xcd + 1) / 8);
    int it = (int)((int64_t)nitems * xcd / 8) + (int)(blockIdx.x >> 3);
    // raw sample pairs (x[2n], x[2n+1]) of frame t: n = lane + 64 r, through a buffer descriptor over the clip
    // whose range check returns 0 outside it (center padding; negative offsets wrap past the range).  With an
    // even clip length and hop a pair never straddles the clip's end, so one 8-byte load per pair.
    // kPairs (launch-time choice, not a runtime branch): every fetch issues the same number of loads on every path,
    // so the compiler's wait counts at the frame loop's merge points stay exact (a conditional fetch made it wait
    // for the next frame's loads before using the current frame's, exposing their latency every frame)
    auto fetch = [&](const float* x, int t, int ln, float2 (&v)[16]) {
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, (int)(n_samples * 4), 0x00020000);
        const int start = t * hop - kFFT;  // center=True: n_fft/2 = 1024 zeros of padding
        if constexpr (kPairs) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                // (bit_cast of the whole vector: extracting the builtin's elements one by one read word 0 twice)
                v[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsrc, 4 * (start + 2 * (ln + 64 * r)), 0, 0));
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i0 = start + 2 * (ln + 64 * r);
                v[r].x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, 4 * i0, 0, 0));
                v[r].y = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, 4 * i0 + 4, 0, 0));
            }
        }
    };
    float2 nxt[16];
    bool have = false;  // nxt holds this wave's first frame of item `it`
    {  // first frame in flight while the tables are staged (unconditional loads: frame 0 of clip 0 when none)
        const int b = it < hi ? it / ng : 0, t0 = it < hi ? (it - b * ng) * kFpb : 0;
        have = it < hi && wave < min(kFpb, T - t0);
        fetch(pcm + (int64_t)b * n_samples, have ? t0 + wave : 0, lane, nxt);
    }
    for (int i = threadIdx.x; i < kTwB + kTwC; i += 256) stw[i] = tw[i];
    if constexpr (kMode == 0) {
        for (int l = threadIdx.x; l < kMelLanes; l += 256) sbl[l] = reinterpret_cast<const int4*>(band)[l];
        if constexpr (kWL)
            for (int i = threadIdx.x; i < nnz / 4; i += 256) swt[i] = gw4[i];
    }
    __syncthreads();
    float* pw = pwb[wave];
    // per-lane constants: this lane's bins, its conjugate partner's lane, the split twiddle base, stage twiddles,
    // the window (frame-invariant, in registers)
    const int fl = bin_lane(lane);
    const int paddr = 4 * lane_of_bin((64 - fl) & 63);
    const float2 wl = rtw[fl];
    float2 tc[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) tc[j] = stw[kTwB + 64 * j + lane];
    const bool l0 = lane & 1, l1 = lane & 2;
    float2 wnd[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) wnd[r] = *reinterpret_cast<const float2*>(window + 2 * (lane + 64 * r));
    for (; it < hi; it += per) {
        const int b = it / ng, t0 = (it - b * ng) * kFpb, nf = min(kFpb, T - t0);
        const float* x = pcm + (int64_t)b * n_samples;
        const int nit = it + per;
        if (!have && wave < nf) {  // (rare: this wave had no frame in its previous item) fetch and wait here, so the
            fetch(x, t0 + wave, lane, nxt);  // loop's wait counts see no loads pending from this path
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        have = false;
        float lmax = 0.f, lmin = INFINITY;
        for (int fi = wave; fi < nf; fi += kWaves) {
            int ln = lane;
            asm volatile("" : "+v"(ln));
            float2 a[16];
            // ---- radix 16 over r in registers: z[ln + 64 r] = windowed sample pairs (prefetched one frame ahead)
    #pragma unroll
            for (int r = 0; r < 16; ++r) {
                a[r] = make_float2(nxt[r].x * wnd[r].x, nxt[r].y * wnd[r].y);
            }
            {  // the next frame of this item, else this wave's first frame of the next item, else (data unused) this one
                int fb = b, ft = t0 + fi;
                if (fi + kWaves < nf) {
                    ft = t0 + fi + kWaves;
                } else if (nit < hi) {
                    const int nb = nit / ng, nt0 = (nit - nb * ng) * kFpb;
                    if (wave < min(kFpb, T - nt0)) {
                        fb = nb;
                        ft = nt0 + wave;
                        have = true;
                    }
                }
                fetch(pcm + (int64_t)fb * n_samples, ft, ln, nxt);
            }
            dft16(a);
            float2 v[16];
            v[0] = a[slot16(0)];
    #pragma unroll
            for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(a[slot16(k1)], stw[(k1 - 1) * 64 + ln]);
            // ---- 64-point DFTs over the lanes (one per k1): six radix-2 DIF stages, lane exchanges in registers
            lane_stage<5, 3>(v, tc[4], false);
            lane_stage<4, 2>(v, tc[3], false);
            lane_stage<3, 1>(v, tc[2], false);
            lane_stage<2, 0>(v, tc[1], false);
            lane_stage<1, 3>(v, tc[0], l1);
            lane_stage<0, 2>(v, tc[0], l0);
            // ---- real-FFT split, 2 X[f] = (Z[f] + Z*[N-f]) + e^{-2 pi i f / 2048} (-i)(Z[f] - Z*[N-f]), f = fl + 64 m:
            // the partner N - f sits in lane lane_of_bin(64 - fl), register r ^ 15 (lane 0: its own register for
            // (16 - m) mod 16, as bins 0, 64, ... pair among themselves)
            float2 wlf = wl;  // opaque per frame: the 14 products wl W32^m would otherwise be hoisted (28 VGPRs)
            asm volatile("" : "+v"(wlf.x), "+v"(wlf.y));
            float p[16];
    #pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = bin_reg(r);
                const float2 zf = v[r];
                float2 zc;
                zc.x = as_<float>(__builtin_amdgcn_ds_bpermute(paddr, bits_(v[r ^ 15].x)));
                zc.y = as_<float>(__builtin_amdgcn_ds_bpermute(paddr, bits_(v[r ^ 15].y)));
                const float2 z0 = v[bin_reg((16 - m) & 15)];
                if (ln == 0) zc = z0;
                float2 w;
                if (m == 0) w = wlf;
                else if (m == 8) w = make_float2(wlf.y, -wlf.x);
                else w = cmul(wlf, rtw[64 * m]);
                const float ex = zf.x + zc.x, ey = zf.y - zc.y, ox = zf.y + zc.y, oy = zc.x - zf.x;
                const float re = fmaf(ox, w.x, fmaf(-oy, w.y, ex));
                const float im = fmaf(ox, w.y, fmaf(oy, w.x, ey));
                p[r] = 0.25f * fmaf(re, re, im * im);
            }
    #pragma unroll
            for (int r = 0; r < 16; ++r) pw[fl + 64 * bin_reg(r)] = p[r];
            if (ln == 0) {  // Nyquist bin: X[1024] = Re z0 - Im z0 (register 0 of lane 0 holds Z[0])
                const float d = v[0].x - v[0].y;
                pw[kFFT] = d * d;
            }
            wave_lds_fence();
            // ---- banded mel: lane l owns the band pair (l, n_mels-1-l) (narrow + wide filter); each band is a
            // fixed-order fma chain over 8-bin steps of b128 reads (power bins and chunk-transposed weights)
            if constexpr (kMode == 1) {
                spectral_shape(pw, ln, bin_hz, roll, sout + (int64_t)b * 3 * T + t0 + fi, T);
            } else if constexpr (kMode == 2) {
                piptrack_frame(pw, ln, pa, (int64_t)b * T + t0 + fi);
            } else {
                const float4* pw4 = reinterpret_cast<const float4*>(pw);
                auto wt = [&](int c) -> float4 {
                    if constexpr (kWL) return swt[c * kMelLanes + ln];
                    else return gw4[c * kMelLanes + ln];
                };
                const int4 bl = sbl[ln];
                // both bands in one loop (the pair's chunk counts sum to about the same for every lane, the larger of
                // the two does not): chunks [0, bl.y) belong to band l, [bl.y, bl.y + bl.w) to band n_mels-1-l; the
                // running sum restarts at the boundary, so each band keeps its own fixed-order chain
                const int nch = bl.y + bl.w, o0 = bl.x >> 2, o1 = (bl.z >> 2) - bl.y;
                float acc = 0.f, acc0 = 0.f;
                for (int c = 0; c < nch; c += 2) {
                    const bool bnd = c == bl.y;
                    acc0 = bnd ? acc : acc0;
                    acc = bnd ? 0.f : acc;
                    const int o = (c < bl.y ? o0 : o1) + c;
                    const float4 p0 = pw4[o], p1 = pw4[o + 1];
                    const float4 w0 = wt(c), w1 = wt(c + 1);
                    acc = fmaf(p0.x, w0.x, acc); acc = fmaf(p0.y, w0.y, acc);
                    acc = fmaf(p0.z, w0.z, acc); acc = fmaf(p0.w, w0.w, acc);
                    acc = fmaf(p1.x, w1.x, acc); acc = fmaf(p1.y, w1.y, acc);
                    acc = fmaf(p1.z, w1.z, acc); acc = fmaf(p1.w, w1.w, acc);
                }
                float acc1 = acc;
                if (bl.w == 0) { acc0 = acc; acc1 = 0.f; }
                const int m0 = ln, m1 = n_mels - 1 - ln;
                if (m0 < (n_mels + 1) / 2) {
                    smel[fi * (n_mels + 1) + m0] = acc0;
                    lmax = fmaxf(lmax, acc0);
                    lmin = fminf(lmin, acc0);
                    if (m1 != m0) {
                        smel[fi * (n_mels + 1) + m1] = acc1;
                        lmax = fmaxf(lmax, acc1);
                        lmin = fminf(lmin, acc1);
                    }
                }
            }
            wave_lds_fence();
        }
        if constexpr (kMode == 0) {
            __syncthreads();
            // write [n_mels][frames] rows: out[b][m][t0 + f]
            for (int i = threadIdx.x; i < n_mels * kFpb; i += 256) {
                const int m = i / kFpb, f = i % kFpb;
                if (f < nf) out[((int64_t)b * n_mels + m) * T + t0 + f] = smel[f * (n_mels + 1) + m];
            }
            // per-clip max / min (non-negative floats order like their bit patterns); wave-reduce first
            for (int o = 32; o > 0; o >>= 1) {
                lmax = fmaxf(lmax, __shfl_xor(lmax, o, 64));
                lmin = fminf(lmin, __shfl_xor(lmin, o, 64));
            }
            if (lane == 0) {
                if (lmax > 0.f) atomicMax(clip_max + b, __float_as_uint(lmax));
                if (lmin < INFINITY) atomicMin(clip_min + b, __float_as_uint(lmin));
            }
            __syncthreads();  // the staging rows are reused by the next item
        }
    }
}

#define HLMC_STFT_ARGS                                                                                          \
    const float* __restrict__ pcm, int nclips, int64_t n_samples, int T, int hop, const float* __restrict__ window,         \
        const float2* __restrict__ rtw, const float2* __restrict__ tw, const int* __restrict__ band,             \
        const int* __restrict__ woff, const float* __restrict__ wts, int n_mels, int nnz, float* __restrict__ out, \
        unsigned* __restrict__ clip_max, unsigned* __restrict__ clip_min, double bin_hz, double roll,            \
        double* __restrict__ sout, PipArgs pa
#define HLMC_STFT_PASS pcm, nclips, n_samples, T, hop, window, rtw, tw, band, woff, wts, n_mels, nnz, out, clip_max, clip_min, bin_hz, roll, sout, pa

// kMode 0 (the mel hot path) is built for 3 waves per SIMD (168 VGPRs; LDS 52 KB: 3 blocks per CU); the
// spectral-shape / piptrack modes keep the default register budget.
template <int kMode>
__global__ __launch_bounds__(256) void stft_mel_kernel(HLMC_STFT_ARGS) {
    if (((n_samples | hop) & 1) == 0) stft_mel_body<kMode, false, true>(HLMC_STFT_PASS);
    else stft_mel_body<kMode, false, false>(HLMC_STFT_PASS);
}
template <bool kWL, bool kPairs>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void stft_mel0_kernel(HLMC_STFT_ARGS) {
    stft_mel_body<0, kWL, kPairs>(HLMC_STFT_PASS);
}

__device__ __forceinline__ float db_of(float S, float amin) { return 10.f * log10f(fmaxf(amin, S)); }

// power_to_db with a per-clip reference, top_db clamp, crop / pad to t_keep frames.
// S [B][rows][T] -> out [B][rows][t_keep]
__global__ void power_to_db_kernel(const float* __restrict__ S, int B, int rows, int T, int t_keep,
                                   const unsigned* __restrict__ clip_max, const unsigned* __restrict__ clip_min,
                                   int ref_max, float ref_value, float amin, float top_db, float* __restrict__ out) {
    const int64_t n = (int64_t)B * rows * t_keep;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(i % t_keep);
        const int64_t br = i / t_keep;
        const int b = (int)(br / rows);
        const float smax = __uint_as_float(clip_max[b]);
        const float ref_db = db_of(ref_max ? smax : fabsf(ref_value), amin);
        const float floor_db = db_of(smax, amin) - ref_db - top_db;  // log_spec.max() - top_db
        float v;
        if (t < T) {
            v = db_of(S[br * T + t], amin) - ref_db;
        } else {  // pad with the clip's minimum dB value
            v = db_of(__uint_as_float(clip_min[b]), amin) - ref_db;
        }
        if (top_db >= 0.f) v = fmaxf(v, floor_db);
        out[i] = v;
    }
}

// extract_mel_spectrogram's dB pass (ref = clip max, top_db floor, crop / pad with the clip minimum) with, when ZS,
// StandardScaler.transform fused in (column = position within the clip; the same float32 / float64 steps as
// power_to_db_kernel followed by zscore_kernel, so the output is bit-identical to that pair).  Four consecutive
// frames per thread (t_keep % 4 == 0): one 16-byte (f32) / 8-byte (bf16) store.
template <bool ZS, typename OutT>
__global__ __launch_bounds__(256) void mel_db_kernel(const float* __restrict__ S, int B, int rows, int T, int t_keep,
                                                     const unsigned* __restrict__ clip_max,
                                                     const unsigned* __restrict__ clip_min, float amin, float top_db,
                                                     const double* __restrict__ mean, const double* __restrict__ scale,
                                                     OutT* __restrict__ out) {
    const int q4 = t_keep >> 2;
    const int64_t n4 = (int64_t)B * rows * q4;
    for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i4 < n4; i4 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t br = i4 / q4;
        const int t0 = (int)(i4 - br * q4) * 4;
        const int b = (int)(br / rows);
        const float smax = __uint_as_float(clip_max[b]);
        const float ref_db = db_of(smax, amin);
        const float floor_db = db_of(smax, amin) - ref_db - top_db;
        const float pad = db_of(__uint_as_float(clip_min[b]), amin) - ref_db;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = t0 + j;
            v[j] = t < T ? db_of(S[br * T + t], amin) - ref_db : pad;
            if (top_db >= 0.f) v[j] = fmaxf(v[j], floor_db);
        }
        if constexpr (ZS) {
            const int64_t c = (br - (int64_t)b * rows) * t_keep + t0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a = (float)((double)v[j] - mean[c + j]);
                v[j] = (float)((double)a / scale[c + j]);
            }
        }
        OutT* o = out + br * t_keep + t0;
        if constexpr (sizeof(OutT) == 4) {
            *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            unsigned w[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                bf16 lo = __float2bfloat16(v[2 * j]), hi = __float2bfloat16(v[2 * j + 1]);
                w[j] = (unsigned)(*reinterpret_cast<unsigned short*>(&lo)) |
                       ((unsigned)(*reinterpret_cast<unsigned short*>(&hi)) << 16);
            }
            *reinterpret_cast<uint2*>(o) = make_uint2(w[0], w[1]);
        }
    }
}

// MFCC: dB (ref 1.0, top_db) then DCT-II ortho over the mel axis: out[b][k][t] = sum_m D[k][m] db[b][m][t]
__global__ __launch_bounds__(256) void mfcc_kernel(const float* __restrict__ S, int n_mels, int T,
                                                   const unsigned* __restrict__ clip_max, const float* __restrict__ D,
                                                   int n_mfcc, float amin, float top_db, float* __restrict__ out) {
    __shared__ float col[128][65];
    const int b = blockIdx.y;
    const int t0 = blockIdx.x * 64;
    const float smax = __uint_as_float(clip_max[b]);
    const float floor_db = db_of(smax, amin) - top_db;
    for (int i = threadIdx.x; i < n_mels * 64; i += 256) {
        const int m = i / 64, tt = i % 64;
        float v = 0.f;
        if (t0 + tt < T) {
            v = db_of(S[((int64_t)b * n_mels + m) * T + t0 + tt], amin);
            if (top_db >= 0.f) v = fmaxf(v, floor_db);
        }
        col[m][tt] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n_mfcc * 64; i += 256) {
        const int k = i / 64, tt = i % 64;
        if (t0 + tt >= T) continue;
        double s = 0.0;
        for (int m = 0; m < n_mels; ++m) s += (double)D[k * n_mels + m] * col[m][tt];
        out[((int64_t)b * n_mfcc + k) * T + t0 + tt] = (float)s;
    }
}

// mean / std (ddof=0) of each row (two-pass in double; one wave per row)
__global__ void row_mean_std_kernel(const float* __restrict__ x, int64_t rows, int64_t cols, float* mean, float* sd) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (r >= rows) return;
    const float* p = x + r * cols;
    double s = 0.0;
    for (int64_t c = lane; c < cols; c += 64) s += p[c];
    s = wave_sum(s);
    const double m = s / (double)cols;
    double q = 0.0;
    for (int64_t c = lane; c < cols; c += 64) { const double d = p[c] - m; q += d * d; }
    q = wave_sum(q);
    if (lane == 0) {
        mean[r] = (float)m;
        sd[r] = (float)sqrt(q / (double)cols);
    }
}

// StandardScaler passes: one thread per column, rows split across blockIdx.y chunks -> partials
__global__ void col_sum_partial_kernel(const float* __restrict__ x, int64_t n, int64_t cols, int64_t rows_per,
                                       const double* __restrict__ mean, double* __restrict__ p0, double* __restrict__ p1) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    const int64_t r0 = blockIdx.y * rows_per, r1 = min(n, r0 + rows_per);
    double s = 0.0, q = 0.0;
    const double mu = mean ? mean[c] : 0.0;
    for (int64_t r = r0; r < r1; ++r) {
        const double d = (double)x[r * cols + c] - mu;
        s += d;
        q += d * d;
    }
    p0[blockIdx.y * cols + c] = s;
    if (p1) p1[blockIdx.y * cols + c] = q;
}
__global__ void col_sum_final_kernel(const double* __restrict__ p, int nchunk, int64_t cols, double* __restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    double s = 0.0;
    for (int k = 0; k < nchunk; ++k) s += p[k * cols + c];
    out[c] = s;
}

template <typename OutT>
__global__ void zscore_kernel(const float* __restrict__ x, int64_t n, int64_t cols, const double* __restrict__ mean,
                              const double* __restrict__ scale, OutT* __restrict__ y) {
    const int64_t total = n * cols;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = i % cols;
        const float a = (float)((double)x[i] - mean[c]);   // X -= mean_ (float64 op, stored float32)
        const float v = (float)((double)a / scale[c]);     // X /= scale_
        y[i] = from_f32<OutT>(v);
    }
}

// Pass B: librosa.estimate_tuning per clip (one 1024-thread block per clip).
// threshold = np.median(mag over all peaks) (exact: 4-pass radix select on the non-negative float bits, the
// two middle elements averaged in float32); residual = mod(12 * log2(pitch / 27.5), 1) in float32, folded
// to [-0.5, 0.5); np.histogram over the 100 host-built linspace edges (99 bins, last bin closed); tuning =
// the first edge of the first fullest bin (bin 50 = 0.0 when no peak passes).
__device__ unsigned radix_select(const float2* __restrict__ cand, const int* __restrict__ cnt, int T, int maxpk,
                                 unsigned k, unsigned* hist, unsigned* shared) {
    unsigned prefix = 0, mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        for (int t = threadIdx.x >> 6; t < T; t += blockDim.x >> 6) {
            const int n = cnt[t];
            for (int j = threadIdx.x & 63; j < n; j += 64) {
                const unsigned u = __float_as_uint(cand[(int64_t)t * maxpk + j].y);
                if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned acc = 0, d = 0;
            for (; d < 256; ++d) {
                if (acc + hist[d] > k) break;
                acc += hist[d];
            }
            shared[0] = d;
            shared[1] = k - acc;
        }
        __syncthreads();
        prefix |= shared[0] << shift;
        mask |= 255u << shift;
        k = shared[1];
        __syncthreads();
    }
    return prefix;
}

__global__ __launch_bounds__(1024) void tuning_kernel(const float2* __restrict__ cand_all, const int* __restrict__ cnt_all,
                                                      int T, int maxpk, const double* __restrict__ edges, int* __restrict__ tidx,
                                                      double* __restrict__ tval) {
    __shared__ unsigned hist[256], sh[4];
    __shared__ unsigned counts[100];
    __shared__ int red[1024];
    const int b = blockIdx.x;
    const float2* cand = cand_all + (int64_t)b * T * maxpk;
    const int* cnt = cnt_all + (int64_t)b * T;
    int n = 0;
    for (int t = threadIdx.x; t < T; t += blockDim.x) n += cnt[t];
    red[threadIdx.x] = n;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    const unsigned total = (unsigned)red[0];
    __syncthreads();
    float thr = 0.f;
    if (total > 0) {
        const unsigned k1 = (total - 1) / 2, k2 = total / 2;
        const float v1 = __uint_as_float(radix_select(cand, cnt, T, maxpk, k1, hist, sh));
        const float v2 = k2 == k1 ? v1 : __uint_as_float(radix_select(cand, cnt, T, maxpk, k2, hist, sh));
        thr = (v1 + v2) / 2.f;
    }
    for (int i = threadIdx.x; i < 100; i += blockDim.x) counts[i] = 0;
    __syncthreads();
    for (int t = threadIdx.x >> 6; t < T; t += blockDim.x >> 6) {
        const int nn = cnt[t];
        for (int j = threadIdx.x & 63; j < nn; j += 64) {
            const float2 pm = cand[(int64_t)t * maxpk + j];
            if (!(pm.y >= thr) || !(pm.x > 0.f)) continue;
            const float o = log2f(pm.x / 27.5f);
            float r = fmodf(12.f * o, 1.f);
            if (r < 0.f) r += 1.f;
            if (r >= 0.5f) r -= 1.f;
            const double x = (double)r;
            if (x < edges[0] || x > edges[99]) continue;
            int lo = 0, hi = 99;  // largest i with edges[i] <= x (x == edges[99] joins the last bin)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (edges[mid] <= x) lo = mid; else hi = mid;
            }
            atomicAdd(&counts[lo], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int best = 50;
        unsigned bc = 0;
        for (int i = 0; i < 99; ++i)
            if (counts[i] > bc) { bc = counts[i]; best = i; }
        tidx[b] = best;
        if (tval) tval[b] = edges[best];
    }
}

// Pass C: chroma[c][t] = sum_k fb[tuning][c][k] S[t][k] (float32), then librosa.util.normalize(norm=inf)
// over the 12 chroma (columns below float32 tiny stay unnormalised).  Grid (ceil(T/16), B); the clip's
// filterbank [12][kSRow] is LDS-resident; one wavefront per frame, lane l owns bins 16 l .. 16 l + 15.
__global__ __launch_bounds__(256) void chroma_kernel(const float* __restrict__ S, int T, const float* __restrict__ fbs,
                                                     const int* __restrict__ tidx, float* __restrict__ out) {
    __shared__ __align__(16) float fb[12 * kSRow];
    const int b = blockIdx.y;
    const float* src = fbs + (int64_t)tidx[b] * 12 * kSRow;
    for (int i = threadIdx.x; i < 12 * kSRow / 4; i += 256)
        reinterpret_cast<float4*>(fb)[i] = reinterpret_cast<const float4*>(src)[i];
    __syncthreads();
    const int wave = threadIdx.x >> 6, ln = threadIdx.x & 63;
    for (int t = blockIdx.x * 16 + wave; t < min(T, (int)blockIdx.x * 16 + 16); t += 4) {
        const float* row = S + ((int64_t)b * T + t) * kSRow;
        float p[17];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float4 v = reinterpret_cast<const float4*>(row)[4 * ln + c];
            p[4 * c] = v.x; p[4 * c + 1] = v.y; p[4 * c + 2] = v.z; p[4 * c + 3] = v.w;
        }
        p[16] = ln == 63 ? row[kFFT] : 0.f;
        float raw[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            const float* w = fb + c * kSRow + 16 * ln;
            float acc = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) acc = fmaf(w[j], p[j], acc);
            if (ln == 63) acc = fmaf(fb[c * kSRow + kFFT], p[16], acc);
            raw[c] = wave_sum(acc);
        }
        if (ln == 0) {
            float mx = 0.f;
#pragma unroll
            for (int c = 0; c < 12; ++c) mx = fmaxf(mx, fabsf(raw[c]));
            const float d = mx < 1.17549435e-38f ? 1.f : mx;
#pragma unroll
            for (int c = 0; c < 12; ++c) out[((int64_t)b * 12 + c) * T + t] = raw[c] / d;
        }
    }
}

// per-clip max / min accumulators: 0 and a large positive float bit pattern, in one launch (two memsets
// were two blit launches, each with its stream bubble)
__global__ void init_minmax_kernel(unsigned* cmax, unsigned* cmin, int64_t B) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B; i += (int64_t)gridDim.x * blockDim.x) {
        cmax[i] = 0u;
        cmin[i] = 0x7f7f7f7fu;
    }
}

inline int gridn(int64_t n, int cap = 8192) { return (int)std::max<int64_t>(1, std::min<int64_t>(cap, (n + 255) / 256)); }

template <typename U>
int upload(const std::vector<U>& v, U** dst) {
    HLMC_HIP(hipMalloc(dst, v.size() * sizeof(U)));
    HLMC_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(U), hipMemcpyHostToDevice));
    return HLMC_OK;
}

}  // namespace

// ============================================================================ entry points (internal)
namespace feat {

int plan_create(int sr, int n_fft, int hop, int n_mels, double fmin, double fmax, MelPlanImpl** out) {
    HLMC_CHECK_ARG(n_fft == 2 * kFFT, "only n_fft = 2048 is implemented (the reference's value)");
    HLMC_CHECK_ARG(n_mels > 0 && n_mels <= 128, "1 <= n_mels <= 128");
    HLMC_CHECK_ARG(hop > 0 && sr > 0, "hop, sr > 0");
    if (fmax <= 0) fmax = sr / 2.0;
    auto* p = new MelPlanImpl();
    p->sr = sr; p->n_fft = n_fft; p->hop = hop; p->n_mels = n_mels; p->fmin = fmin; p->fmax = fmax;
    p->nbins = 1 + n_fft / 2;
    p->dense = slaney_filterbank(sr, n_fft, n_mels, fmin, fmax);
    std::vector<float> win(n_fft);
    // periodic Hann as scipy.signal.get_window('hann', n_fft, fftbins=True) evaluates it (what librosa.stft
    // calls): 0.5 + 0.5 cos(fac) on fac = linspace(-pi, pi, n_fft + 1) (oracle/mel_oracle.py hann_window)
    const double wstep = (M_PI - (-M_PI)) / n_fft;
    for (int j = 0; j < n_fft; ++j) {
        const double jt = j * wstep;   // separate statements: no fused multiply-add, numpy's two roundings
        const double fac = jt + (-M_PI);
        win[j] = (float)(0.5 + 0.5 * std::cos(fac));
    }
    // FFT twiddles: twB[(k1-1)*64 + p] = e^{-2 pi i p k1 / 1024} (k1 1..15, lane p), then the radix-2 lane
    // stages twC[(j-1)*64 + p] = e^{-2 pi i (p mod 2^j) 2^{5-j} / 64} (lane bit j = 1..5)
    std::vector<float2> tw(kTwB + kTwC), rtw(kFFT + 1);
    auto cis = [](double num, double den) {
        return make_float2((float)std::cos(-2.0 * M_PI * num / den), (float)std::sin(-2.0 * M_PI * num / den));
    };
    for (int k1 = 1; k1 < 16; ++k1)
        for (int q = 0; q < 64; ++q) tw[(k1 - 1) * 64 + q] = cis((double)q * k1, kFFT);
    for (int j = 1; j <= 5; ++j)
        for (int q = 0; q < 64; ++q) tw[kTwB + (j - 1) * 64 + q] = cis((double)((q & ((1 << j) - 1)) << (5 - j)), 64);
    for (int f = 0; f <= kFFT; ++f) rtw[f] = make_float2((float)std::cos(-2.0 * M_PI * f / n_fft), (float)std::sin(-2.0 * M_PI * f / n_fft));
    // Banded filterbank for the kernel's mel stage.  Lane l of a wavefront owns the band pair
    // (l, n_mels-1-l) (a narrow and a wide filter).  Each band starts at its first non-zero bin rounded
    // down to a multiple of 4 and spans an even number of 4-bin chunks (zero weights outside the filter).
    // Weights are stored chunk-transposed, W[c][lane][4], so one b128 LDS read across lanes is
    // contiguous; band info per lane is (start0, chunks0, start1, chunks1).
    const int npairs = (n_mels + 1) / 2;
    std::vector<int> lo(n_mels), cnt(n_mels);
    for (int m = 0; m < n_mels; ++m) {
        int l = -1, h = -1;
        for (int f = 0; f < p->nbins; ++f)
            if (p->dense[(size_t)m * p->nbins + f] != 0.f) { if (l < 0) l = f; h = f; }
        if (l < 0) { lo[m] = 0; cnt[m] = 0; continue; }
        lo[m] = l & ~3;
        const int span = h + 1 - lo[m];
        cnt[m] = ((span + 7) / 8) * 2;  // chunks of 4, even
        p->max_band = std::max(p->max_band, h - l + 1);
    }
    std::vector<int> band(4 * kMelLanes, 0);
    int C = 0;
    for (int l = 0; l < npairs; ++l) {
        const int m0 = l, m1 = n_mels - 1 - l;
        band[4 * l] = lo[m0];
        band[4 * l + 1] = cnt[m0];
        band[4 * l + 2] = m1 != m0 ? lo[m1] : 0;
        band[4 * l + 3] = m1 != m0 ? cnt[m1] : 0;
        C = std::max(C, band[4 * l + 1] + band[4 * l + 3]);
    }
    std::vector<float> w((size_t)std::max(1, C) * kMelLanes * 4, 0.f);
    for (int l = 0; l < npairs; ++l) {
        const int ms[2] = {l, n_mels - 1 - l};
        int c0 = 0;
        for (int h = 0; h < (ms[1] != ms[0] ? 2 : 1); ++h) {
            const int m = ms[h];
            for (int e = 0; e < 4 * cnt[m]; ++e) {
                const int f = lo[m] + e;
                const float v = f < p->nbins ? p->dense[(size_t)m * p->nbins + f] : 0.f;
                const int c = c0 + e / 4;
                w[((size_t)c * kMelLanes + l) * 4 + (e & 3)] = v;
            }
            c0 += cnt[m];
        }
    }
    p->nnz = C * kMelLanes * 4;  // floats of the chunk-transposed weight table
    std::vector<int> woff(1, 0);
    int st = HLMC_OK;
    if ((st = upload(win, &p->d_window)) || (st = upload(tw, &p->d_tw)) || (st = upload(rtw, &p->d_rtw)) ||
        (st = upload(band, &p->d_band)) || (st = upload(woff, &p->d_woff)) || (st = upload(w, &p->d_w))) {
        delete p;
        return st;
    }
    *out = p;
    return HLMC_OK;
}

void plan_destroy(MelPlanImpl* p) {
    if (!p) return;
    (void)hipFree(p->d_window); (void)hipFree(p->d_tw); (void)hipFree(p->d_rtw);
    (void)hipFree(p->d_band); (void)hipFree(p->d_woff); (void)hipFree(p->d_w);
    (void)hipFree(p->d_chroma_fb); (void)hipFree(p->d_tune_edges);
    delete p;
}

int64_t frames(const MelPlanImpl* p, int64_t n) { return 1 + n / p->hop; }

// workspace: mel power [B][n_mels][T] f32 + clip max/min
int64_t workspace(const MelPlanImpl* p, int64_t B, int64_t n) {
    return ((B * p->n_mels * frames(p, n) * 4 + 255) & ~int64_t(255)) + 2 * ((B * 4 + 255) & ~int64_t(255));
}

// Persistent grid of the STFT kernels: resident blocks over all CUs (a multiple of 8, one share per XCD), at most
// one per item rounded up to the XCD count.
template <typename K>
static unsigned stft_grid(K kernel, size_t dyn, int64_t nitems) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 256, dyn) != hipSuccess || occ < 1) occ = 1;
    const int64_t resident = (int64_t)std::max(cus, 1) * occ;
    const int64_t want = std::min(resident, (nitems + 7) / 8 * 8);
    return (unsigned)std::max<int64_t>(8, want / 8 * 8);
}

static int mel_power(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, float* out,
                     unsigned* cmax, unsigned* cmin) {
    HLMC_CHECK_ARG(pcm && out && B > 0 && n > 0, "bad melspectrogram arguments");
    HLMC_CHECK_ARG(B <= 65535, "batch <= 65535");
    HLMC_CHECK_ARG(n < kMaxStftSamples, "clip length < 2^29 samples");
    const int T = (int)frames(p, n);
    init_minmax_kernel<<<(unsigned)((B + 255) / 256), 256, 0, s>>>(cmax, cmin, B);  // 0x7f7f7f7f: large positive float
    HLMC_LAUNCHED();
    HLMC_CHECK_ARG(p->n_mels <= 2 * kMelLanes, "n_mels <= 128");
    const int64_t nitems = B * ((T + kFpb - 1) / kFpb);
    const bool wl = (size_t)p->nnz * 4 <= (size_t)kMaxWLds;  // filterbank staged in LDS
    const size_t dyn = (4 * kMelLanes + (wl ? (size_t)p->nnz : 0) + (size_t)kFpb * (p->n_mels + 1)) * 4;
    {  // algorithmic work: radix-2-equivalent FFT 2.5 N log2 N + window + |X|^2 + banded mel; PCM in, mel out
        const double nf = p->n_fft, lg = std::log2(nf);
        probe::site(probe::kStftMel, (double)B * T * (2.5 * nf * lg + nf + 3.0 * (nf / 2 + 1) + 2.0 * p->nnz),
                    (double)B * ((double)n * 4 + (double)p->n_mels * T * 4));
    }
    HLMC_PROBE_BEGIN(s);
    const bool pairs = ((n | p->hop) & 1) == 0;  // 8-byte sample-pair loads (even clip length and hop)
    auto launch = [&](auto kern) {
        kern<<<stft_grid(kern, dyn, nitems), 256, dyn, s>>>(pcm, (int)B, n, T, p->hop, p->d_window, p->d_rtw, p->d_tw,
                                                            p->d_band, p->d_woff, p->d_w, p->n_mels, p->nnz, out, cmax,
                                                            cmin, 0.0, 0.0, nullptr, PipArgs{});
    };
    if (wl) {
        if (pairs) launch(stft_mel0_kernel<true, true>);
        else launch(stft_mel0_kernel<true, false>);
    } else {
        if (pairs) launch(stft_mel0_kernel<false, true>);
        else launch(stft_mel0_kernel<false, false>);
    }
    HLMC_PROBE_END(s);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int melspectrogram(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, float* out, void* ws) {
    HLMC_CHECK_ARG(ws, "workspace required");
    unsigned* c = reinterpret_cast<unsigned*>(ws);  // clip max / min scratch (2*B words)
    return mel_power(p, s, pcm, B, n, out, c, c + B);
}

int mel_db(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, int64_t t_keep, float amin,
           float top_db, float* out, void* ws) {
    HLMC_CHECK_ARG(ws, "workspace required");
    const int T = (int)frames(p, n);
    char* w = reinterpret_cast<char*>(ws);
    float* S = reinterpret_cast<float*>(w);
    const int64_t sb = (B * p->n_mels * T * 4 + 255) & ~int64_t(255);
    unsigned* cmax = reinterpret_cast<unsigned*>(w + sb);
    unsigned* cmin = reinterpret_cast<unsigned*>(w + sb + ((B * 4 + 255) & ~int64_t(255)));
    HLMC_TRY(mel_power(p, s, pcm, B, n, S, cmax, cmin));
    const int64_t tot = B * p->n_mels * t_keep;
    if (t_keep % 4 == 0 && ((uintptr_t)out & 15) == 0)
        mel_db_kernel<false, float><<<gridn(tot / 4), 256, 0, s>>>(S, (int)B, p->n_mels, T, (int)t_keep, cmax, cmin,
                                                                   amin, top_db, nullptr, nullptr, out);
    else
        power_to_db_kernel<<<gridn(tot), 256, 0, s>>>(S, (int)B, p->n_mels, T, (int)t_keep, cmax, cmin, 1, 1.f, amin,
                                                       top_db, out);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int mel_db_zscore(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, int64_t t_keep,
                  float amin, float top_db, const double* mean, const double* scale, int dtype, void* out, void* ws) {
    HLMC_CHECK_ARG(ws && mean && scale && out, "bad mel_db_zscore arguments");
    HLMC_CHECK_ARG(t_keep > 0 && t_keep % 4 == 0, "t_keep must be a positive multiple of 4");
    HLMC_CHECK_ARG(dtype == HLMC_F32 || dtype == HLMC_BF16, "out dtype f32 or bf16");
    HLMC_CHECK_ARG(((uintptr_t)out & (dtype == HLMC_F32 ? 15 : 7)) == 0, "out must be 16-byte (f32) / 8-byte (bf16) aligned");
    const int T = (int)frames(p, n);
    char* w = reinterpret_cast<char*>(ws);
    float* S = reinterpret_cast<float*>(w);
    const int64_t sb = (B * p->n_mels * T * 4 + 255) & ~int64_t(255);
    unsigned* cmax = reinterpret_cast<unsigned*>(w + sb);
    unsigned* cmin = reinterpret_cast<unsigned*>(w + sb + ((B * 4 + 255) & ~int64_t(255)));
    HLMC_TRY(mel_power(p, s, pcm, B, n, S, cmax, cmin));
    const unsigned g = gridn(B * p->n_mels * t_keep / 4);
    if (dtype == HLMC_BF16)
        mel_db_kernel<true, bf16><<<g, 256, 0, s>>>(S, (int)B, p->n_mels, T, (int)t_keep, cmax, cmin, amin, top_db,
                                                    mean, scale, reinterpret_cast<bf16*>(out));
    else
        mel_db_kernel<true, float><<<g, 256, 0, s>>>(S, (int)B, p->n_mels, T, (int)t_keep, cmax, cmin, amin, top_db,
                                                     mean, scale, reinterpret_cast<float*>(out));
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int mfcc(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, int n_mfcc, const float* dct,
         float amin, float top_db, float* out, void* ws) {
    HLMC_CHECK_ARG(ws && n_mfcc > 0 && n_mfcc <= p->n_mels, "bad mfcc arguments");
    const int T = (int)frames(p, n);
    char* w = reinterpret_cast<char*>(ws);
    float* S = reinterpret_cast<float*>(w);
    const int64_t sb = (B * p->n_mels * T * 4 + 255) & ~int64_t(255);
    unsigned* cmax = reinterpret_cast<unsigned*>(w + sb);
    unsigned* cmin = reinterpret_cast<unsigned*>(w + sb + ((B * 4 + 255) & ~int64_t(255)));
    HLMC_TRY(mel_power(p, s, pcm, B, n, S, cmax, cmin));
    dim3 grid((T + 63) / 64, (unsigned)B);
    mfcc_kernel<<<grid, 256, 0, s>>>(S, p->n_mels, T, cmax, dct, n_mfcc, amin, top_db, out);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

// generic power_to_db over [B][per_clip] with per-clip max computed here (ws: 2*B uint)
__global__ void clip_max_kernel(const float* __restrict__ S, int64_t per, unsigned* cmax, unsigned* cmin) {
    const int b = blockIdx.y;
    float mx = 0.f, mn = INFINITY;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = S[(int64_t)b * per + i];
        mx = fmaxf(mx, v);
        mn = fminf(mn, v);
    }
    if (mx > 0.f) atomicMax(cmax + b, __float_as_uint(mx));
    if (mn < INFINITY) atomicMin(cmin + b, __float_as_uint(fmaxf(mn, 0.f)));
}

int power_to_db(hipStream_t s, const float* S, int64_t B, int64_t per, int ref_max, float ref_value, float amin,
                float top_db, float* out, void* ws) {
    HLMC_CHECK_ARG(S && out && ws && B > 0 && B <= 65535, "bad power_to_db arguments");
    unsigned* cmax = reinterpret_cast<unsigned*>(ws);
    unsigned* cmin = cmax + B;
    init_minmax_kernel<<<(unsigned)((B + 255) / 256), 256, 0, s>>>(cmax, cmin, B);
    HLMC_LAUNCHED();
    dim3 g(std::min<int64_t>(64, (per + 255) / 256), (unsigned)B);
    clip_max_kernel<<<g, 256, 0, s>>>(S, per, cmax, cmin);
    HLMC_LAUNCHED();
    power_to_db_kernel<<<gridn(B * per), 256, 0, s>>>(S, (int)B, 1, (int)per, (int)per, cmax, cmin, ref_max, ref_value,
                                                      amin, top_db, out);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int spectral_shape(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, double roll_percent,
                   double* out) {
    HLMC_CHECK_ARG(pcm && out && B > 0 && n > 0 && B <= 65535, "bad spectral_shape arguments");
    HLMC_CHECK_ARG(roll_percent > 0.0 && roll_percent < 1.0, "0 < roll_percent < 1");
    const int T = (int)frames(p, n);
    HLMC_CHECK_ARG(n < kMaxStftSamples, "clip length < 2^29 samples");
    const unsigned grid = stft_grid(stft_mel_kernel<1>, 0, B * ((T + kFpb - 1) / kFpb));
    stft_mel_kernel<1><<<grid, 256, 0, s>>>(pcm, (int)B, n, T, p->hop, p->d_window, p->d_rtw, p->d_tw, p->d_band, p->d_woff,
                                            p->d_w, 0, 0, nullptr, nullptr, nullptr, (double)p->sr / p->n_fft,
                                            roll_percent, out, PipArgs{});
    HLMC_LAUNCHED();
    return HLMC_OK;
}

// librosa.filters.chroma(sr, n_fft, n_chroma=12, tuning, ctroct=5, octwidth=2, norm=2, base_c=True) in double,
// stored float32 [12][kSRow] (bins 0..n_fft/2), for every tuning edge of estimate_tuning's histogram.
static std::vector<float> chroma_filterbank(int sr, int n_fft, double tuning) {
    const int nc = 12, nb = n_fft / 2 + 1;
    std::vector<double> frq(n_fft), bw(n_fft);
    const double a440 = 440.0 * std::pow(2.0, tuning / nc);
    const double step = (double)sr / n_fft;
    for (int k = 1; k < n_fft; ++k) frq[k] = nc * std::log2(((double)k * step) / (a440 / 16));
    frq[0] = frq[1] - 1.5 * nc;
    for (int k = 0; k + 1 < n_fft; ++k) bw[k] = std::max(frq[k + 1] - frq[k], 1.0);
    bw[n_fft - 1] = 1.0;
    std::vector<double> w((size_t)nc * n_fft);
    const double half = std::round(nc / 2.0);
    for (int c = 0; c < nc; ++c)
        for (int k = 0; k < n_fft; ++k) {
            double d = frq[k] - c + half + 10.0 * nc;
            d = d - std::floor(d / nc) * nc;  // np.remainder (Python modulo)
            d -= half;
            const double z = 2.0 * d / bw[k];
            w[(size_t)c * n_fft + k] = std::exp(-0.5 * z * z);
        }
    for (int k = 0; k < n_fft; ++k) {
        double ss = 0.0;
        for (int c = 0; c < nc; ++c) ss += w[(size_t)c * n_fft + k] * w[(size_t)c * n_fft + k];
        const double len = std::sqrt(ss);
        const double oct = (frq[k] / nc - 5.0) / 2.0;
        const double sc = std::exp(-0.5 * oct * oct);
        for (int c = 0; c < nc; ++c) {
            double v = w[(size_t)c * n_fft + k];
            if (len >= 2.2250738585072014e-308) v /= len;
            w[(size_t)c * n_fft + k] = v * sc;
        }
    }
    std::vector<float> out((size_t)nc * kSRow, 0.f);
    for (int c = 0; c < nc; ++c)  // np.roll(wts, -3, axis=0): row c <- row (c + 3) % 12
        for (int k = 0; k < nb; ++k) out[(size_t)c * kSRow + k] = (float)w[(size_t)((c + 3) % nc) * n_fft + k];
    return out;
}

// piptrack frequency mask on np.fft.rfftfreq(n_fft, 1 / sr): 150 <= f < min(4000, sr / 2) -> [kmin, kmax)
static void pip_range(int sr, int n_fft, int* kmin, int* kmax) {
    const double val = 1.0 / (n_fft * (1.0 / sr));
    const double fmax = std::min(4000.0, sr / 2.0);
    *kmin = -1;
    *kmax = 0;
    for (int k = 0; k <= n_fft / 2; ++k) {
        const double f = (double)k * val;
        if (f >= 150.0 && f < fmax) {
            if (*kmin < 0) *kmin = k;
            *kmax = k + 1;
        }
    }
}
static int pip_slots(int sr, int n_fft) {
    int kmin, kmax;
    pip_range(sr, n_fft, &kmin, &kmax);
    return std::max(8, ((kmax - kmin + 2) / 2 + 7) / 8 * 8);
}

int chroma_tables(MelPlanImpl* p) {
    if (p->d_chroma_fb) return HLMC_OK;
    // np.linspace(-0.5, 0.5, 100, endpoint=False) edges
    std::vector<double> edges(100);
    const double stp = 1.0 / 100;
    for (int i = 0; i < 100; ++i) edges[i] = (double)i * stp + -0.5;
    std::vector<float> all;
    all.reserve((size_t)99 * 12 * kSRow);
    for (int i = 0; i < 99; ++i) {
        const std::vector<float> f = chroma_filterbank(p->sr, p->n_fft, edges[i]);
        all.insert(all.end(), f.begin(), f.end());
    }
    int st = HLMC_OK;
    if ((st = upload(edges, &p->d_tune_edges)) || (st = upload(all, &p->d_chroma_fb))) return st;
    pip_range(p->sr, p->n_fft, &p->pip_kmin, &p->pip_kmax);
    return HLMC_OK;
}

int64_t chroma_workspace(const MelPlanImpl* p, int64_t B, int64_t n) {
    const int64_t T = frames(p, n);
    auto al = [](int64_t x) { return (x + 255) & ~int64_t(255); };
    const int64_t mp = pip_slots(p->sr, p->n_fft);
    return al(B * T * kSRow * 4) + al(B * T * mp * 8) + al(B * T * 4) + al(B * 4);
}

int chroma_stft(MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, float* out, double* tuning,
                void* ws) {
    HLMC_CHECK_ARG(pcm && out && ws && B > 0 && n > 0 && B <= 65535, "bad chroma_stft arguments");
    HLMC_TRY(chroma_tables(p));
    const int mp = pip_slots(p->sr, p->n_fft);
    HLMC_CHECK_ARG(p->pip_kmin >= 1 && p->pip_kmax <= p->n_fft / 2 && (p->pip_kmax - p->pip_kmin + 1) / 2 < mp,
                   "piptrack frequency mask out of range");
    const int T = (int)frames(p, n);
    auto al = [](int64_t x) { return (x + 255) & ~int64_t(255); };
    char* w = reinterpret_cast<char*>(ws);
    PipArgs pa;
    pa.S = reinterpret_cast<float*>(w);
    pa.cand = reinterpret_cast<float2*>(w + al(B * T * kSRow * 4));
    pa.cnt = reinterpret_cast<int*>(w + al(B * T * kSRow * 4) + al(B * T * (int64_t)mp * 8));
    int* tidx = reinterpret_cast<int*>(w + al(B * T * kSRow * 4) + al(B * T * (int64_t)mp * 8) + al(B * T * 4));
    pa.maxpk = mp;
    pa.kmin = p->pip_kmin;
    pa.kmax = p->pip_kmax;
    pa.sr = p->sr;
    pa.n_fft = p->n_fft;
    HLMC_CHECK_ARG(n < kMaxStftSamples, "clip length < 2^29 samples");
    const unsigned grid = stft_grid(stft_mel_kernel<2>, 0, B * ((T + kFpb - 1) / kFpb));
    stft_mel_kernel<2><<<grid, 256, 0, s>>>(pcm, (int)B, n, T, p->hop, p->d_window, p->d_rtw, p->d_tw, p->d_band, p->d_woff,
                                            p->d_w, 0, 0, nullptr, nullptr, nullptr, 0.0, 0.0, nullptr, pa);
    HLMC_LAUNCHED();
    tuning_kernel<<<(unsigned)B, 1024, 0, s>>>(pa.cand, pa.cnt, T, mp, p->d_tune_edges, tidx, tuning);
    HLMC_LAUNCHED();
    chroma_kernel<<<dim3((T + 15) / 16, (unsigned)B), 256, 0, s>>>(pa.S, T, p->d_chroma_fb, tidx, out);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int zcr_rms(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, double* zcr, float* rms) {
    HLMC_CHECK_ARG(pcm && zcr && rms && B > 0 && n > 0 && B <= 65535, "bad zcr_rms arguments");
    HLMC_CHECK_ARG(p->n_fft == kZrFrame, "frame_length = 2048 only");
    const int T = (int)frames(p, n);
    dim3 grid((T + 15) / 16, (unsigned)B);
    zcr_rms_kernel<<<grid, 256, 0, s>>>(pcm, n, T, p->hop, zcr, rms);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

int row_mean_std(hipStream_t s, const float* x, int64_t rows, int64_t cols, float* mean, float* sd) {
    HLMC_CHECK_ARG(x && mean && sd && rows > 0 && cols > 0, "bad row_mean_std arguments");
    row_mean_std_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(x, rows, cols, mean, sd);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

static int col_chunks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(256, n / 64)); }
int64_t colstats_workspace(int64_t n, int64_t cols) { return 2 * (int64_t)col_chunks(n) * cols * 8; }

int colstats(hipStream_t s, const float* x, int64_t n, int64_t cols, const double* mean, double* o0, double* o1, void* ws) {
    HLMC_CHECK_ARG(x && o0 && ws && n > 0 && cols > 0, "bad colstats arguments");
    const int nc = col_chunks(n);
    const int64_t rp = (n + nc - 1) / nc;
    double* p0 = reinterpret_cast<double*>(ws);
    double* p1 = o1 ? p0 + (int64_t)nc * cols : nullptr;
    dim3 g((unsigned)((cols + 255) / 256), nc);
    col_sum_partial_kernel<<<g, 256, 0, s>>>(x, n, cols, rp, mean, p0, p1);
    HLMC_LAUNCHED();
    col_sum_final_kernel<<<(unsigned)((cols + 255) / 256), 256, 0, s>>>(p0, nc, cols, o0);
    HLMC_LAUNCHED();
    if (o1) {
        col_sum_final_kernel<<<(unsigned)((cols + 255) / 256), 256, 0, s>>>(p1, nc, cols, o1);
        HLMC_LAUNCHED();
    }
    return HLMC_OK;
}

int zscore(hipStream_t s, const float* x, int64_t n, int64_t cols, const double* mean, const double* scale, int dtype,
           void* out) {
    HLMC_CHECK_ARG(x && mean && scale && out, "bad zscore arguments");
    if (dtype == HLMC_BF16)
        zscore_kernel<bf16><<<gridn(n * cols), 256, 0, s>>>(x, n, cols, mean, scale, reinterpret_cast<bf16*>(out));
    else
        zscore_kernel<float><<<gridn(n * cols), 256, 0, s>>>(x, n, cols, mean, scale, reinterpret_cast<float*>(out));
    HLMC_LAUNCHED();
    return HLMC_OK;
}

}  // namespace feat
}  // namespace hlmc
