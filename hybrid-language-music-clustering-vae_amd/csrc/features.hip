// Audio features on gfx950: framed STFT -> |X|^2 -> Slaney mel -> dB (-> DCT-II MFCC), mean/std
// pooling and the StandardScaler fit/apply.  Replaces librosa / sklearn calls of
// src/1_preprocessing.py:48-70,115-121,305-311 and src/1_preprocessing_advanced.py:97-114,376-391.
//
// STFT kernel: one 256-thread workgroup per (clip, group of frames).  A 2048-point real frame is
// packed into a 1024-point complex sequence (even/odd samples), transformed with a radix-4 Stockham
// FFT in LDS (5 stages, one butterfly per thread per stage), and split back into the 1025 real-FFT
// bins.  Window / twiddle tables are built on the host in double precision.  The Slaney filterbank is
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

__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

// stft -> power -> mel for FPB frames of one clip. out [B][n_mels][T]; clip_max/min (uint bits of f32 >= 0)
// LDS: frame buffers, the real-FFT twiddles (e^{-2 pi i f/2048}; the 1024-point twiddles are its even
// entries), the banded filterbank and the frame's power spectrum.  Two threads per mel band.
constexpr int kMaxW = 4096;  // packed filterbank weights held in LDS
template <int FPB>
__global__ __launch_bounds__(256) void stft_mel_kernel(const float* __restrict__ pcm, int64_t n_samples, int T,
                                                       int hop, const float* __restrict__ window,
                                                       const float2* __restrict__ tw, const float2* __restrict__ rtw,
                                                       const int* __restrict__ band, const int* __restrict__ woff,
                                                       const float* __restrict__ wts, int n_mels, int nnz,
                                                       float* __restrict__ out, unsigned* __restrict__ clip_max,
                                                       unsigned* __restrict__ clip_min) {
    __shared__ float2 buf[kFFT];
    __shared__ float2 tmp[kFFT];
    __shared__ float2 srtw[kFFT + 1];
    __shared__ int sband[128][3];
    __shared__ float pw[kFFT + 1];
    __shared__ float mel[FPB][129];
    extern __shared__ float sw[];  // nnz packed filterbank weights (dynamic, exact size)
    const int b = blockIdx.y;
    const int t0 = blockIdx.x * FPB;
    const float* x = pcm + (int64_t)b * n_samples;
    // this thread's 4 samples of a frame: pairs kk = tid, tid + 256, tid + 512, tid + 768
    auto fetch = [&](int t, float* v) {
        const int64_t start = (int64_t)t * hop - kFFT;  // center=True: pad n_fft/2 = 1024 zeros
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i0 = start + 2 * (threadIdx.x + 256 * q), i1 = i0 + 1;
            v[2 * q] = (i0 >= 0 && i0 < n_samples) ? x[i0] : 0.f;
            v[2 * q + 1] = (i1 >= 0 && i1 < n_samples) ? x[i1] : 0.f;
        }
    };
    for (int i = threadIdx.x; i <= kFFT; i += 256) srtw[i] = rtw[i];
    for (int i = threadIdx.x; i < nnz; i += 256) sw[i] = wts[i];
    for (int m = threadIdx.x; m < n_mels; m += 256) {
        sband[m][0] = band[2 * m];
        sband[m][1] = band[2 * m + 1];
        sband[m][2] = woff[m];
    }
    float lmax = 0.f, lmin = INFINITY;
    const int nf = min(FPB, T - t0);
    float2 wv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) wv[q] = *reinterpret_cast<const float2*>(window + 2 * (threadIdx.x + 256 * q));
    float cur[8];
    fetch(t0, cur);
    for (int f = 0; f < nf; ++f) {
        // pack even/odd windowed samples: z[k] = x[2k] w[2k] + i x[2k+1] w[2k+1]
#pragma unroll
        for (int q = 0; q < 4; ++q)
            buf[threadIdx.x + 256 * q] = make_float2(cur[2 * q] * wv[q].x, cur[2 * q + 1] * wv[q].y);
        __syncthreads();
        if (f + 1 < nf) fetch(t0 + f + 1, cur);  // next frame's samples are in flight during this FFT
        // 1024-point complex FFT, Stockham radix-4 (5 stages), twiddle(k) = srtw[2k]
        {
            float2* src = buf;
            float2* dst = tmp;
            const int j = threadIdx.x;
#pragma unroll
            for (int st = 0; st < 5; ++st) {
                const int Ns = 1 << (2 * st);
                const int k = j & (Ns - 1);
                float2 a[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) a[r] = src[j + r * (kFFT / 4)];
                const int step = kFFT / (4 * Ns);
#pragma unroll
                for (int r = 1; r < 4; ++r) {
                    // e^{-2 pi i m / 1024} = srtw[2m] for 2m <= 1024, else -srtw[2m - 1024]
                    const int f2 = 2 * ((k * r * step) & (kFFT - 1));
                    float2 w = srtw[f2 <= kFFT ? f2 : f2 - kFFT];
                    if (f2 > kFFT) w = make_float2(-w.x, -w.y);
                    a[r] = cmul(a[r], w);
                }
                const float2 b0 = make_float2(a[0].x + a[2].x, a[0].y + a[2].y);
                const float2 b1 = make_float2(a[0].x - a[2].x, a[0].y - a[2].y);
                const float2 b2 = make_float2(a[1].x + a[3].x, a[1].y + a[3].y);
                const float2 b3 = make_float2(a[1].y - a[3].y, -(a[1].x - a[3].x));  // -i (a1 - a3)
                const int d = ((j >> (2 * st)) << (2 * st + 2)) + k;
                dst[d] = make_float2(b0.x + b2.x, b0.y + b2.y);
                dst[d + Ns] = make_float2(b1.x + b3.x, b1.y + b3.y);
                dst[d + 2 * Ns] = make_float2(b0.x - b2.x, b0.y - b2.y);
                dst[d + 3 * Ns] = make_float2(b1.x - b3.x, b1.y - b3.y);
                __syncthreads();
                float2* tt = src;
                src = dst;
                dst = tt;
            }
            // after 5 stages the spectrum Z is in tmp
        }
        // real-FFT split: X[f] = E[f] + e^{-2 pi i f / 2048} O[f],  f = 0..1024
        for (int fb = threadIdx.x; fb <= kFFT; fb += 256) {
            const float2 zf = tmp[fb & (kFFT - 1)];
            const float2 zc = tmp[(kFFT - fb) & (kFFT - 1)];
            const float2 e = make_float2(0.5f * (zf.x + zc.x), 0.5f * (zf.y - zc.y));
            const float2 o = make_float2(0.5f * (zf.y + zc.y), -0.5f * (zf.x - zc.x));
            const float2 ot = cmul(o, srtw[fb]);
            const float re = e.x + ot.x, im = e.y + ot.y;
            pw[fb] = re * re + im * im;
        }
        __syncthreads();
        // banded mel: threads (2m, 2m+1) share band m, interleaved bins, combined in a fixed order
        {
            const int m = threadIdx.x >> 1, h = threadIdx.x & 1;
            float s = 0.f;
            if (m < n_mels) {
                const int f0 = sband[m][0], nb = sband[m][1], wo = sband[m][2];
                for (int q = h; q < nb; q += 2) s = fmaf(pw[f0 + q], sw[wo + q], s);
            }
            const float o = __shfl_xor(s, 1, 64);
            const float tot = h == 0 ? s + o : o + s;
            if (m < n_mels && h == 0) {
                mel[f][m] = tot;
                lmax = fmaxf(lmax, tot);
                lmin = fminf(lmin, tot);
            }
        }
        __syncthreads();
    }
    // write [n_mels][frames] slabs: out[b][m][t0 + f]
    for (int i = threadIdx.x; i < n_mels * FPB; i += 256) {
        const int m = i / FPB, f = i % FPB;
        if (f < nf) out[((int64_t)b * n_mels + m) * T + t0 + f] = mel[f][m];
    }
    // per-clip max / min (non-negative floats order like their bit patterns); wave-reduce first
    for (int o = 32; o > 0; o >>= 1) {
        lmax = fmaxf(lmax, __shfl_xor(lmax, o, 64));
        lmin = fminf(lmin, __shfl_xor(lmin, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        if (lmax > 0.f) atomicMax(clip_max + b, __float_as_uint(lmax));
        if (lmin < INFINITY) atomicMin(clip_min + b, __float_as_uint(lmin));
    }
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
    for (int j = 0; j < n_fft; ++j) win[j] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * j / n_fft));
    std::vector<float2> tw(kFFT), rtw(kFFT + 1);
    for (int k = 0; k < kFFT; ++k) tw[k] = make_float2((float)std::cos(-2.0 * M_PI * k / kFFT), (float)std::sin(-2.0 * M_PI * k / kFFT));
    for (int f = 0; f <= kFFT; ++f) rtw[f] = make_float2((float)std::cos(-2.0 * M_PI * f / n_fft), (float)std::sin(-2.0 * M_PI * f / n_fft));
    std::vector<int> band(2 * n_mels), woff(n_mels);
    std::vector<float> w;
    for (int m = 0; m < n_mels; ++m) {
        int lo = -1, hi = -1;
        for (int f = 0; f < p->nbins; ++f)
            if (p->dense[(size_t)m * p->nbins + f] != 0.f) { if (lo < 0) lo = f; hi = f; }
        if (lo < 0) { lo = 0; hi = -1; }
        band[2 * m] = lo;
        band[2 * m + 1] = hi - lo + 1;
        woff[m] = (int)w.size();
        for (int f = lo; f <= hi; ++f) w.push_back(p->dense[(size_t)m * p->nbins + f]);
        p->max_band = std::max(p->max_band, hi - lo + 1);
    }
    p->nnz = (int)w.size();
    if (w.empty()) w.push_back(0.f);
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
    delete p;
}

int64_t frames(const MelPlanImpl* p, int64_t n) { return 1 + n / p->hop; }

// workspace: mel power [B][n_mels][T] f32 + clip max/min
int64_t workspace(const MelPlanImpl* p, int64_t B, int64_t n) {
    return ((B * p->n_mels * frames(p, n) * 4 + 255) & ~int64_t(255)) + 2 * ((B * 4 + 255) & ~int64_t(255));
}

static int mel_power(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, float* out,
                     unsigned* cmax, unsigned* cmin) {
    HLMC_CHECK_ARG(pcm && out && B > 0 && n > 0, "bad melspectrogram arguments");
    HLMC_CHECK_ARG(B <= 65535, "batch <= 65535");
    const int T = (int)frames(p, n);
    HLMC_HIP(hipMemsetAsync(cmax, 0, B * sizeof(unsigned), s));
    HLMC_HIP(hipMemsetAsync(cmin, 0x7f, B * sizeof(unsigned), s));  // 0x7f7f7f7f = large positive float
    HLMC_CHECK_ARG(p->nnz <= kMaxW, "filterbank too large for the LDS-resident mel stage");
    constexpr int FPB = 8;
    dim3 grid((T + FPB - 1) / FPB, (unsigned)B);
    stft_mel_kernel<FPB><<<grid, 256, (size_t)std::max(1, p->nnz) * sizeof(float), s>>>(pcm, n, T, p->hop, p->d_window, p->d_tw, p->d_rtw, p->d_band, p->d_woff,
                                              p->d_w, p->n_mels, p->nnz, out, cmax, cmin);
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
    power_to_db_kernel<<<gridn(tot), 256, 0, s>>>(S, (int)B, p->n_mels, T, (int)t_keep, cmax, cmin, 1, 1.f, amin, top_db, out);
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
    HLMC_HIP(hipMemsetAsync(cmax, 0, B * sizeof(unsigned), s));
    HLMC_HIP(hipMemsetAsync(cmin, 0x7f, B * sizeof(unsigned), s));
    dim3 g(std::min<int64_t>(64, (per + 255) / 256), (unsigned)B);
    clip_max_kernel<<<g, 256, 0, s>>>(S, per, cmax, cmin);
    HLMC_LAUNCHED();
    power_to_db_kernel<<<gridn(B * per), 256, 0, s>>>(S, (int)B, 1, (int)per, (int)per, cmax, cmin, ref_max, ref_value,
                                                      amin, top_db, out);
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
