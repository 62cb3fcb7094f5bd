// Cluster-quality metrics on the GPU: the silhouette score of the reference's k sweep
// and final clustering — sklearn.metrics.silhouette_score(X, labels) (metric="euclidean") at
// src/Convolutional_VAE.py:320,337,361,399, src/Conditional_VAE.py:298, src/Simple_VAE.py:247,256,262.
//
//   S[i][c] = sum over j with label c of ||x_i - x_j||      (O(N^2 D): the kernel below)
//   a_i = S[i][l_i] / (n_{l_i} - 1),  b_i = min_{c != l_i} S[i][c] / n_c,  s_i = (b_i - a_i) / max(a_i, b_i),
//   s_i = 0 for singleton clusters (sklearn's nan_to_num), score = mean_i s_i.
// Distances are direct fp32 sums of squared differences (no |x|^2 + |y|^2 - 2xy cancellation), per-row
// cluster sums accumulate in float64 in a fixed order; the mean is a fixed-order f64 tree: deterministic.
#include <algorithm>

#include "features.hpp"

namespace hlmc {
namespace {

constexpr int kSilRows = 64;   // rows i per block (4 threads per row)
constexpr int kSilTile = 64;   // rows j per LDS tile

__global__ void sil_count_kernel(const int32_t* __restrict__ labels, int64_t n, int k, int32_t* __restrict__ counts) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int l = labels[i];
        if (l >= 0 && l < k) atomicAdd(&counts[l], 1);  // integer: order-independent
    }
}

// S[i][c] (f64) for the block's 64 rows: thread (row r = tid / 4, sub = tid % 4) holds x_i in registers and
// takes every 4th j of each LDS tile; its per-cluster sums live in LDS (private row, padded), and the 4
// subs are combined in order at the end.  One launch covers the label window [c0, c0 + kw) (as many
// accumulator rows as LDS holds); rows j outside it are skipped, so over all windows every distance is
// computed exactly once.
template <int DMAX>
__global__ __launch_bounds__(256) void sil_sums_kernel(const float* __restrict__ X, int64_t n, int d,
                                                       const int32_t* __restrict__ labels, int k, int c0, int kw,
                                                       double* __restrict__ S) {
    extern __shared__ double sil_sh[];
    constexpr int DS = DMAX + 4;                   // tile row stride: the 4 rows one wave reads at once
                                                   // land on disjoint bank groups (16-B reads stay aligned)
    const int kp = kw + 1;                         // padded accumulator row
    double* acc = sil_sh;                          // [256][kp]
    float* xt = reinterpret_cast<float*>(acc + 256 * kp);  // [kSilTile][DS]
    int* lt = reinterpret_cast<int*>(xt + kSilTile * DS);
    const int tid = threadIdx.x, r = tid >> 2, sub = tid & 3;
    const int64_t i = (int64_t)blockIdx.x * kSilRows + r;
    float xi[DMAX];
#pragma unroll
    for (int c = 0; c < DMAX; ++c) xi[c] = (i < n && c < d) ? X[i * d + c] : 0.f;
    for (int c = 0; c < kp; ++c) acc[tid * kp + c] = 0.0;
    for (int64_t j0 = 0; j0 < n; j0 += kSilTile) {
        __syncthreads();
        for (int e = tid; e < kSilTile * DMAX; e += 256) {
            const int jr = e / DMAX, c = e - jr * DMAX;
            const int64_t j = j0 + jr;
            xt[jr * DS + c] = (j < n && c < d) ? X[j * d + c] : 0.f;
        }
        for (int e = tid; e < kSilTile; e += 256) {
            const int l = (j0 + e < n) ? labels[j0 + e] - c0 : -1;
            lt[e] = (l >= 0 && l < kw) ? l : -1;
        }
        __syncthreads();
        if (i >= n) continue;
        for (int q = sub; q < kSilTile; q += 4) {
            const int l = lt[q];
            if (l < 0) continue;
            const float4* xj = reinterpret_cast<const float4*>(xt + q * DS);
            float s2 = 0.f;
#pragma unroll
            for (int c = 0; c < DMAX / 4; ++c) {
                const float4 v = xj[c];
                const float e0 = xi[4 * c] - v.x, e1 = xi[4 * c + 1] - v.y, e2 = xi[4 * c + 2] - v.z,
                            e3 = xi[4 * c + 3] - v.w;
                s2 = fmaf(e0, e0, s2);
                s2 = fmaf(e1, e1, s2);
                s2 = fmaf(e2, e2, s2);
                s2 = fmaf(e3, e3, s2);
            }
            acc[tid * kp + l] += (double)sqrtf(s2);
        }
    }
    __syncthreads();
    if (i >= n || sub != 0) return;
    for (int c = 0; c < kw; ++c) {
        double v = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) v += acc[(tid + u) * kp + c];
        S[i * k + c0 + c] = v;
    }
}

// s_i from S and the cluster sizes; block partial sums of s_i (f64) for the mean
__global__ __launch_bounds__(256) void sil_samples_kernel(const double* __restrict__ S, int64_t n, int k,
                                                          const int32_t* __restrict__ labels,
                                                          const int32_t* __restrict__ counts,
                                                          double* __restrict__ samples, double* __restrict__ part) {
    __shared__ double red[256];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int li = labels[i];
        const int ni = counts[li];
        double s = 0.0;
        if (ni > 1) {
            const double a = S[i * k + li] / (double)(ni - 1);
            double b = INFINITY;
            for (int c = 0; c < k; ++c)
                if (c != li && counts[c] > 0) b = fmin(b, S[i * k + c] / (double)counts[c]);
            const double m = fmax(a, b);
            s = m > 0.0 ? (b - a) / m : 0.0;
        }
        if (samples) samples[i] = s;
        acc += s;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void sil_mean_kernel(const double* __restrict__ part, int nblk, int64_t n, double* __restrict__ out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int b = threadIdx.x; b < nblk; b += 256) s += part[b];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0] / (double)n;
}

constexpr int kSilFinalBlocks = 512;

// ---------------------------------------------------------------- Davies-Bouldin / Calinski-Harabasz
// sklearn.metrics.davies_bouldin_score (src/Convolutional_VAE.py:400) and calinski_harabasz_score
// (src/Simple_VAE.py:257,263): per-cluster centroids (f64), each point's distance to its own centroid,
// then the k x k finish.  Block partials over contiguous row ranges, reduced in block order.
constexpr int kCluBlocks = 64;

// part[blk][c][d] = sum of x[i][d] over the block's rows with label c (thread d owns column d), for the
// labels of the window [c0, c0 + kw)
__global__ __launch_bounds__(256) void clu_sums_kernel(const float* __restrict__ X, int64_t n, int d,
                                                       const int32_t* __restrict__ labels, int k, int c0, int kw,
                                                       double* __restrict__ part) {
    extern __shared__ double clu_sh[];  // [kw][d]
    for (int e = threadIdx.x; e < kw * d; e += blockDim.x) clu_sh[e] = 0.0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = blockIdx.x * per, r1 = min(n, r0 + per);
    for (int c = threadIdx.x; c < d; c += blockDim.x)
        for (int64_t i = r0; i < r1; ++i) {
            const int l = labels[i] - c0;
            if (l >= 0 && l < kw) clu_sh[l * d + c] += (double)X[i * d + c];
        }
    __syncthreads();
    for (int e = threadIdx.x; e < kw * d; e += blockDim.x)
        part[(int64_t)blockIdx.x * k * d + (int64_t)c0 * d + e] = clu_sh[e];
}

// centroids[c][d] = sum_blk part / count[c]; mean[d] = sum over all rows / n
__global__ void clu_centroid_kernel(const double* __restrict__ part, int nblk, int k, int d,
                                    const int32_t* __restrict__ counts, int64_t n, double* __restrict__ cent,
                                    double* __restrict__ mean) {
    for (int c = threadIdx.x; c < d; c += blockDim.x) {
        double tot = 0.0;
        for (int l = 0; l < k; ++l) {
            double v = 0.0;
            for (int b = 0; b < nblk; ++b) v += part[((int64_t)b * k + l) * d + c];
            cent[l * d + c] = counts[l] > 0 ? v / (double)counts[l] : 0.0;
            tot += v;
        }
        mean[c] = tot / (double)n;
    }
}

// part2[blk][c] = {sum ||x - cent_c||, sum ||x - cent_c||^2} over the block's rows of cluster c: one wave per row
__global__ __launch_bounds__(256) void clu_dist_kernel(const float* __restrict__ X, int64_t n, int d,
                                                       const int32_t* __restrict__ labels, int k,
                                                       const double* __restrict__ cent, double* __restrict__ part2) {
    extern __shared__ double clu_sh[];  // [4 waves][k][2]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int e = threadIdx.x; e < 4 * k * 2; e += blockDim.x) clu_sh[e] = 0.0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = blockIdx.x * per, r1 = min(n, r0 + per);
    for (int64_t i = r0 + wv; i < r1; i += 4) {
        const int l = labels[i];
        double q = 0.0;
        for (int c = lane; c < d; c += 64) {
            const double e = (double)X[i * d + c] - cent[l * d + c];
            q += e * e;
        }
        q = wave_sum(q);
        if (lane == 0) {
            clu_sh[(wv * k + l) * 2] += sqrt(q);
            clu_sh[(wv * k + l) * 2 + 1] += q;
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < k * 2; e += blockDim.x) {
        double v = 0.0;
        for (int w = 0; w < 4; ++w) v += clu_sh[w * k * 2 + e];
        part2[(int64_t)blockIdx.x * k * 2 + e] = v;
    }
}

// out[0] = Davies-Bouldin, out[1] = Calinski-Harabasz (sklearn 1.7 definitions, f64)
__global__ void clu_finish_kernel(const double* __restrict__ part2, int nblk, int k, int d,
                                  const int32_t* __restrict__ counts, int64_t n, const double* __restrict__ cent,
                                  const double* __restrict__ mean, double* __restrict__ intra,
                                  double* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double extra_disp = 0.0, intra_disp = 0.0;
    bool intra_zero = true;
    for (int l = 0; l < k; ++l) {
        double sd = 0.0, sq = 0.0;
        for (int b = 0; b < nblk; ++b) {
            sd += part2[((int64_t)b * k + l) * 2];
            sq += part2[((int64_t)b * k + l) * 2 + 1];
        }
        intra[l] = counts[l] > 0 ? sd / (double)counts[l] : 0.0;
        intra_disp += sq;
        double e2 = 0.0;
        for (int c = 0; c < d; ++c) {
            const double e = cent[l * d + c] - mean[c];
            e2 += e * e;
        }
        extra_disp += (double)counts[l] * e2;
        if (fabs(intra[l]) > 1e-8) intra_zero = false;  // np.allclose(intra, 0): atol 1e-8
    }
    out[1] = intra_disp == 0.0 ? 1.0 : extra_disp * (double)(n - k) / (intra_disp * (double)(k - 1));
    double score = 0.0;
    bool cd_zero = true;
    for (int a = 0; a < k; ++a) {
        double best = 0.0;
        for (int b = 0; b < k; ++b) {
            double q = 0.0;
            for (int c = 0; c < d; ++c) {
                const double e = cent[a * d + c] - cent[b * d + c];
                q += e * e;
            }
            const double cd = sqrt(q);
            if (fabs(cd) > 1e-8) cd_zero = false;
            const double r = cd == 0.0 ? 0.0 : (intra[a] + intra[b]) / cd;  // sklearn: distance 0 -> inf -> 0
            best = fmax(best, r);
        }
        score += best;
    }
    out[0] = (intra_zero || cd_zero) ? 0.0 : score / (double)k;
}

template <int DMAX>
int launch_sums(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, double* S) {
    const size_t tile = (size_t)kSilTile * (DMAX + 4) * sizeof(float) + kSilTile * sizeof(int);
    const int kw_max = std::min(64, (int)((160 * 1024 - tile) / (256 * sizeof(double))) - 1);
    const unsigned grid = (unsigned)((n + kSilRows - 1) / kSilRows);
    for (int c0 = 0; c0 < k; c0 += kw_max) {   // label windows (one launch for k <= kw_max)
        const int kw = std::min(kw_max, k - c0);
        const size_t sh = (size_t)256 * (kw + 1) * sizeof(double) + tile;
        sil_sums_kernel<DMAX><<<grid, 256, sh, s>>>(X, n, d, labels, k, c0, kw, S);
        HLMC_LAUNCHED();
    }
    return HLMC_OK;
}

size_t counts_bytes(int k) { return ((size_t)k * sizeof(int32_t) + 255) / 256 * 256; }

constexpr int kCluWin = 96 * 1024 / sizeof(double);   // doubles of the clu_sums LDS label window

}  // namespace

namespace metrics {

size_t silhouette_workspace(int64_t n, int k) {
    return ((size_t)n * k * sizeof(double) + 255) / 256 * 256 + counts_bytes(k) + kSilFinalBlocks * sizeof(double);
}

int silhouette(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, double* samples,
               double* score, void* ws, size_t ws_bytes) {
    HLMC_CHECK_ARG(X && labels && score && ws, "silhouette: NULL argument");
    HLMC_CHECK_ARG(n >= 2 && d >= 1 && d <= 128, "silhouette: need n >= 2 and 1 <= d <= 128 (row held in registers)");
    HLMC_CHECK_ARG(k >= 2 && k <= n - 1, "silhouette: number of labels must be in [2, n - 1] (sklearn)");
    HLMC_CHECK_ARG(ws_bytes >= silhouette_workspace(n, k), "silhouette: workspace too small");
    char* w = static_cast<char*>(ws);
    double* S = reinterpret_cast<double*>(w);
    int32_t* counts = reinterpret_cast<int32_t*>(w + ((size_t)n * k * sizeof(double) + 255) / 256 * 256);
    double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(counts) + counts_bytes(k));
    HLMC_HIP(hipMemsetAsync(counts, 0, counts_bytes(k), s));
    sil_count_kernel<<<(unsigned)std::min<int64_t>(1024, (n + 255) / 256), 256, 0, s>>>(labels, n, k, counts);
    HLMC_LAUNCHED();
    if (d <= 32) HLMC_TRY(launch_sums<32>(s, X, n, d, labels, k, S));
    else if (d <= 64) HLMC_TRY(launch_sums<64>(s, X, n, d, labels, k, S));
    else HLMC_TRY(launch_sums<128>(s, X, n, d, labels, k, S));
    const int nb = (int)std::min<int64_t>(kSilFinalBlocks, (n + 255) / 256);
    sil_samples_kernel<<<nb, 256, 0, s>>>(S, n, k, labels, counts, samples, part);
    HLMC_LAUNCHED();
    sil_mean_kernel<<<1, 256, 0, s>>>(part, nb, n, score);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

size_t cluster_scores_workspace(int k, int d) {
    return (size_t)kCluBlocks * k * d * sizeof(double) + (size_t)kCluBlocks * k * 2 * sizeof(double) +
           (size_t)k * d * sizeof(double) + (size_t)d * sizeof(double) + counts_bytes(k) + (size_t)k * sizeof(double);
}

int cluster_scores(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, double* out2,
                   void* ws, size_t ws_bytes) {
    HLMC_CHECK_ARG(X && labels && out2 && ws, "cluster_scores: NULL argument");
    HLMC_CHECK_ARG(n >= 2 && d >= 1 && d <= 4096, "cluster_scores: need n >= 2, 1 <= d <= 4096");
    HLMC_CHECK_ARG(k >= 2 && k < n, "cluster_scores: number of labels must be in [2, n - 1]");
    HLMC_CHECK_ARG(4 * 2 * (size_t)k * sizeof(double) <= 64 * 1024, "cluster_scores: k too large (<= 1024)");
    HLMC_CHECK_ARG(ws_bytes >= cluster_scores_workspace(k, d), "cluster_scores: workspace too small");
    double* part = static_cast<double*>(ws);
    double* part2 = part + (size_t)kCluBlocks * k * d;
    double* cent = part2 + (size_t)kCluBlocks * k * 2;
    double* mean = cent + (size_t)k * d;
    int32_t* counts = reinterpret_cast<int32_t*>(mean + d);
    double* intra = reinterpret_cast<double*>(reinterpret_cast<char*>(counts) + counts_bytes(k));
    HLMC_HIP(hipMemsetAsync(counts, 0, counts_bytes(k), s));
    sil_count_kernel<<<(unsigned)std::min<int64_t>(1024, (n + 255) / 256), 256, 0, s>>>(labels, n, k, counts);
    HLMC_LAUNCHED();
    const int kw_max = std::max(1, kCluWin / d);
    for (int c0 = 0; c0 < k; c0 += kw_max) {   // label windows of the LDS accumulators (one launch usually)
        const int kw = std::min(kw_max, k - c0);
        clu_sums_kernel<<<kCluBlocks, 256, (size_t)kw * d * sizeof(double), s>>>(X, n, d, labels, k, c0, kw, part);
        HLMC_LAUNCHED();
    }
    clu_centroid_kernel<<<1, 256, 0, s>>>(part, kCluBlocks, k, d, counts, n, cent, mean);
    HLMC_LAUNCHED();
    clu_dist_kernel<<<kCluBlocks, 256, (size_t)4 * k * 2 * sizeof(double), s>>>(X, n, d, labels, k, cent, part2);
    HLMC_LAUNCHED();
    clu_finish_kernel<<<1, 64, 0, s>>>(part2, kCluBlocks, k, d, counts, n, cent, mean, intra, out2);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

}  // namespace metrics
}  // namespace hlmc
