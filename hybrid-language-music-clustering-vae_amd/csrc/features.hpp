// Internal declarations of the feature (mel / MFCC / scaler) and K-Means kernels.
#pragma once
#include <vector>

#include "ops.hpp"

namespace hlmc {

struct MelPlanImpl {
    int sr, n_fft, hop, n_mels;
    double fmin, fmax;
    int nbins;                       // 1 + n_fft/2
    std::vector<float> dense;        // [n_mels][nbins] (host copy, librosa.filters.mel)
    // device tables
    float* d_window = nullptr;       // [n_fft]
    float2* d_tw = nullptr;          // FFT twiddles: W1024^{p k1} [15][64], radix-2 lane stages [5][64]
    float2* d_rtw = nullptr;         // [n_fft/2+1] e^{-2 pi i f / n_fft}
    int* d_band = nullptr;           // [n_mels][2] first bin, count
    int* d_woff = nullptr;           // [n_mels] offset into d_w
    float* d_w = nullptr;            // packed weights
    int max_band = 0;
    int nnz = 0;
    // chroma_stft tables (built on first use): 99 filterbanks [12][1028] f32 (one per tuning edge), edges
    float* d_chroma_fb = nullptr;
    double* d_tune_edges = nullptr;
    int pip_kmin = -1, pip_kmax = 0;
};

namespace feat {
int plan_create(int sr, int n_fft, int hop, int n_mels, double fmin, double fmax, MelPlanImpl** out);
void plan_destroy(MelPlanImpl* p);
int64_t frames(const MelPlanImpl* p, int64_t n);
int64_t workspace(const MelPlanImpl* p, int64_t B, int64_t n);
int melspectrogram(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, float* out, void* ws);
int mel_db(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, int64_t t_keep, float amin,
           float top_db, float* out, void* ws);
int mel_db_zscore(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, int64_t t_keep,
                  float amin, float top_db, const double* mean, const double* scale, int dtype, void* out, void* ws);
int mfcc(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, int n_mfcc, const float* dct,
         float amin, float top_db, float* out, void* ws);
int power_to_db(hipStream_t s, const float* S, int64_t B, int64_t per, int ref_max, float ref_value, float amin,
                float top_db, float* out, void* ws);
int spectral_shape(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, double roll_percent,
                   double* out);
int zcr_rms(const MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, double* zcr, float* rms);
int64_t chroma_workspace(const MelPlanImpl* p, int64_t B, int64_t n);
int chroma_stft(MelPlanImpl* p, hipStream_t s, const float* pcm, int64_t B, int64_t n, float* out, double* tuning,
                void* ws);
int row_mean_std(hipStream_t s, const float* x, int64_t rows, int64_t cols, float* mean, float* sd);
int64_t colstats_workspace(int64_t n, int64_t cols);
int colstats(hipStream_t s, const float* x, int64_t n, int64_t cols, const double* mean, double* o0, double* o1, void* ws);
int zscore(hipStream_t s, const float* x, int64_t n, int64_t cols, const double* mean, const double* scale, int dtype,
           void* out);
}  // namespace feat

namespace km {
int center(hipStream_t s, const float* X, int64_t n, int d, float* mean, float* var, float* Xc);
int sqdist_rows(hipStream_t s, const float* X, int64_t n, int d, const int64_t* cand, int ncand, float* out);
int assign(hipStream_t s, const float* X, int64_t n, int d, const float* C, int k, int32_t* labels, const int32_t* old,
           int32_t* n_changed);
int sums(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, float* sm, float* w);
size_t sums_ws(int64_t n, int k);
int sums_part(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, float* sm, float* w,
              void* ws, size_t ws_bytes);
int inertia(hipStream_t s, const float* X, int64_t n, int d, const float* C, const int32_t* labels, float* out,
            float* tmp);
int rowdist(hipStream_t s, const float* X, int64_t n, int d, const float* C, const int32_t* labels, float* out);
// restart-batched (R restarts in lockstep; active = bitmask of the restarts to run)
int assign_batch(hipStream_t s, const float* X, int64_t n, int d, const float* C, int k, int R, uint64_t active,
                 int32_t* labels, const int32_t* old, int32_t* n_changed);
int sums_batch(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, int R, uint64_t active,
               float* sm, float* w, void* ws, size_t ws_bytes);
int update_batch(hipStream_t s, int k, int d, int R, uint64_t active, const float* sm, const float* w,
                 const float* C_old, float* C_new, float* info);
int pp_search(hipStream_t s, int64_t n, int R, int T, const float* prev, int prevT, const int32_t* best,
              const double* rvals, int64_t* cand, int32_t* amb);
int pp_dist(hipStream_t s, const float* X, int64_t n, int d, int R, int T, const int64_t* cand, const float* prev,
            int prevT, const int32_t* best, float* out);
int inertia_batch(hipStream_t s, const float* X, int64_t n, int d, const float* C, int k, const int32_t* labels, int R,
                  float* out, float* tmp);
}  // namespace km

// cluster-quality metrics (metrics.hip): silhouette (sklearn silhouette_score / silhouette_samples),
// Davies-Bouldin + Calinski-Harabasz.  Labels are 0..k-1 int32.
namespace metrics {
size_t silhouette_workspace(int64_t n, int k);
int silhouette(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, double* samples,
               double* score, void* ws, size_t ws_bytes);
size_t cluster_scores_workspace(int k, int d);
int cluster_scores(hipStream_t s, const float* X, int64_t n, int d, const int32_t* labels, int k, double* out2,
                   void* ws, size_t ws_bytes);
}  // namespace metrics

}  // namespace hlmc
