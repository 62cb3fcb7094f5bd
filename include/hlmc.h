/* libhlmc — MI355X (gfx950) hot path of Shahriar1638/Hybrid-Language-Music-Clustering-VAE.
 *
 * C ABI: plain device pointers (caller-owned, contiguous, 16-byte aligned), sizes, scalars.
 * Every call is stream-ordered and asynchronous on `stream` (a hipStream_t; NULL = default stream),
 * performs no device allocation and no host<->device synchronisation unless stated.
 * Return 0 (HLMC_OK) on success or a negative hlmc_status; hlmc_last_error() gives a thread-local
 * message.  The library never aborts the process.
 *
 * The reference is pure Python; it has no FFI.  Each entry point below names the reference call it
 * replaces (file:line in the reference repo) — the Python package in
 * hybrid-language-music-clustering-vae_amd/ binds them with ctypes.
 */
#ifndef HLMC_H_
#define HLMC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum hlmc_status {
    HLMC_OK = 0,
    HLMC_EINVAL = -1, /* bad shape / pointer / argument */
    HLMC_EHIP = -2,   /* HIP runtime error */
    HLMC_EUNSUP = -3, /* configuration not supported */
    HLMC_EDEVICE = -4, /* a kernel reported a fault through the device status word (hlmc_device_status) */
};

enum hlmc_dtype { HLMC_F32 = 0, HLMC_BF16 = 1 };

int hlmc_version(void);
const char* hlmc_last_error(void);
/* Device status word: bits a kernel raised instead of hanging or returning silently wrong values (bit 0: the one-launch
 * BatchNorm backward's grid-wide arrival count timed out, its outputs are NaN).  No synchronisation: kernels write it
 * with system-scope stores into pinned host memory, so a launch's bit is visible once the launch has completed.  While a
 * bit is raised, hlmc_net_backward / hlmc_op_bn_bwd return HLMC_EDEVICE.  clear != 0 resets the word.  Returns the bits. */
int hlmc_device_status(int clear);
/* test hook: largest R * C taking the one-launch BatchNorm backward (-1: the default 2^22; 0: two passes everywhere)
 * and the arrival spin's poll bound (-1: the default).  Not for production use. */
int hlmc_test_bn_fused(int64_t max_elems, int spin_max);

/* ============================================================== features
 * Replaces librosa.feature.melspectrogram + librosa.power_to_db at
 *   src/1_preprocessing_advanced.py:97-114 and src/1_preprocessing.py:48-58,
 * librosa.feature.mfcc at src/1_preprocessing.py:61-70, the mean/std pooling at
 * src/1_preprocessing.py:115-121 and sklearn StandardScaler at src/1_preprocessing_advanced.py:376-382.
 * STFT: center=True (zero pad n_fft/2), periodic Hann, hop; power |X|^2; Slaney mel (norm='slaney'). */
typedef struct hlmc_mel_plan hlmc_mel_plan;

int hlmc_mel_plan_create(int sr, int n_fft, int hop, int n_mels, double fmin, double fmax, hlmc_mel_plan** out);
int hlmc_mel_plan_destroy(hlmc_mel_plan* plan);
/* host copy of the dense [n_mels][1 + n_fft/2] float32 filterbank (librosa.filters.mel) */
int hlmc_mel_filterbank(const hlmc_mel_plan* plan, float* out_host);
int64_t hlmc_mel_frames(const hlmc_mel_plan* plan, int64_t n_samples);
/* bytes of scratch for hlmc_mel_db / hlmc_mfcc */
int64_t hlmc_mel_workspace(const hlmc_mel_plan* plan, int64_t batch, int64_t n_samples);
/* power mel spectrogram: pcm [batch][n_samples] f32 -> out [batch][n_mels][T] f32 (ws: >= 8*batch bytes) */
int hlmc_melspectrogram(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch,
                        int64_t n_samples, float* out, void* ws);
/* extract_mel_spectrogram: mel -> power_to_db(ref=max over ALL frames of the clip, amin, top_db)
 * -> keep the first t_keep frames (pad with the clip minimum if t_keep > T). out [batch][n_mels][t_keep] */
int hlmc_mel_db(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch, int64_t n_samples,
                int64_t t_keep, float amin, float top_db, float* out, void* ws);
/* hlmc_mel_db followed by StandardScaler.transform (hlmc_zscore_apply with cols = n_mels * t_keep) in the same
 * dB pass: the fitted mel scaler applied to freshly extracted clips (src/1_preprocessing_advanced.py:97-114, then
 * the transform half of mel_scaler.fit_transform at :376-379 on the flattened mel).  Bit-identical to that pair.
 * t_keep % 4 == 0; out [batch][n_mels][t_keep] f32 (16-byte aligned) or bf16 (8-byte aligned). */
int hlmc_mel_db_zscore(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch, int64_t n_samples,
                       int64_t t_keep, float amin, float top_db, const double* mean, const double* scale,
                       int out_dtype, void* out, void* ws);
/* librosa.power_to_db on a [batch][per_clip] array: ref_max!=0 -> ref = per-clip max, else ref_value
 * (ws: >= 8*batch bytes) */
int hlmc_power_to_db(void* stream, const float* S, int64_t batch, int64_t per_clip, int ref_max, float ref_value,
                     float amin, float top_db, float* out, void* ws);
/* librosa.feature.mfcc(n_mfcc): power_to_db(ref=1.0, top_db=80) then DCT-II ortho over mels.
 * out [batch][n_mfcc][T] */
int hlmc_mfcc(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch, int64_t n_samples,
              int n_mfcc, float* out, void* ws);
/* Handcrafted spectral features of src/1_preprocessing.py:73-91 and src/1_preprocessing_advanced.py:133-137,
 * same framing as the plan (center=True, periodic Hann, n_fft, hop; T = hlmc_mel_frames):
 * librosa.feature.spectral_centroid / spectral_bandwidth (p=2, norm=True) / spectral_rolloff(roll_percent)
 * on |STFT| (power 1).  out [batch][3][T] f64, rows centroid, bandwidth, rolloff (Hz). */
int hlmc_spectral_shape(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch, int64_t n_samples,
                        double roll_percent, double* out);
/* librosa.feature.zero_crossing_rate(frame_length=n_fft, hop) (edge padding, threshold 1e-10) -> zcr [batch][T]
 * f64 and librosa.feature.rms(frame_length=n_fft, hop) (zero padding) -> rms [batch][T] f32.  n_fft = 2048. */
int hlmc_zcr_rms(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch, int64_t n_samples,
                 double* zcr, float* rms);
/* librosa.feature.chroma_stft(y, sr, n_fft, hop) of src/1_preprocessing.py:94-102 and
 * src/1_preprocessing_advanced.py:139-141: power |STFT|^2 -> estimate_tuning (piptrack fmin 150, fmax 4000,
 * threshold 0.1; median-magnitude peaks; 0.01-semitone histogram) -> filters.chroma(tuning) -> norm=inf.
 * out [batch][12][T] f32; tuning [batch] f64 (nullable); ws: hlmc_chroma_workspace bytes. */
int64_t hlmc_chroma_workspace(const hlmc_mel_plan* plan, int64_t batch, int64_t n_samples);
int hlmc_chroma_stft(const hlmc_mel_plan* plan, void* stream, const float* pcm, int64_t batch, int64_t n_samples,
                     float* out, double* tuning, void* ws);
/* mean and std (ddof=0) of each row of x [rows][cols] (the mean/std pooling of the feature vectors) */
int hlmc_row_mean_std(void* stream, const float* x, int64_t rows, int64_t cols, float* mean, float* std);
/* StandardScaler fit, two passes with float64 accumulators (sklearn _incremental_mean_and_var):
 *   pass 1: sum[c] = sum_i x[i][c];  pass 2: corr[c] = sum_i (x - mean), m2[c] = sum_i (x - mean)^2
 * (all-reduce the outputs of each pass across ranks for a distributed fit). */
int64_t hlmc_colstats_workspace(int64_t n, int64_t cols);
int hlmc_colstats_sum(void* stream, const float* x, int64_t n, int64_t cols, double* sum, void* ws);
int hlmc_colstats_centered(void* stream, const float* x, int64_t n, int64_t cols, const double* mean, double* corr,
                           double* m2, void* ws);
/* StandardScaler.transform: y = f32(f32(x - mean) / scale) evaluated in float64; out dtype f32 or bf16 */
int hlmc_zscore_apply(void* stream, const float* x, int64_t n, int64_t cols, const double* mean, const double* scale,
                      int out_dtype, void* out);

/* ============================================================== VAE engine
 * Replaces the nn.Module forward/backward of
 *   HybridVAE        src/Convolutional_VAE.py:75-185   (kind 0; cfg = {latent, text_dim (0 = audio-only), H, W})
 *   ConditionalVAE   src/Conditional_VAE.py:109-231    (kind 1; cfg = {latent, text_dim, num_classes, H, W})
 *   VAE (Simple)     src/Simple_VAE.py:47-105          (kind 2; cfg = {input_dim, latent, n_hidden, h_1..h_n})
 * and the torch train step of src/Convolutional_VAE.py:224-240.  Parameters are bound in the
 * reference's registration order (hlmc_net_param_info) as fp32 "master" tensors; dtype selects the
 * activation / MFMA operand type (HLMC_F32 exact fp32 MFMA, HLMC_BF16 bf16 MFMA with fp32 accumulate). */
typedef struct hlmc_net hlmc_net;
enum hlmc_net_kind { HLMC_NET_HYBRID = 0, HLMC_NET_CVAE = 1, HLMC_NET_SIMPLE = 2 };

int hlmc_net_create(int kind, const int64_t* cfg, int ncfg, int dtype, hlmc_net** out);
int hlmc_net_destroy(hlmc_net* net);
int hlmc_net_num_params(const hlmc_net* net);
/* name (NUL-terminated, truncated to cap), ndim and shape (<= 4 dims) of parameter i */
int hlmc_net_param_info(const hlmc_net* net, int i, char* name, int cap, int* ndim, int64_t* shape);
/* float buffers: every BatchNorm's running_mean, running_var (in registration order);
 * num_batches_tracked (int64) is passed separately, one per BatchNorm */
int hlmc_net_num_bn(const hlmc_net* net);
int64_t hlmc_net_state_bytes(const hlmc_net* net);
int64_t hlmc_net_workspace_bytes(const hlmc_net* net, int64_t batch);
/* params / grads: arrays of num_params device pointers (fp32); running: 2*num_bn device pointers
 * (mean, var per BN); nbt: num_bn device int64 pointers; state: hlmc_net_state_bytes of device memory */
int hlmc_net_bind(hlmc_net* net, float* const* params, float* const* grads, float* const* running,
                  int64_t* const* nbt, void* state);
/* Forward.  train!=0: BatchNorm batch statistics (running stats updated), dropout mask applied (Simple);
 * eps [batch][latent] is the reparameterisation noise (torch.randn_like in the reference); eps = NULL draws it on
 * the device from the net's Philox4x32-10 stream (hlmc_net_set_rng; no host launch), kept for the backward.
 * in0 is read again by hlmc_net_backward (the first conv's weight gradient): it must stay allocated and unchanged
 * until then (stream order).
 * hybrid/cvae: in0 = audio [B][1][H][W], in1 = text [B][text_dim], in2 = condition [B][C] (cvae);
 * simple: in0 = x [B][input_dim], dropout = uint8 keep-mask per hidden unit (NULL = no dropout).
 * outputs: recon [B][...], recon_text [B][text_dim] (hybrid with text, cvae), mu, logvar [B][latent],
 * z [B][latent] (simple; nullable elsewhere).  Saves activations in ws for hlmc_net_backward. */
int hlmc_net_forward(hlmc_net* net, void* stream, int64_t batch, int train, const float* in0, const float* in1,
                     const float* in2, const float* eps, const uint8_t* dropout, float* recon, float* recon_text,
                     float* mu, float* logvar, float* z, void* ws);
/* Device reparameterisation noise (replaces torch.randn_like, src/Convolutional_VAE.py:162-165): the stream is
 * Philox4x32-10 keyed by `seed`; element g is component g % 4 of the block at counter g / 4, mapped by Box-Muller.
 * set_rng positions a net's stream (offset % 4 == 0); every forward drawing its own eps advances it by
 * round4(batch * latent).  hlmc_randn writes elements offset .. offset + n - 1 of stream `seed` to out. */
int hlmc_net_set_rng(hlmc_net* net, uint64_t seed, uint64_t offset);
int hlmc_net_get_rng(const hlmc_net* net, uint64_t* seed, uint64_t* offset);
int hlmc_randn(void* stream, float* out, int64_t n, uint64_t seed, uint64_t offset);
/* encoder only (latent extraction, src/Convolutional_VAE.py:286-303): mu, logvar */
int hlmc_net_encode(hlmc_net* net, void* stream, int64_t batch, int train, const float* in0, const float* in1,
                    const float* in2, float* mu, float* logvar, void* ws);
/* decoder only: HybridVAE.decode(z) (src/Convolutional_VAE.py:167-179), ConditionalVAE.decode(z, condition)
 * (src/Conditional_VAE.py:206-225), VAE.decode(z) (src/Simple_VAE.py:95-96).  z [B][latent]; cond [B][C]
 * (cvae, else NULL); dropout: the forward's keep-mask layout (Simple, train; only the decoder blocks' part is
 * read; NULL = none).  train != 0: decoder BatchNorms use batch statistics and update running stats.
 * recon [B][...], recon_text [B][text_dim] (hybrid with text, cvae; else NULL).  Inference only: a later
 * hlmc_net_backward needs a full hlmc_net_forward. */
int hlmc_net_decode(hlmc_net* net, void* stream, int64_t batch, int train, const float* z, const float* cond,
                    const uint8_t* dropout, float* recon, float* recon_text, void* ws);
/* Backward of the last hlmc_net_forward (same ws): writes (overwrites) all parameter gradients.
 * d_recon_text may be NULL when the model has no text branch. */
int hlmc_net_backward(hlmc_net* net, void* stream, int64_t batch, const float* d_recon, const float* d_recon_text,
                      const float* d_mu, const float* d_logvar, void* ws);

/* torch.optim.Adam step over every bound parameter (exp_avg / exp_avg_sq: num_params device pointers),
 * refreshing the packed GEMM weight layouts in the same pass. */
int hlmc_net_adam_step(hlmc_net* net, void* stream, float* const* exp_avg, float* const* exp_avg_sq, float lr,
                       float beta1, float beta2, float eps, float weight_decay, int step);
/* The same step with its step-dependent coefficients read from device memory (coef_dev: 6 floats written by
 * hlmc_adam_coef on the host and copied before each launch) — the form a captured HIP graph replays. */
int hlmc_net_adam_step_dev(hlmc_net* net, void* stream, float* const* exp_avg, float* const* exp_avg_sq,
                           const float* coef_dev);
/* torch.optim.Adam step coefficients for `step` (host): {b1, b2, eps, wd, lr/(1-b1^step), sqrt(1-b2^step)}. */
int hlmc_adam_coef(float lr, float beta1, float beta2, float eps, float weight_decay, int step, float* out6);
/* trust != 0: forward re-packs weights only when they changed through hlmc_net_adam_step (a caller that
 * writes parameters any other way must pass 0, the default, so forward always re-packs). */
int hlmc_net_set_trust_packs(hlmc_net* net, int trust);

/* enable != 0 (single process): hlmc_net_backward returns with the last weight gradients (encoder layers
 * 0-1) still in flight on the engine's weight-gradient stream, and the next hlmc_net_adam_step(_dev) updates
 * every other parameter first, then waits for them (Adam overlaps the tail of the backward pass).  Those
 * gradients are final only after that Adam step (or the next forward / backward, which wait for them).
 * Ignored while bucket sync is enabled. */
int hlmc_net_set_overlap_adam(hlmc_net* net, int enable);
/* Make every gradient of the last hlmc_net_backward final on `stream` (joins a pending tail; no-op otherwise). */
int hlmc_net_settle(hlmc_net* net, void* stream);

/* Data-parallel gradient buckets (the reference trains on one device; its DDP counterpart is the gradient
 * all-reduce of SURVEY.md §8e).  Bucket k = parameters [starts[k], starts[k-1]) in registration order
 * (starts[-1] = num_params), listed in the order hlmc_net_backward finishes them; the last start is 0.
 * Returns the bucket count (<= cap entries written) or a negative status. */
int hlmc_net_grad_buckets(const hlmc_net* net, int* starts, int cap);
/* enable != 0: every later hlmc_net_backward records one event per bucket once all of its gradients are
 * written (backward internally runs weight gradients on a second stream). */
int hlmc_net_set_bucket_sync(hlmc_net* net, int enable);
/* Make `stream` wait until bucket k of the last hlmc_net_backward is final (enqueue-only, no host sync). */
int hlmc_net_bucket_wait(hlmc_net* net, int k, void* stream);

/* ============================================================== live kernel timing (measurement only)
 * Arm: launches of the op kinds in `mask` (1 conv_s2 GEMM, 2 sub-pixel GEMM, 4 conv weight-gradient GEMM,
 * 8 linear GEMM, 16 linear weight-gradient GEMM, 32 STFT-mel, 64 BatchNorm / reduction streaming family) are
 * bracketed by HIP events on their launch
 * stream (up to max_launches; their algorithmic flops / bytes are summed).  Read: synchronises on the last
 * event, returns the count, the summed kernel time and work (and per-launch ms into ms_each[cap_each]), and
 * disarms.  bench.py uses this for the roofline of its dominant kernel inside the timed region. */
int hlmc_probe_arm(int mask, int max_launches);
int hlmc_probe_read(int* launches, double* total_ms, double* flops, double* bytes, float* ms_each, int cap_each);

/* ============================================================== losses
 * loss_function (src/Convolutional_VAE.py:187-194), cvae_loss_function (src/Conditional_VAE.py:233-246),
 * vae_loss (src/Simple_VAE.py:108-114).  sums3 (device, double[3]) receives
 *   { sum (ra-a)^2, sum (rt-t)^2, sum (1 + lv - mu^2 - exp lv) }; the caller forms the reference's tuple. */
int hlmc_loss_sums(void* stream, const float* ra, const float* a, int64_t na, const float* rt, const float* t,
                   int64_t nt, const float* mu, const float* lv, int64_t nl, double* sums3, void* ws);
int64_t hlmc_loss_workspace(int64_t na, int64_t nt, int64_t nl);
/* coef (DEVICE float[3]) = {ca, ct, ck}:  d ra = ca (ra - a), d rt = ct (rt - t), d mu = ck mu,
 * d lv = -0.5 ck (1 - exp lv).  For the summed hybrid loss with upstream grads (gT, gA, gX, gK) of
 * (total, l_audio, l_text, kld): ca = 2 (gT + gA), ct = 2 (w_text gT + gX), ck = beta gT + gK. */
int hlmc_loss_backward(void* stream, const float* ra, const float* a, int64_t na, float* dra, const float* rt,
                       const float* t, int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl,
                       const float* coef, float* dmu, float* dlv);
/* hlmc_loss_sums and hlmc_loss_backward in one pass over the inputs (same outputs; the gradient does not
 * depend on the sums).  Used by the fused train step; ws as for hlmc_loss_sums. */
int hlmc_loss_sums_backward(void* stream, const float* ra, const float* a, int64_t na, float* dra, const float* rt,
                            const float* t, int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl,
                            const float* coef, float* dmu, float* dlv, double* sums3, void* ws);

/* ============================================================== optimizer
 * torch.optim.Adam(lr, betas, eps, weight_decay) step (src/Convolutional_VAE.py:208,235) over
 * n tensors in one launch.  ptr arrays are HOST arrays of device pointers. */
int hlmc_adam_step(void* stream, int n, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numel, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int step, void* scratch);
int64_t hlmc_adam_scratch_bytes(int n);

/* ============================================================== K-Means (sklearn semantics)
 * Device kernels under the Python KMeans host (src/Convolutional_VAE.py:317-319,
 * src/Conditional_VAE.py:293-295, :528; src/Simple_VAE.py:244-261).  X row-major float32 [n][d]. */
/* X_mean = sequential float32 column sums / n (numpy mean(axis=0) order); Xc = X - X_mean;
 * var (nullable) = np.var(X, axis=0) in the same order (sklearn's tolerance input) */
int hlmc_km_center(void* stream, const float* X, int64_t n, int d, float* mean, float* var, float* Xc);
/* out[t][i] = float32(max(0, ||x_c||^2 - 2 x_c.x_i + ||x_i||^2)) evaluated in float64, c = cand[t]
 * (cand is a HOST array of ncand <= 16 row indices) — sklearn _euclidean_distances_upcast */
int hlmc_km_sqdist_rows(void* stream, const float* X, int64_t n, int d, const int64_t* cand, int ncand, float* out);
/* E-step: labels[i] = argmin_j (||c_j||^2 + (-2) x_i.c_j) (float32, first minimum);
 * n_changed (device int32) += count(labels != labels_old) when labels_old != NULL */
int hlmc_km_assign(void* stream, const float* X, int64_t n, int d, const float* centers, int k, int32_t* labels,
                   const int32_t* labels_old, int32_t* n_changed);
/* M-step sums in index order (float32, as sklearn's single-thread loop): sums [k][d], weight [k] */
int hlmc_km_sums(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, float* sums,
                 float* weight);
/* The same sums through a stable partition of the rows by label (device workspace of
 * hlmc_km_sums_workspace(n, k) bytes): the rows of each cluster become one contiguous list in row order and
 * one 1024-thread block per (64-column slab, cluster) runs a loader/adder ring: 15 loader waves gather 64-row
 * chunks into an 8-slot LDS ring, one adder wave adds them in row order.  Limits: 0 < n < 2^30, k <= 8192.
 * n <= 4096 rows take hlmc_km_sums instead (one launch is faster there); the results are the same bits. */
int64_t hlmc_km_sums_workspace(int64_t n, int k);
int hlmc_km_sums_part(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, float* sums,
                      float* weight, void* ws, int64_t ws_bytes);
/* per-row ||x_i - c_{l_i}||^2 in sklearn's _euclidean_dense_dense float32 order -> out [n] */
int hlmc_km_rowdist(void* stream, const float* X, int64_t n, int d, const float* centers, const int32_t* labels,
                    float* out);
/* sum of the row distances accumulated sequentially in float32 (sklearn _inertia_dense) -> out[0]; tmp [n] */
int hlmc_km_inertia(void* stream, const float* X, int64_t n, int d, const float* centers, const int32_t* labels,
                    float* out, float* tmp);

/* ---- R <= 64 restarts (n_init) in lockstep: the same arithmetic per restart, one launch per stage for all.
 * Restart r's centres are centers + r*k*d, its labels labels + r*n; `active` is a bitmask of the restarts a launch
 * runs (the others are left untouched).  The restarts of KMeans(n_init=10) share X and are independent objects. */
int hlmc_km_assign_batch(void* stream, const float* X, int64_t n, int d, const float* centers, int k, int R,
                         uint64_t active, int32_t* labels, const int32_t* labels_old, int32_t* n_changed);
/* hlmc_km_sums_part per restart; ws: R * hlmc_km_sums_workspace(n, k) bytes; sums [R][k][d], weight [R][k] */
int hlmc_km_sums_batch(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, int R,
                       uint64_t active, float* sums, float* weight, void* ws, int64_t ws_bytes);
/* Lloyd centre update (sklearn: centers_new *= 1 / weight_in_clusters, reciprocal in double):
 * C_new[r][j] = sums[r][j] * (float)(1.0 / weight[r][j]); info[r][j] (j < k) = ||C_new[r][j] - C_old[r][j]||^2 in
 * _euclidean_dense_dense float32 order, info[r][k] = 1 when a cluster of restart r is empty (nothing else is written
 * for it: the host relocates, sklearn _relocate_empty_clusters_dense), else 0.  info: [R][k + 1] floats */
int hlmc_km_update_batch(void* stream, int k, int d, int R, uint64_t active, const float* sums, const float* weight,
                         const float* C_old, float* C_new, float* info);
/* k-means++ candidate draw of every restart (sklearn _kmeans_plusplus): restart r's closest distances are the row
 * prev + (r*prevT + best[r])*n; cand[r][t] = min(searchsorted(np.cumsum(closest, dtype=float64), rvals[r][t]), n-1)
 * from a parallel float64 prefix with a rigorous error bracket around numpy's sequential cumsum; amb[r][t] = 1 where
 * the bracket cannot decide (the caller redoes that trial with numpy; rvals within ~1e-11 relative of a prefix).
 * best, rvals: HOST arrays [R], [R*T]; cand (int64), amb (int32): device [R*T]; R*T <= 64 */
int hlmc_km_pp_search(void* stream, int64_t n, int R, int T, const float* prev, int prevT, const int32_t* best,
                      const double* rvals, int64_t* cand, int32_t* amb);
/* out[r][t][i] = min(closest_r[i], sqdist(X[cand[r][t]], X[i])) (hlmc_km_sqdist_rows arithmetic, candidates from the
 * DEVICE array cand [R*T]); prev == NULL: the plain distances (first centre), else closest_r as in hlmc_km_pp_search */
int hlmc_km_pp_dist(void* stream, const float* X, int64_t n, int d, int R, int T, const int64_t* cand, const float* prev,
                    int prevT, const int32_t* best, float* out);
/* hlmc_km_inertia per restart: out [R], tmp [R][n] */
int hlmc_km_inertia_batch(void* stream, const float* X, int64_t n, int d, const float* centers, int k,
                          const int32_t* labels, int R, float* out, float* tmp);

/* ============================================================== cluster-quality metrics
 * sklearn.metrics.silhouette_score / silhouette_samples (metric "euclidean"), replacing the calls at
 * src/Convolutional_VAE.py:320,337,361,399, src/Conditional_VAE.py:298, src/Simple_VAE.py:247,256,262.
 * X [n][d] f32 (d <= 128), labels int32 in [0, k), 2 <= k <= 64.  samples (nullable) [n] f64, score: device
 * f64 scalar.  Deterministic (fixed-order f64 reductions). */
int64_t hlmc_silhouette_workspace(int64_t n, int k);
int hlmc_silhouette(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, double* samples,
                    double* score, void* ws, int64_t ws_bytes);
/* out2 (device f64[2]) = { davies_bouldin_score, calinski_harabasz_score } (src/Convolutional_VAE.py:400,
 * src/Simple_VAE.py:257,263); every label in [0, k) must occur. */
int64_t hlmc_cluster_scores_workspace(int k, int d);
int hlmc_cluster_scores(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, double* out2,
                        void* ws, int64_t ws_bytes);


/* ============================================================== op-level entry points
 * The kernels hlmc_net_* is built from, on NHWC activations (dtype HLMC_F32 / HLMC_BF16 for x, y, packed
 * weights; bias / dW always f32).  ws = split-K scratch (>= 256 MiB is always enough at B <= 256).
 *   conv_s2   y[B,Hi/2,Wi/2,Co] = Conv2d(k3,s2,p1)(x[B,Hi,Wi,Ci]) + bias;  wp [Co][3][3][Ci]
 *   subpixel  y[B,2Hi,2Wi,Co]  = ConvTranspose2d(k3,s2,p1,op1)(x[B,Hi,Wi,Ci]) + bias; wp [Co][3][3][Ci]
 *             (w_torch[Ci][Co][kh][kw] -> wp[co][kh][kw][ci]; also the data gradient of conv_s2)
 *   wgrad_s2  dW[M][C][3][3] = sum_{b,r,c} L[b,r,c,m] Xh[b,2r-1+kh,2c-1+kw,ci]   (L [B,Hl,Wl,M], Xh [B,2Hl,2Wl,C])
 *   linear    y[m*ldy+n] (+)= act(sum_k x[m*ldx+k] w[n*ldw+k] + bias[n]), act 0 none / 1 relu
 *   linear_wgrad dW[n][k] = sum_b dy[b*lddy+n] x[b*ldx+k]
 *   conv_c1_s2 / convT_c1 / wgrad_c1: the single-channel first / last layers (f32 input image). */
int hlmc_op_conv_s2(void* stream, int dtype, const void* x, int B, int Hi, int Wi, int Ci, const void* wp,
                    const float* bias, int Co, void* y, void* ws, int64_t ws_bytes);
int hlmc_op_subpixel(void* stream, int dtype, const void* x, int B, int Hi, int Wi, int Ci, const void* wp,
                     const float* bias, int Co, void* y, void* ws, int64_t ws_bytes);
int hlmc_op_wgrad_s2(void* stream, int dtype, const void* L, int B, int Hl, int Wl, int M, const void* Xh, int C,
                     float* dW, void* ws, int64_t ws_bytes);
/* relu_ref (nullable, row stride ldy, act 0): y zeroed where relu_ref <= 0 after the accumulate (a dense layer's
 * data gradient with the ReLU backward of the layer below fused into the epilogue). */
int hlmc_op_linear(void* stream, int dtype, const void* x, int ldx, int M, int K, const void* w, int ldw,
                   const float* bias, int N, void* y, int ldy, int act, int accumulate, int out_f32, void* ws,
                   int64_t ws_bytes, const void* relu_ref);
/* db (nullable): the bias gradient sum_b dy[b][n], from the same GEMM (a virtual ones column on x). */
int hlmc_op_linear_wgrad(void* stream, int dtype, const void* dy, int lddy, const void* x, int ldx, int Mb, int N,
                         int K, float* dW, float* db, void* ws, int64_t ws_bytes);
int hlmc_op_conv_c1_s2(void* stream, int dtype, const float* x, int B, int Hi, int Wi, const float* w,
                       const float* bias, int Co, void* y);
int hlmc_op_convT_c1(void* stream, int dtype, const void* x, int B, int Hi, int Wi, int Ci, const float* w,
                     const float* bias, float* y);
int hlmc_op_wgrad_c1(void* stream, int dtype, const void* L, int B, int Hl, int Wl, int M, const float* Xh,
                     float* dW, void* ws, int64_t ws_bytes);
/* The train-mode forward of the LDS halo-tile conv (kind 0: conv_s2) / sub-pixel conv (kind 1: subpixel), bf16, at
 * the shapes where hlmc_net_forward runs them (conv Ci 32 -> Co 64 at Wi 64, Ci 64 -> 128 at Wi 32; sub-pixel
 * Ci 64 -> 32 at Wi 32, Ci 128 -> 64 at Wi 16), as the engine launches them:
 *   - out_sums (device f64 [2 Co]) = (sum_rows y | sum_rows y^2) of the stored bf16 output, from the epilogue's exact
 *     statistics accumulator (the next BatchNorm's batch statistics; src/Convolutional_VAE.py:80-100, 124-139);
 *   - gamma != NULL: x is the PRE-BatchNorm map of the layer below; its train-mode BatchNorm2d (batch statistics,
 *     biased variance, eps) + LeakyReLU(0.01) is applied while the input is staged.  mean_out / invstd_out [Ci]
 *     receive the batch statistics, running_mean / running_var / num_batches_tracked (nullable) are updated as
 *     torch does (momentum, unbiased variance), a_out [B,Hi,Wi,Ci] bf16 receives the activation.
 * ws: hlmc_op_halo_workspace(Ci, Co) bytes.  Returns an error for any other shape. */
/* Train-mode BatchNorm2d + LeakyReLU(0.01) backward of one layer (the engine's bn_act_bwd: the moments pass
 * [sum dz | sum dz * xhat] into an exact accumulator, then the apply pass dy = gamma invstd (dz - mean dz -
 * xhat mean(dz xhat)) with its conv-bias column sums), src/Convolutional_VAE.py:80-100 / 124-139 backward.
 * da / y / dy: [R][C] in `dtype` (bf16 or f32; da = grad of the activation, y = the pre-BN map); mean / invstd:
 * the forward batch statistics; dgamma / dbeta [C] (f32) written; dbias (nullable, f32 [C]) = column sums of the
 * stored dy.  ws: hlmc_op_bn_bwd_workspace(C) bytes (zeroed here). */
int64_t hlmc_op_bn_bwd_workspace(int C);
int hlmc_op_bn_bwd(void* stream, int dtype, const void* da, const void* y, int64_t R, int C, const float* mean,
                   const float* invstd, const float* gamma, const float* beta, void* dy, float* dgamma, float* dbeta,
                   float* dbias, void* ws, int64_t ws_bytes);
int64_t hlmc_op_halo_workspace(int Ci, int Co);
int hlmc_op_halo_fwd(void* stream, int kind, const void* x, int B, int Hi, int Wi, int Ci, const void* wp,
                     const float* bias, int Co, void* y, double* out_sums, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum, float eps,
                     float* mean_out, float* invstd_out, void* a_out, void* ws, int64_t ws_bytes);

#ifdef __cplusplus
}
#endif
#endif /* HLMC_H_ */
