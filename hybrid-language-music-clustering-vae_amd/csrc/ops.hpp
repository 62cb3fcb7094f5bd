// Internal op layer: shape-checked launchers for every kernel of the hot path.
// All tensors are caller-owned device pointers; activations are NHWC (channel fastest).
#pragma once
#include "common.hpp"

namespace hlmc {

struct Ws {  // split-K / reduction scratch handed down by the caller
    float* p;
    size_t bytes;
};

namespace ops {

// ---------------------------------------------------------------- GEMM-shaped (gemm_ops.hip)
// Optional fused BatchNorm statistics of a conv output: the producer adds [sum(C) | sum of squares(C)] of the
// values it stores to acc (a zeroed exact accumulator of 2C columns, common.hpp XAcc) and sets done; done = false:
// the caller computes them separately (into the same accumulator).
struct ColStats {
    XAcc acc;
    bool done;
};
// Fused BatchNorm(+LeakyReLU 0.01) backward moments of a data-gradient producer's output da (conv_c1_s2 as the
// output convT's data gradient): y / mean / invstd / gamma / beta of the BN layer whose output gradient it
// writes; acc (2C columns, zeroed) receives [sum dz | sum dz*xhat] and done is set (else computed separately).
struct BnBwdFuse {
    const void* y;
    const float *mean, *invstd, *gamma, *beta;
    XAcc acc;
    bool done;
};
// y[B, Hi/2, Wi/2, Co] = conv3x3_s2_p1(x[B,Hi,Wi,Ci]) + bias ; wp packed [Co][3][3][Ci]
// Train-mode BatchNorm + LeakyReLU(0.01) of a conv's input applied while an LDS halo-tile kernel stages it: x is
// then the layer-below pre-BN map y, acc its statistics (2 Ci columns, delivered by its producer); the kernel
// writes mean / invstd / running statistics like bn_act_train and the activation a_out (Ci channels, x's layout)
// for the weight gradient that reads it.  Only where *_takes_input_bn says so (bf16 halo shapes, train mode).
struct BnInput {
    XAcc acc;
    int64_t R;
    float *mean, *invstd, *rmean, *rvar;
    int64_t* nbt;
    float momentum, eps;
    const float *gamma, *beta;
    void* a_out;
};
template <typename T>
bool conv_s2_takes_input_bn(int B, int Hi, int Wi, int Ci, int Co);
template <typename T>
bool subpixel_takes_input_bn(int B, int Hi, int Wi, int Ci, int Co);
// xin (nullable): BnInput (train-mode BatchNorm of the input applied while staging; needs st)
template <typename T>
int conv_s2(hipStream_t s, const T* x, int B, int Hi, int Wi, int Ci, const T* wp, const float* bias, int Co, T* y, Ws ws,
            ColStats* st = nullptr, const BnInput* xin = nullptr);
template <typename T>
size_t conv_s2_ws(int B, int Hi, int Wi, int Ci, int Co);

// y[B, 2Hi, 2Wi, Co] = convT3x3_s2_p1_op1(x[B,Hi,Wi,Ci]) + bias ; wp packed [Co][3][3][Ci]
// (also the data gradient of a stride-2 conv with the conv weight re-packed [Ci_conv][3][3][Co_conv])
template <typename T>
int subpixel(hipStream_t s, const T* x, int B, int Hi, int Wi, int Ci, const T* wp, const float* bias, int Co, T* y, Ws ws,
             ColStats* st = nullptr, const BnInput* xin = nullptr);
template <typename T>
size_t subpixel_ws(int B, int Hi, int Wi, int Ci, int Co);

// dW[M][C][3][3] = sum_{b,r,c} L[b,r,c,m] * Xh[b, 2r-1+kh, 2c-1+kw, ci]   (L low-res [B,Hl,Wl,M], Xh [B,2Hl,2Wl,C])
template <typename T>
int wgrad_s2(hipStream_t s, const T* L, int B, int Hl, int Wl, int M, const T* Xh, int C, float* dW, Ws ws,
             XAcc bias_acc = XAcc{}, float* dbias = nullptr);  // dbias: the layer's bias gradient from bias_acc
template <typename T>
size_t wgrad_s2_ws(int B, int Hl, int Wl, int M, int C);

// y[m*ldy + n] (+)= act(sum_k x[m*ldx+k] * w[n*ldw+k] + bias[n]),  act 0 none / 1 relu
// relu_ref (nullable, row stride ldy, act == 0): the stored value is zeroed where relu_ref <= 0 — the data gradient
// of a dense layer with the ReLU backward of the layer below applied in the epilogue (after the accumulate)
template <typename T, typename OutT>
int linear(hipStream_t s, const T* x, int ldx, int M, int K, const T* w, int ldw, const float* bias, int N, OutT* y,
           int ldy, int act, int accumulate, Ws ws, const OutT* relu_ref = nullptr);
template <typename T>
size_t linear_ws(int M, int K, int N);

// dW[n][k] = sum_b dy[b*lddy+n] * x[b*ldx+k];  db[n] = sum_b dy[b*lddy+n] (nullable: the same GEMM with a
// virtual ones column appended to x, so no separate column-sum launches)
template <typename T>
int linear_wgrad(hipStream_t s, const T* dy, int lddy, const T* x, int ldx, int Mb, int N, int K, float* dW, float* db,
                 Ws ws);
template <typename T>
size_t linear_wgrad_ws(int Mb, int N, int K);

// ---------------------------------------------------------------- edge convs with one channel (kernels.hip)
// y[B,Hi/2,Wi/2,32] = sum_taps x[B,Hi,Wi] * w[co*9+tap] (+ bias)  (conv1 fwd, convT6 dgrad)
template <typename T>
int conv_c1_s2(hipStream_t s, const float* x, int B, int Hi, int Wi, const float* w, const float* bias, int Co, T* y,
               ColStats* st = nullptr, BnBwdFuse* bf = nullptr);
// y[B,2Hi,2Wi] = convT(x[B,Hi,Wi,Ci]) with w[ci*9+tap] + bias (convT6 fwd, 1 output channel)
template <typename T>
int convT_c1(hipStream_t s, const T* x, int B, int Hi, int Wi, int Ci, const float* w, const float* bias, float* y);
// dW[m*9+tap] = sum L[b,r,c,m] * Xh[b, 2r-1+kh, 2c-1+kw]   (Xh single channel f32)
template <typename T>
int wgrad_c1(hipStream_t s, const T* L, int B, int Hl, int Wl, int M, const float* Xh, float* dW, Ws ws);
size_t wgrad_c1_ws(int B, int Hl, int Wl, int M);

// ---------------------------------------------------------------- batch norm / activation (kernels.hip)
// Statistics travel through exact accumulators (common.hpp XAcc): the caller owns them and zeroes them before the
// producer runs; bn_acc_bytes(C) per BatchNorm pair table (2C columns), bias_acc_bytes(C) per bias column sum.
size_t bn_acc_bytes(int C);
size_t bias_acc_bytes(int C);
// Train-mode statistics over R rows of an [R][C] map (a moments pass into acc); writes mean / invstd and updates
// running stats.
template <typename T>
int bn_stats(hipStream_t s, const T* y, int64_t R, int C, float* mean, float* invstd, float* run_mean, float* run_var,
             int64_t* nbt, float momentum, float eps, XAcc acc);
// Column sums / sums of squares of an [R][C] map into the (zeroed) accumulator acc (2C columns): the statistics a
// consumer finalizes itself when the producer could not deliver them
template <typename T>
int bn_moments(hipStream_t s, const T* y, int64_t R, int C, XAcc acc);
// Eval-mode statistics from running buffers.
int bn_eval_stats(hipStream_t s, const float* run_mean, const float* run_var, int C, float eps, float* mean, float* invstd);
// a = act(gamma*(y-mean)*invstd + beta) [* mask * mscale];  act: 0 lrelu(0.01), 1 relu, 2 none
// Train-mode BatchNorm + activation with the statistics finalized inside the activation kernel (C <= 512): the
// column totals come from acc (have_stats: delivered by the producer; else a moments pass into acc first);
// writes mean / invstd and updates the running statistics like bn_stats.
template <typename T>
int bn_act_train(hipStream_t s, const T* y, int64_t R, int C, XAcc acc, bool have_stats, float* mean, float* invstd,
                 float* run_mean, float* run_var, int64_t* nbt, float momentum, float eps, const float* gamma,
                 const float* beta, int act, const uint8_t* mask, float mscale, T* a, int lda);
template <typename T>
int bn_act(hipStream_t s, const T* y, int64_t R, int C, const float* mean, const float* invstd, const float* gamma,
           const float* beta, int act, const uint8_t* mask, float mscale, T* a, int lda);
// backward through act+BN: dy from da (ld lda); dgamma, dbeta.  mom: zeroed accumulator of the moments (2C
// columns; fused->done: the producer of da already delivered them there).  bias_acc (may be off): the column sums
// of dy (the conv bias gradient) are added there; dbias (nullable, needs bias_acc): also reduce them into dbias
// here (else the caller runs colsum_finalize, e.g. on the weight-gradient stream).  sums: 2C floats of scratch,
// needed for C > 512 only.
template <typename T>
int bn_act_bwd(hipStream_t s, const T* da, int lda, const T* y, int64_t R, int C, const float* mean, const float* invstd,
               const float* gamma, const float* beta, int act, const uint8_t* mask, float mscale, T* dy, float* dgamma,
               float* dbeta, XAcc mom, const BnBwdFuse* fused, XAcc bias_acc, float* dbias, float* sums);
// out[c] = total of column c of acc (C columns)
int colsum_finalize(hipStream_t s, XAcc acc, int C, float* out);
// out[c] (f64) = column c of an exact accumulator (the op-level statistics entry)
int colsum_to_f64(hipStream_t s, XAcc acc, int C, double* out);

// ---------------------------------------------------------------- misc elementwise (kernels.hip)
// Up to 4 float copies in one launch (segments with null dst or src are skipped): the small per-step copies
// (latent outputs, eps, latent gradients) each cost a launch plus a stream bubble on their own.
struct CopySeg {
    float* dst;
    const float* src;
    int64_t n;
};
int copy_segments(hipStream_t s, const CopySeg* segs, int nseg);
template <typename T> int cast_from_f32(hipStream_t s, const float* x, T* y, int64_t n);
template <typename T> int cast_to_f32(hipStream_t s, const T* x, float* y, int64_t n);
// rows x cols submatrix copy with leading dims (T -> T)
template <typename T> int copy2d(hipStream_t s, const T* x, int ldx, T* y, int ldy, int rows, int cols);
template <typename T> int cast2d_from_f32(hipStream_t s, const float* x, int ldx, T* y, int ldy, int rows, int cols);
// NHWC [B,h,w,C] <-> flat NCHW [B, C*h*w] (ld = row stride of the flat side)
// relu_ref (nullable, row stride ldy): y zeroed where relu_ref <= 0 (ReLU backward fused into the relayout)
template <typename T>
int nhwc_to_flat(hipStream_t s, const T* x, int B, int h, int w, int C, T* y, int ldy, const T* relu_ref = nullptr);
template <typename T> int flat_to_nhwc(hipStream_t s, const T* x, int ldx, int B, int h, int w, int C, T* y);
// db[n] = sum_r dy[r*ld + n]
template <typename T> int colsum(hipStream_t s, const T* dy, int ld, int rows, int cols, float* db, Ws ws);
size_t colsum_ws(int rows, int cols);
// z = mu + eps * exp(0.5 logvar)  (z written as T with row stride ldz)
// eps ~ N(0,1), element offset + i of the Philox4x32-10 stream `seed` (offset % 4 == 0) -> out[i]
int randn(hipStream_t s, float* out, int64_t n, uint64_t seed, uint64_t offset);
// reparam_fwd with eps drawn on the device (the same stream elements as randn) and stored to eps_out; mu_out /
// lv_out (nullable): copies of mu / lv written by the same launch (the caller's latent outputs)
template <typename T>
int reparam_rng(hipStream_t s, const float* mu, const float* lv, uint64_t seed, uint64_t offset, int n_rows, int L,
                float* eps_out, T* z, int ldz, float* mu_out = nullptr, float* lv_out = nullptr);
// mu_out / lv_out / eps_keep (nullable): copies of mu / lv / eps written by the same launch
template <typename T>
int reparam_fwd(hipStream_t s, const float* mu, const float* lv, const float* eps, int n_rows, int L, T* z, int ldz,
                float* mu_out = nullptr, float* lv_out = nullptr, float* eps_keep = nullptr);
// latent-head gradients in one pass: gmu = d_mu + dz ; glv = d_lv + dz * eps * 0.5 exp(0.5 lv), written as T
// (the operand of the heads' data / weight gradients); d_mu / d_lv: the caller's loss gradients (nullable: 0)
template <typename T>
int reparam_bwd(hipStream_t s, const T* dz, int lddz, const float* lv, const float* eps, const float* d_mu,
                const float* d_lv, int n_rows, int L, T* gmu, T* glv);

// ---------------------------------------------------------------- loss (kernels.hip)
// partial sums: out[0] = sum (ra-a)^2, out[1] = sum (rt-t)^2, out[2] = sum(1 + lv - mu^2 - e^lv)  (double)
int vae_sums(hipStream_t s, const float* ra, const float* a, int64_t na, const float* rt, const float* t, int64_t nt,
             const float* mu, const float* lv, int64_t nl, double* out3, Ws ws);
size_t vae_sums_ws(int64_t na, int64_t nt, int64_t nl);
// gradients: dra = ca*(ra-a), drt = ct*(rt-t), dmu = ck*mu, dlv = ck*(-0.5)*(1 - e^lv)... (see kernels.hip)
int vae_loss_bwd(hipStream_t s, const float* ra, const float* a, int64_t na, float* dra, const float* rt, const float* t,
                 int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl, const float* coef, float* dmu,
                 float* dlv);
// both in one pass: the sums (out3) and the gradients
int vae_sums_bwd(hipStream_t s, const float* ra, const float* a, int64_t na, float* dra, const float* rt, const float* t,
                 int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl, const float* coef, float* dmu,
                 float* dlv, double* out3, Ws ws);

// ---------------------------------------------------------------- optimizer / packing (kernels.hip)
struct AdamArgs {
    float lr, beta1, beta2, eps, weight_decay;
    int step;
};
int adam(hipStream_t s, int ntensors, float* const* p, const float* const* g, float* const* m, float* const* v,
         const int64_t* numel, AdamArgs a);
// One parameter tensor of a fused Adam + GEMM-weight-pack launch.  taps 9 (conv weight [d0][d1][3][3]
// -> P0 [d0][3][3][ld0 >= d1], P1 [d1][3][3][ld1 >= d0]) or 1 (linear [d0][d1] -> P0 copy, P1 transpose) or
// 0 (unpacked tensor of n elements).  tile0 = first block of this job in the launch (ascending).
struct AdamJob {
    float* p;
    const float* g;
    float* m;
    float* v;
    void* p0;
    void* p1;
    int64_t n;
    int d0, d1, taps, ld0, ld1;
    int tile0, nt1;
};
int adam_job_tiles(AdamJob& j);  // sets nt1, returns the job's block count
template <typename T>
int adam_pack(hipStream_t s, const AdamJob* jobs_dev, int njobs, int total_tiles, AdamArgs a,
              const float* coef_dev = nullptr,  // coef_dev: 6 device floats (adam_coef_host) used instead of a
              int tile_begin = 0);              // launch tiles [tile_begin, total_tiles) only
// torch.optim.Adam step coefficients {beta1, beta2, eps, weight_decay, lr / (1 - beta1^t), sqrt(1 - beta2^t)}
void adam_coef_host(const AdamArgs& a, float* out6);
template <typename T>
int pack(hipStream_t s, const AdamJob* jobs_dev, int njobs, int total_tiles);  // packing only (g/m/v unused)

}  // namespace ops
}  // namespace hlmc
