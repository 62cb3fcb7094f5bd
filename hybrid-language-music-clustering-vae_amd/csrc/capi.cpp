// extern "C" boundary of libhlmc (declared in include/hlmc.h).
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "engine.hpp"
#include "features.hpp"

namespace hlmc {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }
// HLMC_EDEVICE while a kernel's fault bit is raised in the device status word (common.hpp)
static int device_status_ok() {
    const unsigned st = ops::dev_status_take(false);
    if (st == 0) return HLMC_OK;
    set_error("device status " + std::to_string(st) +
              (st & kDevBnCountTimeout ? ": a one-launch BatchNorm backward's grid-wide arrival count timed out (grid not "
                                         "co-resident); that launch's dgamma / dbeta / dy are NaN" : "") +
              " -- clear with hlmc_device_status(1)");
    return HLMC_EDEVICE;
}

namespace probe {
int g_mask = 0;
Site g_site{0, 0.0, 0.0};
static std::vector<hipEvent_t> g_ev;  // start/stop pairs
static int g_cap = 0, g_n = 0;
static double g_flops = 0.0, g_bytes = 0.0;
void begin(hipStream_t s) {
    if (g_n < g_cap) (void)hipEventRecord(g_ev[2 * g_n], s);
}
void end(hipStream_t s) {
    if (g_n >= g_cap) return;
    (void)hipEventRecord(g_ev[2 * g_n + 1], s);
    g_flops += g_site.flops;
    g_bytes += g_site.bytes;
    ++g_n;
}
}  // namespace probe



}  // namespace hlmc

using namespace hlmc;

struct hlmc_mel_plan {
    MelPlanImpl* impl;
    float* d_dct = nullptr;  // DCT-II (ortho) matrix [n_mfcc][n_mels], built on first use
    int dct_n = 0;
};
struct hlmc_net {
    std::unique_ptr<NetBase> impl;
};

#define S(stream) reinterpret_cast<hipStream_t>(stream)

extern "C" {

int hlmc_version(void) { return 1; }

int hlmc_probe_arm(int mask, int max_launches) {
    HLMC_CHECK_ARG(mask >= 0 && max_launches >= 0, "bad arguments");
    const size_t need = 2 * (size_t)max_launches;
    while (probe::g_ev.size() < need) {
        hipEvent_t e;
        HLMC_HIP(hipEventCreate(&e));
        probe::g_ev.push_back(e);
    }
    probe::g_cap = max_launches;
    probe::g_n = 0;
    probe::g_flops = probe::g_bytes = 0.0;
    probe::g_mask = max_launches > 0 ? mask : 0;
    return HLMC_OK;
}
int hlmc_probe_read(int* launches, double* total_ms, double* flops, double* bytes, float* ms_each, int cap_each) {
    HLMC_CHECK_ARG(launches && total_ms && flops && bytes, "NULL argument");
    double tot = 0.0;
    for (int i = 0; i < probe::g_n; ++i) {
        float ms = 0.f;
        HLMC_HIP(hipEventSynchronize(probe::g_ev[2 * i + 1]));
        HLMC_HIP(hipEventElapsedTime(&ms, probe::g_ev[2 * i], probe::g_ev[2 * i + 1]));
        if (ms_each && i < cap_each) ms_each[i] = ms;
        tot += ms;
    }
    *launches = probe::g_n;
    *total_ms = tot;
    *flops = probe::g_flops;
    *bytes = probe::g_bytes;
    probe::g_mask = 0;
    return HLMC_OK;
}
const char* hlmc_last_error(void) { return get_error(); }
int hlmc_device_status(int clear) { return (int)ops::dev_status_take(clear != 0); }
int hlmc_test_bn_fused(int64_t max_elems, int spin_max) {
    ops::test_bn_fused(max_elems, spin_max);
    return HLMC_OK;
}

// ------------------------------------------------------------------------------------ features
int hlmc_mel_plan_create(int sr, int n_fft, int hop, int n_mels, double fmin, double fmax, hlmc_mel_plan** out) {
    HLMC_CHECK_ARG(out, "out is NULL");
    MelPlanImpl* impl = nullptr;
    HLMC_TRY(feat::plan_create(sr, n_fft, hop, n_mels, fmin, fmax, &impl));
    auto* p = new hlmc_mel_plan();
    p->impl = impl;
    *out = p;
    return HLMC_OK;
}
int hlmc_mel_plan_destroy(hlmc_mel_plan* p) {
    if (!p) return HLMC_OK;
    feat::plan_destroy(p->impl);
    if (p->d_dct) (void)hipFree(p->d_dct);
    delete p;
    return HLMC_OK;
}
int hlmc_mel_filterbank(const hlmc_mel_plan* p, float* out_host) {
    HLMC_CHECK_ARG(p && out_host, "NULL argument");
    std::memcpy(out_host, p->impl->dense.data(), p->impl->dense.size() * sizeof(float));
    return HLMC_OK;
}
int64_t hlmc_mel_frames(const hlmc_mel_plan* p, int64_t n) { return p ? feat::frames(p->impl, n) : -1; }
int64_t hlmc_mel_workspace(const hlmc_mel_plan* p, int64_t B, int64_t n) { return p ? feat::workspace(p->impl, B, n) : -1; }
int hlmc_melspectrogram(const hlmc_mel_plan* p, void* stream, const float* pcm, int64_t B, int64_t n, float* out,
                        void* ws) {
    HLMC_CHECK_ARG(p, "plan is NULL");
    return feat::melspectrogram(p->impl, S(stream), pcm, B, n, out, ws);
}
int hlmc_mel_db(const hlmc_mel_plan* p, void* stream, const float* pcm, int64_t B, int64_t n, int64_t t_keep, float amin,
                float top_db, float* out, void* ws) {
    HLMC_CHECK_ARG(p && t_keep > 0, "bad arguments");
    return feat::mel_db(p->impl, S(stream), pcm, B, n, t_keep, amin, top_db, out, ws);
}
int hlmc_mel_db_zscore(const hlmc_mel_plan* p, void* stream, const float* pcm, int64_t B, int64_t n, int64_t t_keep,
                       float amin, float top_db, const double* mean, const double* scale, int out_dtype, void* out,
                       void* ws) {
    HLMC_CHECK_ARG(p, "plan is NULL");
    return feat::mel_db_zscore(p->impl, S(stream), pcm, B, n, t_keep, amin, top_db, mean, scale, out_dtype, out, ws);
}
int hlmc_power_to_db(void* stream, const float* S_, int64_t B, int64_t per, int ref_max, float ref_value, float amin,
                     float top_db, float* out, void* ws) {
    return feat::power_to_db(S(stream), S_, B, per, ref_max, ref_value, amin, top_db, out, ws);
}
int hlmc_mfcc(const hlmc_mel_plan* cp, void* stream, const float* pcm, int64_t B, int64_t n, int n_mfcc, float* out, void* ws) {
    HLMC_CHECK_ARG(cp, "plan is NULL");
    auto* p = const_cast<hlmc_mel_plan*>(cp);
    if (!p->d_dct || p->dct_n != n_mfcc) {
        const int M = p->impl->n_mels;
        std::vector<float> D((size_t)n_mfcc * M);
        for (int k = 0; k < n_mfcc; ++k)
            for (int m = 0; m < M; ++m) {
                // scipy.fftpack.dct(type=2, norm='ortho') as a matrix; the phase k (2m + 1) reduced modulo 4M in
                // integers so cos sees an argument below 2 pi (oracle/mel_oracle.py dct_ortho_matrix)
                const long ph = ((long)k * (2 * m + 1)) % (4L * M);
                const double c = k == 0 ? std::sqrt(1.0 / M) : std::cos(M_PI * ph / (2.0 * M)) * std::sqrt(2.0 / M);
                D[(size_t)k * M + m] = (float)c;
            }
        if (p->d_dct) (void)hipFree(p->d_dct);
        HLMC_HIP(hipMalloc(&p->d_dct, D.size() * sizeof(float)));
        HLMC_HIP(hipMemcpy(p->d_dct, D.data(), D.size() * sizeof(float), hipMemcpyHostToDevice));
        p->dct_n = n_mfcc;
    }
    return feat::mfcc(p->impl, S(stream), pcm, B, n, n_mfcc, p->d_dct, 1e-10f, 80.f, out, ws);
}
int hlmc_spectral_shape(const hlmc_mel_plan* p, void* stream, const float* pcm, int64_t B, int64_t n,
                        double roll_percent, double* out) {
    HLMC_CHECK_ARG(p, "null plan");
    return feat::spectral_shape(p->impl, S(stream), pcm, B, n, roll_percent, out);
}
int64_t hlmc_chroma_workspace(const hlmc_mel_plan* p, int64_t B, int64_t n) {
    return p ? feat::chroma_workspace(p->impl, B, n) : -1;
}
int hlmc_chroma_stft(const hlmc_mel_plan* p, void* stream, const float* pcm, int64_t B, int64_t n, float* out,
                     double* tuning, void* ws) {
    HLMC_CHECK_ARG(p, "null plan");
    return feat::chroma_stft(p->impl, S(stream), pcm, B, n, out, tuning, ws);
}
int hlmc_zcr_rms(const hlmc_mel_plan* p, void* stream, const float* pcm, int64_t B, int64_t n, double* zcr, float* rms) {
    HLMC_CHECK_ARG(p, "null plan");
    return feat::zcr_rms(p->impl, S(stream), pcm, B, n, zcr, rms);
}
int hlmc_row_mean_std(void* stream, const float* x, int64_t rows, int64_t cols, float* mean, float* sd) {
    return feat::row_mean_std(S(stream), x, rows, cols, mean, sd);
}
int64_t hlmc_colstats_workspace(int64_t n, int64_t cols) { return feat::colstats_workspace(n, cols); }
int hlmc_colstats_sum(void* stream, const float* x, int64_t n, int64_t cols, double* sum, void* ws) {
    return feat::colstats(S(stream), x, n, cols, nullptr, sum, nullptr, ws);
}
int hlmc_colstats_centered(void* stream, const float* x, int64_t n, int64_t cols, const double* mean, double* corr,
                           double* m2, void* ws) {
    HLMC_CHECK_ARG(mean && m2, "mean and m2 required");
    return feat::colstats(S(stream), x, n, cols, mean, corr, m2, ws);
}
int hlmc_zscore_apply(void* stream, const float* x, int64_t n, int64_t cols, const double* mean, const double* scale,
                      int out_dtype, void* out) {
    return feat::zscore(S(stream), x, n, cols, mean, scale, out_dtype, out);
}

// ------------------------------------------------------------------------------------ engine
int hlmc_net_create(int kind, const int64_t* cfg, int ncfg, int dtype, hlmc_net** out) {
    HLMC_CHECK_ARG(out, "out is NULL");
    std::unique_ptr<NetBase> n;
    HLMC_TRY(make_net(kind, cfg, ncfg, dtype, &n));
    auto* h = new hlmc_net();
    h->impl = std::move(n);
    *out = h;
    return HLMC_OK;
}
int hlmc_net_destroy(hlmc_net* n) {
    delete n;
    return HLMC_OK;
}
int hlmc_net_num_params(const hlmc_net* n) { return n ? (int)n->impl->params.size() : -1; }
int hlmc_net_param_info(const hlmc_net* n, int i, char* name, int cap, int* ndim, int64_t* shape) {
    HLMC_CHECK_ARG(n && i >= 0 && i < (int)n->impl->params.size(), "bad parameter index");
    const ParamInfo& p = n->impl->params[i];
    if (name && cap > 0) {
        std::strncpy(name, p.name.c_str(), cap - 1);
        name[cap - 1] = 0;
    }
    if (ndim) *ndim = (int)p.shape.size();
    if (shape)
        for (size_t k = 0; k < p.shape.size(); ++k) shape[k] = p.shape[k];
    return HLMC_OK;
}
int hlmc_net_num_bn(const hlmc_net* n) { return n ? n->impl->n_bn : -1; }
int64_t hlmc_net_state_bytes(const hlmc_net* n) { return n ? (int64_t)n->impl->state_bytes() : -1; }
int64_t hlmc_net_workspace_bytes(const hlmc_net* n, int64_t batch) {
    return (n && batch > 0) ? (int64_t)n->impl->ws_bytes(batch) : -1;
}
int hlmc_net_bind(hlmc_net* h, float* const* params, float* const* grads, float* const* running, int64_t* const* nbt,
                  void* state) {
    HLMC_CHECK_ARG(h && params && grads && running && nbt, "NULL argument");
    NetBase& n = *h->impl;
    const size_t np = n.params.size();
    HLMC_CHECK_ARG(state || n.state_bytes() == 0, "state buffer required");
    n.P.assign(params, params + np);
    n.G.assign(grads, grads + np);
    n.RM.clear();
    n.RV.clear();
    for (int i = 0; i < n.n_bn; ++i) {
        n.RM.push_back(running[2 * i]);
        n.RV.push_back(running[2 * i + 1]);
    }
    n.NBT.assign(nbt, nbt + n.n_bn);
    for (size_t i = 0; i < np; ++i) HLMC_CHECK_ARG(n.P[i] && n.G[i], "NULL parameter / grad pointer");
    n.state = reinterpret_cast<char*>(state);
    n.packs_valid = false;
    return n.bind_state(nullptr);
}
int hlmc_net_forward(hlmc_net* h, void* stream, int64_t batch, int train, const float* in0, const float* in1,
                     const float* in2, const float* eps, const uint8_t* dropout, float* recon, float* recon_text,
                     float* mu, float* logvar, float* z, void* ws) {
    HLMC_CHECK_ARG(h && ws && batch > 0, "bad arguments");
    HLMC_CHECK_ARG(!h->impl->P.empty(), "net is not bound");
    ForwardArgs a{batch, train, in0, in1, in2, eps, dropout, recon, recon_text, mu, logvar, z, ws, false};
    return h->impl->forward(S(stream), a);
}
int hlmc_net_encode(hlmc_net* h, void* stream, int64_t batch, int train, const float* in0, const float* in1,
                    const float* in2, float* mu, float* logvar, void* ws) {
    HLMC_CHECK_ARG(h && ws && batch > 0, "bad arguments");
    HLMC_CHECK_ARG(!h->impl->P.empty(), "net is not bound");
    ForwardArgs a{batch, train, in0, in1, in2, nullptr, nullptr, nullptr, nullptr, mu, logvar, nullptr, ws, true};
    return h->impl->forward(S(stream), a);
}
int hlmc_net_decode(hlmc_net* h, void* stream, int64_t batch, int train, const float* z, const float* cond,
                    const uint8_t* dropout, float* recon, float* recon_text, void* ws) {
    HLMC_CHECK_ARG(h && ws && batch > 0 && z && recon, "bad arguments");
    HLMC_CHECK_ARG(!h->impl->P.empty(), "net is not bound");
    ForwardArgs a{batch, train, z, nullptr, cond, nullptr, dropout, recon, recon_text, nullptr, nullptr, nullptr, ws,
                  false, true};
    return h->impl->forward(S(stream), a);
}
int hlmc_net_backward(hlmc_net* h, void* stream, int64_t batch, const float* d_recon, const float* d_recon_text,
                      const float* d_mu, const float* d_logvar, void* ws) {
    HLMC_CHECK_ARG(h && ws && d_recon && d_mu && d_logvar, "bad arguments");
    HLMC_TRY(device_status_ok());
    BackwardArgs a{batch, d_recon, d_recon_text, d_mu, d_logvar, ws};
    return h->impl->backward(S(stream), a);
}

int hlmc_net_adam_step(hlmc_net* h, void* stream, float* const* exp_avg, float* const* exp_avg_sq, float lr, float b1,
                       float b2, float eps, float wd, int step) {
    HLMC_CHECK_ARG(h && exp_avg && exp_avg_sq && step >= 1, "bad arguments");
    HLMC_CHECK_ARG(!h->impl->P.empty(), "net is not bound");
    return h->impl->adam_step(S(stream), exp_avg, exp_avg_sq, ops::AdamArgs{lr, b1, b2, eps, wd, step});
}
int hlmc_net_adam_step_dev(hlmc_net* h, void* stream, float* const* exp_avg, float* const* exp_avg_sq,
                           const float* coef_dev) {
    HLMC_CHECK_ARG(h && exp_avg && exp_avg_sq && coef_dev, "bad arguments");
    HLMC_CHECK_ARG(!h->impl->P.empty(), "net is not bound");
    return h->impl->adam_step(S(stream), exp_avg, exp_avg_sq, ops::AdamArgs{0.f, 0.f, 0.f, 0.f, 0.f, 1}, coef_dev);
}
int hlmc_adam_coef(float lr, float b1, float b2, float eps, float wd, int step, float* out6) {
    HLMC_CHECK_ARG(out6 && step >= 1, "bad arguments");
    ops::adam_coef_host(ops::AdamArgs{lr, b1, b2, eps, wd, step}, out6);
    return HLMC_OK;
}
int hlmc_net_set_trust_packs(hlmc_net* h, int trust) {
    HLMC_CHECK_ARG(h, "net is NULL");
    h->impl->trust_packs = trust != 0;
    if (!trust) h->impl->packs_valid = false;
    return HLMC_OK;
}
int hlmc_net_settle(hlmc_net* h, void* stream) {
    HLMC_CHECK_ARG(h, "net is NULL");
    return h->impl->settle(S(stream));
}
int hlmc_net_set_rng(hlmc_net* h, uint64_t seed, uint64_t offset) {
    HLMC_CHECK_ARG(h && offset % 4 == 0, "net is NULL / offset not a multiple of 4");
    h->impl->rng_seed = seed;
    h->impl->rng_offset = offset;
    return HLMC_OK;
}
int hlmc_net_get_rng(const hlmc_net* h, uint64_t* seed, uint64_t* offset) {
    HLMC_CHECK_ARG(h && seed && offset, "NULL argument");
    *seed = h->impl->rng_seed;
    *offset = h->impl->rng_offset;
    return HLMC_OK;
}
int hlmc_randn(void* stream, float* out, int64_t n, uint64_t seed, uint64_t offset) {
    return ops::randn(S(stream), out, n, seed, offset);
}
int hlmc_net_set_overlap_adam(hlmc_net* h, int enable) {
    HLMC_CHECK_ARG(h, "net is NULL");
    h->impl->overlap_adam = enable != 0;
    return HLMC_OK;
}
int hlmc_net_grad_buckets(const hlmc_net* h, int* starts, int cap) {
    HLMC_CHECK_ARG(h && starts && cap > 0, "NULL argument");
    const auto& b = h->impl->bucket_starts;
    for (int k = 0; k < (int)b.size() && k < cap; ++k) starts[k] = b[k];
    return (int)b.size();
}
int hlmc_net_set_bucket_sync(hlmc_net* h, int enable) {
    HLMC_CHECK_ARG(h, "net is NULL");
    h->impl->bucket_sync = enable != 0;
    return HLMC_OK;
}
int hlmc_net_bucket_wait(hlmc_net* h, int k, void* stream) {
    HLMC_CHECK_ARG(h, "net is NULL");
    auto& ev = h->impl->bucket_ev;
    HLMC_CHECK_ARG(h->impl->bucket_sync && k >= 0 && k < (int)ev.size() && ev[k],
                   "bucket events not recorded (hlmc_net_set_bucket_sync + hlmc_net_backward first)");
    HLMC_HIP(hipStreamWaitEvent(S(stream), ev[k], 0));
    return HLMC_OK;
}

// ------------------------------------------------------------------------------------ loss / optim
int64_t hlmc_loss_workspace(int64_t na, int64_t nt, int64_t nl) { return (int64_t)ops::vae_sums_ws(na, nt, nl); }
int hlmc_loss_sums(void* stream, const float* ra, const float* a, int64_t na, const float* rt, const float* t, int64_t nt,
                   const float* mu, const float* lv, int64_t nl, double* sums3, void* ws) {
    HLMC_CHECK_ARG(sums3 && ws && (na == 0 || (ra && a)) && (nt == 0 || (rt && t)) && (nl == 0 || (mu && lv)), "bad arguments");
    return ops::vae_sums(S(stream), ra, a, na, rt, t, nt, mu, lv, nl, sums3,
                         Ws{reinterpret_cast<float*>(ws), ops::vae_sums_ws(na, nt, nl)});
}
int hlmc_loss_backward(void* stream, const float* ra, const float* a, int64_t na, float* dra, const float* rt,
                       const float* t, int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl,
                       const float* coef, float* dmu, float* dlv) {
    HLMC_CHECK_ARG(coef && (na == 0 || (ra && a && dra)) && (nt == 0 || (rt && t && drt)) &&
                       (nl == 0 || (mu && lv && dmu && dlv)), "bad arguments");
    return ops::vae_loss_bwd(S(stream), ra, a, na, dra, rt, t, nt, drt, mu, lv, nl, coef, dmu, dlv);
}
int hlmc_loss_sums_backward(void* stream, const float* ra, const float* a, int64_t na, float* dra, const float* rt,
                            const float* t, int64_t nt, float* drt, const float* mu, const float* lv, int64_t nl,
                            const float* coef, float* dmu, float* dlv, double* sums3, void* ws) {
    HLMC_CHECK_ARG(coef && sums3 && ws && (na == 0 || (ra && a && dra)) && (nt == 0 || (rt && t && drt)) &&
                       (nl == 0 || (mu && lv && dmu && dlv)), "bad arguments");
    return ops::vae_sums_bwd(S(stream), ra, a, na, dra, rt, t, nt, drt, mu, lv, nl, coef, dmu, dlv, sums3,
                             Ws{reinterpret_cast<float*>(ws), ops::vae_sums_ws(na, nt, nl)});
}
int64_t hlmc_adam_scratch_bytes(int) { return 0; }
int hlmc_adam_step(void* stream, int n, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const int64_t* numel, float lr, float b1, float b2, float eps, float wd, int step, void* scratch) {
    HLMC_CHECK_ARG(n >= 0 && step >= 1 && p && g && m && v && numel, "bad adam arguments");
    ops::AdamArgs a{lr, b1, b2, eps, wd, step};
    (void)scratch;
    return ops::adam(S(stream), n, p, g, m, v, numel, a);
}

// ------------------------------------------------------------------------------------ kmeans
int hlmc_km_center(void* stream, const float* X, int64_t n, int d, float* mean, float* var, float* Xc) {
    return km::center(S(stream), X, n, d, mean, var, Xc);
}
int hlmc_km_sqdist_rows(void* stream, const float* X, int64_t n, int d, const int64_t* cand, int ncand, float* out) {
    return km::sqdist_rows(S(stream), X, n, d, cand, ncand, out);
}
int hlmc_km_assign(void* stream, const float* X, int64_t n, int d, const float* C, int k, int32_t* labels,
                   const int32_t* old, int32_t* n_changed) {
    return km::assign(S(stream), X, n, d, C, k, labels, old, n_changed);
}
int hlmc_km_sums(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, float* sums, float* w) {
    return km::sums(S(stream), X, n, d, labels, k, sums, w);
}
int64_t hlmc_km_sums_workspace(int64_t n, int k) { return (int64_t)km::sums_ws(n, k); }
int hlmc_km_sums_part(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, float* sums,
                      float* w, void* ws, int64_t ws_bytes) {
    return km::sums_part(S(stream), X, n, d, labels, k, sums, w, ws, (size_t)ws_bytes);
}
int hlmc_km_inertia(void* stream, const float* X, int64_t n, int d, const float* C, const int32_t* labels, float* out,
                    float* tmp) {
    return km::inertia(S(stream), X, n, d, C, labels, out, tmp);
}
int hlmc_km_assign_batch(void* stream, const float* X, int64_t n, int d, const float* C, int k, int R, uint64_t active,
                         int32_t* labels, const int32_t* old, int32_t* n_changed) {
    return km::assign_batch(S(stream), X, n, d, C, k, R, active, labels, old, n_changed);
}
int hlmc_km_sums_batch(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, int R,
                       uint64_t active, float* sums, float* w, void* ws, int64_t ws_bytes) {
    return km::sums_batch(S(stream), X, n, d, labels, k, R, active, sums, w, ws, (size_t)std::max<int64_t>(0, ws_bytes));
}
int hlmc_km_update_batch(void* stream, int k, int d, int R, uint64_t active, const float* sums, const float* w,
                         const float* C_old, float* C_new, float* info) {
    return km::update_batch(S(stream), k, d, R, active, sums, w, C_old, C_new, info);
}
int hlmc_km_pp_search(void* stream, int64_t n, int R, int T, const float* prev, int prevT, const int32_t* best,
                      const double* rvals, int64_t* cand, int32_t* amb) {
    return km::pp_search(S(stream), n, R, T, prev, prevT, best, rvals, cand, amb);
}
int hlmc_km_pp_dist(void* stream, const float* X, int64_t n, int d, int R, int T, const int64_t* cand, const float* prev,
                    int prevT, const int32_t* best, float* out) {
    return km::pp_dist(S(stream), X, n, d, R, T, cand, prev, prevT, best, out);
}
int hlmc_km_inertia_batch(void* stream, const float* X, int64_t n, int d, const float* C, int k, const int32_t* labels,
                          int R, float* out, float* tmp) {
    return km::inertia_batch(S(stream), X, n, d, C, k, labels, R, out, tmp);
}
int hlmc_km_rowdist(void* stream, const float* X, int64_t n, int d, const float* C, const int32_t* labels, float* out) {
    return km::rowdist(S(stream), X, n, d, C, labels, out);
}

// ------------------------------------------------------------------------------------ metrics
int64_t hlmc_silhouette_workspace(int64_t n, int k) { return (int64_t)metrics::silhouette_workspace(n, k); }
int hlmc_silhouette(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, double* samples,
                    double* score, void* ws, int64_t ws_bytes) {
    return metrics::silhouette(S(stream), X, n, d, labels, k, samples, score, ws, (size_t)ws_bytes);
}
int64_t hlmc_cluster_scores_workspace(int k, int d) { return (int64_t)metrics::cluster_scores_workspace(k, d); }
int hlmc_cluster_scores(void* stream, const float* X, int64_t n, int d, const int32_t* labels, int k, double* out2,
                        void* ws, int64_t ws_bytes) {
    return metrics::cluster_scores(S(stream), X, n, d, labels, k, out2, ws, (size_t)ws_bytes);
}


// ------------------------------------------------------------------------------------ op-level entries
// Individual GEMM-family kernels (the building blocks of hlmc_net_*), exposed for testing and reuse.
#define DT_DISPATCH(dtype, CALL_F32, CALL_BF16) ((dtype) == HLMC_BF16 ? (CALL_BF16) : (CALL_F32))
int hlmc_op_conv_s2(void* stream, int dtype, const void* x, int B, int Hi, int Wi, int Ci, const void* wp,
                    const float* bias, int Co, void* y, void* ws, int64_t ws_bytes) {
    Ws w{reinterpret_cast<float*>(ws), (size_t)ws_bytes};
    return DT_DISPATCH(dtype,
        ops::conv_s2<float>(S(stream), (const float*)x, B, Hi, Wi, Ci, (const float*)wp, bias, Co, (float*)y, w),
        ops::conv_s2<bf16>(S(stream), (const bf16*)x, B, Hi, Wi, Ci, (const bf16*)wp, bias, Co, (bf16*)y, w));
}
int hlmc_op_subpixel(void* stream, int dtype, const void* x, int B, int Hi, int Wi, int Ci, const void* wp,
                     const float* bias, int Co, void* y, void* ws, int64_t ws_bytes) {
    Ws w{reinterpret_cast<float*>(ws), (size_t)ws_bytes};
    return DT_DISPATCH(dtype,
        ops::subpixel<float>(S(stream), (const float*)x, B, Hi, Wi, Ci, (const float*)wp, bias, Co, (float*)y, w),
        ops::subpixel<bf16>(S(stream), (const bf16*)x, B, Hi, Wi, Ci, (const bf16*)wp, bias, Co, (bf16*)y, w));
}
int hlmc_op_wgrad_s2(void* stream, int dtype, const void* Lo, int B, int Hl, int Wl, int M, const void* Xh, int C,
                     float* dW, void* ws, int64_t ws_bytes) {
    Ws w{reinterpret_cast<float*>(ws), (size_t)ws_bytes};
    return DT_DISPATCH(dtype,
        ops::wgrad_s2<float>(S(stream), (const float*)Lo, B, Hl, Wl, M, (const float*)Xh, C, dW, w),
        ops::wgrad_s2<bf16>(S(stream), (const bf16*)Lo, B, Hl, Wl, M, (const bf16*)Xh, C, dW, w));
}
int hlmc_op_linear(void* stream, int dtype, const void* x, int ldx, int M, int K, const void* wt, int ldw,
                   const float* bias, int N, void* y, int ldy, int act, int accumulate, int out_f32, void* ws,
                   int64_t ws_bytes, const void* relu_ref) {
    Ws w{reinterpret_cast<float*>(ws), (size_t)ws_bytes};
    if (dtype == HLMC_BF16 && out_f32)
        return ops::linear<bf16, float>(S(stream), (const bf16*)x, ldx, M, K, (const bf16*)wt, ldw, bias, N, (float*)y,
                                        ldy, act, accumulate, w, (const float*)relu_ref);
    if (dtype == HLMC_BF16)
        return ops::linear<bf16, bf16>(S(stream), (const bf16*)x, ldx, M, K, (const bf16*)wt, ldw, bias, N, (bf16*)y,
                                       ldy, act, accumulate, w, (const bf16*)relu_ref);
    return ops::linear<float, float>(S(stream), (const float*)x, ldx, M, K, (const float*)wt, ldw, bias, N, (float*)y,
                                     ldy, act, accumulate, w, (const float*)relu_ref);
}
int hlmc_op_linear_wgrad(void* stream, int dtype, const void* dy, int lddy, const void* x, int ldx, int Mb, int N,
                         int K, float* dW, float* db, void* ws, int64_t ws_bytes) {
    Ws w{reinterpret_cast<float*>(ws), (size_t)ws_bytes};
    return DT_DISPATCH(dtype,
        ops::linear_wgrad<float>(S(stream), (const float*)dy, lddy, (const float*)x, ldx, Mb, N, K, dW, db, w),
        ops::linear_wgrad<bf16>(S(stream), (const bf16*)dy, lddy, (const bf16*)x, ldx, Mb, N, K, dW, db, w));
}
int hlmc_op_conv_c1_s2(void* stream, int dtype, const float* x, int B, int Hi, int Wi, const float* w,
                       const float* bias, int Co, void* y) {
    return DT_DISPATCH(dtype, ops::conv_c1_s2<float>(S(stream), x, B, Hi, Wi, w, bias, Co, (float*)y),
                       ops::conv_c1_s2<bf16>(S(stream), x, B, Hi, Wi, w, bias, Co, (bf16*)y));
}
int hlmc_op_convT_c1(void* stream, int dtype, const void* x, int B, int Hi, int Wi, int Ci, const float* w,
                     const float* bias, float* y) {
    return DT_DISPATCH(dtype, ops::convT_c1<float>(S(stream), (const float*)x, B, Hi, Wi, Ci, w, bias, y),
                       ops::convT_c1<bf16>(S(stream), (const bf16*)x, B, Hi, Wi, Ci, w, bias, y));
}
int hlmc_op_wgrad_c1(void* stream, int dtype, const void* Lo, int B, int Hl, int Wl, int M, const float* Xh,
                     float* dW, void* ws, int64_t ws_bytes) {
    Ws w{reinterpret_cast<float*>(ws), (size_t)ws_bytes};
    return DT_DISPATCH(dtype, ops::wgrad_c1<float>(S(stream), (const float*)Lo, B, Hl, Wl, M, Xh, dW, w),
                       ops::wgrad_c1<bf16>(S(stream), (const bf16*)Lo, B, Hl, Wl, M, Xh, dW, w));
}

// LDS halo-tile forward (conv_s2 / subpixel, bf16) with the train-mode epilogue statistics and, when gamma is given,
// the layer below's BatchNorm + LeakyReLU(0.01) applied while the input is staged (the engine's BnInput path):
// x is then the pre-BN map, whose exact statistics this entry first accumulates with the moments pass the engine's
// producers would have delivered.  out_sums[2 Co] = (sum y | sum y^2) over the stored bf16 outputs.
int64_t hlmc_op_bn_bwd_workspace(int C) {
    if (C <= 0) return 0;
    return (int64_t)(((ops::bn_acc_bytes(C) + 255) & ~(size_t)255) + ((ops::bias_acc_bytes(C) + 255) & ~(size_t)255) +
                     2 * (size_t)C * sizeof(float));
}
int hlmc_op_bn_bwd(void* stream, int dtype, const void* da, const void* y, int64_t R, int C, const float* mean,
                   const float* invstd, const float* gamma, const float* beta, void* dy, float* dgamma, float* dbeta,
                   float* dbias, void* ws, int64_t ws_bytes) {
    HLMC_CHECK_ARG(da && y && mean && invstd && gamma && beta && dy && dgamma && dbeta && ws && R > 1 && C > 0,
                   "hlmc_op_bn_bwd: arguments");
    HLMC_CHECK_ARG(ws_bytes >= hlmc_op_bn_bwd_workspace(C), "hlmc_op_bn_bwd: workspace too small");
    HLMC_TRY(device_status_ok());
    hipStream_t s = S(stream);
    unsigned char* w = static_cast<unsigned char*>(ws);
    const size_t o1 = (ops::bn_acc_bytes(C) + 255) & ~(size_t)255, o2 = o1 + ((ops::bias_acc_bytes(C) + 255) & ~(size_t)255);
    HLMC_HIP(hipMemsetAsync(ws, 0, o2, s));
    XAcc mom{reinterpret_cast<unsigned long long*>(w), xacc_shards(C), 2 * C};
    XAcc bacc{reinterpret_cast<unsigned long long*>(w + o1), xacc_shards(C), C};
    float* sums = reinterpret_cast<float*>(w + o2);
    return DT_DISPATCH(dtype,
        ops::bn_act_bwd<float>(s, (const float*)da, C, (const float*)y, R, C, mean, invstd, gamma, beta, 0, nullptr,
                               1.f, (float*)dy, dgamma, dbeta, mom, nullptr, dbias ? bacc : XAcc{}, dbias, sums),
        ops::bn_act_bwd<bf16>(s, (const bf16*)da, C, (const bf16*)y, R, C, mean, invstd, gamma, beta, 0, nullptr, 1.f,
                              (bf16*)dy, dgamma, dbeta, mom, nullptr, dbias ? bacc : XAcc{}, dbias, sums));
}
static size_t halo_acc_off(int Ci) { return (XAcc::bytes(xacc_shards(Ci), 2 * Ci) + 255) & ~(size_t)255; }
int64_t hlmc_op_halo_workspace(int Ci, int Co) {
    return (int64_t)(halo_acc_off(Ci) + XAcc::bytes(xacc_shards(Co), 2 * Co));
}
int hlmc_op_halo_fwd(void* stream, int kind, const void* x, int B, int Hi, int Wi, int Ci, const void* wp,
                     const float* bias, int Co, void* y, double* out_sums, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum, float eps,
                     float* mean_out, float* invstd_out, void* a_out, void* ws, int64_t ws_bytes) {
    HLMC_CHECK_ARG(kind == 0 || kind == 1, "hlmc_op_halo_fwd: kind 0 (conv_s2) or 1 (subpixel)");
    HLMC_CHECK_ARG(out_sums && ws && ws_bytes >= hlmc_op_halo_workspace(Ci, Co), "hlmc_op_halo_fwd: workspace / out_sums");
    const bool xin = gamma != nullptr;
    HLMC_CHECK_ARG(kind == 0 ? ops::conv_s2_takes_input_bn<bf16>(B, Hi, Wi, Ci, Co)
                             : ops::subpixel_takes_input_bn<bf16>(B, Hi, Wi, Ci, Co),
                   "hlmc_op_halo_fwd: not an LDS halo-tile shape");
    if (xin) HLMC_CHECK_ARG(beta && mean_out && invstd_out && a_out, "hlmc_op_halo_fwd: input BatchNorm arguments");
    hipStream_t s = S(stream);
    unsigned char* w = static_cast<unsigned char*>(ws);
    XAcc ain{reinterpret_cast<unsigned long long*>(w), xacc_shards(Ci), 2 * Ci};
    XAcc aout{reinterpret_cast<unsigned long long*>(w + halo_acc_off(Ci)), xacc_shards(Co), 2 * Co};
    HLMC_HIP(hipMemsetAsync(ws, 0, (size_t)hlmc_op_halo_workspace(Ci, Co), s));
    const int64_t R = (int64_t)B * Hi * Wi;
    ops::BnInput bi{};
    if (xin) {
        HLMC_TRY(ops::bn_moments<bf16>(s, (const bf16*)x, R, Ci, ain));
        bi.acc = ain; bi.R = R; bi.mean = mean_out; bi.invstd = invstd_out; bi.rmean = running_mean;
        bi.rvar = running_var; bi.nbt = num_batches_tracked; bi.momentum = momentum; bi.eps = eps; bi.gamma = gamma;
        bi.beta = beta; bi.a_out = a_out;
    }
    ops::ColStats st{aout, false};
    Ws none{nullptr, 0};
    if (kind == 0)
        HLMC_TRY(ops::conv_s2<bf16>(s, (const bf16*)x, B, Hi, Wi, Ci, (const bf16*)wp, bias, Co, (bf16*)y, none, &st,
                                    xin ? &bi : nullptr));
    else
        HLMC_TRY(ops::subpixel<bf16>(s, (const bf16*)x, B, Hi, Wi, Ci, (const bf16*)wp, bias, Co, (bf16*)y, none, &st,
                                     xin ? &bi : nullptr));
    HLMC_CHECK_ARG(st.done, "hlmc_op_halo_fwd: statistics not delivered by the halo kernel");
    return ops::colsum_to_f64(s, aout, 2 * Co, out_sums);
}

}  // extern "C"
