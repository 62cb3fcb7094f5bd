// Native VAE engine.  Each reference model is a fixed schedule of libhlmc kernels:
//   HybridVAE      src/Convolutional_VAE.py:75-185  (+ audio-only variant)
//   ConditionalVAE src/Conditional_VAE.py:109-231
//   VAE (Simple)   src/Simple_VAE.py:47-105
// Activations are NHWC in T (float or bf16), every saved tensor lives in the caller's workspace,
// parameters are the caller's fp32 tensors (torch registration order), gradients are overwritten.
#include "engine.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <functional>

namespace hlmc {
namespace {

constexpr float kBnEps = 1e-5f;
constexpr float kBnMomentum = 0.1f;
constexpr int ENC_CH[7] = {1, 32, 64, 128, 256, 512, 512};
constexpr int DEC_CH[7] = {512, 512, 256, 128, 64, 32, 1};

inline int pad8(int64_t n) { return (int)((n + 7) & ~int64_t(7)); }

template <typename T>
class NetT : public NetBase {
  public:
    // ---------------------------------------------------------------- packing of GEMM weights
    struct Pack {
        int d0 = 0, d1 = 0, taps = 0, ld0 = 0, ld1 = 0;
        size_t off0 = SIZE_MAX, off1 = SIZE_MAX;
    };
    std::vector<Pack> packs;
    size_t jobs_off = 0, ajobs_off = 0, state_size = 0;
    int njobs = 0, pack_tiles = 0, adam_tiles = 0;
    std::vector<ops::AdamJob> ajobs;  // host copy of the uploaded Adam job list (kept alive for the async copy)
    std::vector<float*> ajobs_m, ajobs_v;

    void register_pack(int widx, int taps) {
        if ((int)packs.size() < (int)params.size()) packs.resize(params.size());
        Pack& p = packs[widx];
        const auto& sh = params[widx].shape;
        p.d0 = (int)sh[0];
        p.d1 = (int)sh[1];
        p.taps = taps;
    }
    void finalize_state() {
        packs.resize(params.size());
        Arena A;
        for (auto& p : packs) {
            if (!p.taps) continue;
            p.ld0 = p.taps == 1 ? pad8(p.d1) : p.d1;
            p.ld1 = p.taps == 1 ? pad8(p.d0) : p.d0;
            p.off0 = A.take((size_t)p.d0 * p.taps * p.ld0 * sizeof(T));
            p.off1 = A.take((size_t)p.d1 * p.taps * p.ld1 * sizeof(T));
            ++njobs;
        }
        jobs_off = A.take(sizeof(ops::AdamJob) * std::max<size_t>(1, njobs));
        ajobs_off = A.take(sizeof(ops::AdamJob) * std::max<size_t>(1, params.size()));
        state_size = A.used;
    }
    size_t state_bytes() const override { return state_size; }
    ops::AdamJob job_for(size_t i, float* m, float* v) const {
        const Pack& p = packs[i];
        ops::AdamJob j{P[i], G[i], m, v, nullptr, nullptr, params[i].numel(), 0, 0, 0, 0, 0, 0, 0};
        if (p.taps) {
            j.p0 = state + p.off0;
            j.p1 = state + p.off1;
            j.d0 = p.d0; j.d1 = p.d1; j.taps = p.taps; j.ld0 = p.ld0; j.ld1 = p.ld1;
        }
        return j;
    }
    std::vector<ops::AdamJob> pjobs;
    int bind_state(hipStream_t s) override {
        pjobs.clear();
        pack_tiles = 0;
        for (size_t i = 0; i < packs.size(); ++i) {
            if (!packs[i].taps) continue;
            ops::AdamJob j = job_for(i, nullptr, nullptr);
            j.tile0 = pack_tiles;
            pack_tiles += ops::adam_job_tiles(j);
            pjobs.push_back(j);
        }
        if (!pjobs.empty())
            HLMC_HIP(hipMemcpyAsync(state + jobs_off, pjobs.data(), pjobs.size() * sizeof(ops::AdamJob), hipMemcpyHostToDevice, s));
        ajobs_m.clear();  // Adam job list is rebuilt on the next adam_step (parameter pointers changed)
        HLMC_HIP(hipStreamSynchronize(s));
        return HLMC_OK;
    }
    int pack_all(hipStream_t s) {
        if (trust_packs && packs_valid) return HLMC_OK;
        HLMC_TRY(ops::pack<T>(s, reinterpret_cast<const ops::AdamJob*>(state + jobs_off), njobs, pack_tiles));
        packs_valid = true;
        return HLMC_OK;
    }
    int adam_step(hipStream_t s, float* const* m, float* const* v, const ops::AdamArgs& a, const float* coef_dev) override {
        // one launch: torch-Adam update of every parameter + refresh of the packed GEMM weights
        const size_t np = params.size();
        if (ajobs_m.size() != np || !std::equal(ajobs_m.begin(), ajobs_m.end(), m) ||
            !std::equal(ajobs_v.begin(), ajobs_v.end(), v)) {
            ajobs_m.assign(m, m + np);
            ajobs_v.assign(v, v + np);
            ajobs.clear();
            adam_tiles = 0;
            for (size_t i = 0; i < np; ++i) {
                ops::AdamJob j = job_for(i, m[i], v[i]);
                j.tile0 = adam_tiles;
                adam_tiles += ops::adam_job_tiles(j);
                ajobs.push_back(j);
            }
            HLMC_HIP(hipMemcpyAsync(state + ajobs_off, ajobs.data(), ajobs.size() * sizeof(ops::AdamJob),
                                    hipMemcpyHostToDevice, s));
        }
        const auto* jd = reinterpret_cast<const ops::AdamJob*>(state + ajobs_off);
        if (join_pending) {
            // every gradient but the late ones is final once the side stream passed prelate_ev
            const int tsplit = ajobs[this->late_params].tile0;
            HLMC_HIP(hipStreamWaitEvent(s, prelate_ev, 0));
            HLMC_TRY(ops::adam_pack<T>(s, jd, (int)np, adam_tiles, a, coef_dev, tsplit));
            HLMC_TRY(join(s));
            join_pending = false;
            HLMC_TRY(ops::adam_pack<T>(s, jd, (int)np, tsplit, a, coef_dev, 0));
        } else {
            HLMC_TRY(ops::adam_pack<T>(s, jd, (int)np, adam_tiles, a, coef_dev));
        }
        packs_valid = true;
        return HLMC_OK;
    }
    T* P0(int w) const { return reinterpret_cast<T*>(state + packs[w].off0); }
    T* P1(int w) const { return reinterpret_cast<T*>(state + packs[w].off1); }
    int ld0(int w) const { return packs[w].ld0; }
    int ld1(int w) const { return packs[w].ld1; }

    // ---------------------------------------------------------------- workspace
    char* ws = nullptr;
    Ws scratch{nullptr, 0};
    Ws scratch2{nullptr, 0};  // split-K / reduction scratch of the weight-gradient stream
    size_t scratch_off = 0, scratch2_off = 0, scratch_bytes = 0;
    int64_t planned_B = -1;
    size_t ws_total = 0;

    T* AT(size_t off) const { return reinterpret_cast<T*>(ws + off); }
    float* AF(size_t off) const { return reinterpret_cast<float*>(ws + off); }
    uint8_t* AU8(size_t off) const { return reinterpret_cast<uint8_t*>(ws + off); }

    void need(size_t b) { scratch_bytes = std::max(scratch_bytes, b); }
    // exact statistics accumulators (common.hpp XAcc): every BatchNorm layer's forward statistics in one region, its
    // backward moments and bias column sums in the next; zeroed by one memset per train forward (and by backward
    // when it runs again without a forward in between)
    size_t xf_total = 0, xb_total = 0, xf_base = 0, xb_base = 0;
    bool bwd_acc_clean = false;
    int zero_acc_fwd(hipStream_t s) {
        if (xf_total + xb_total) HLMC_HIP(hipMemsetAsync(ws + xf_base, 0, xf_total + xb_total, s));
        bwd_acc_clean = true;
        return HLMC_OK;
    }
    int zero_acc_bwd(hipStream_t s) {
        if (!bwd_acc_clean && xb_total) HLMC_HIP(hipMemsetAsync(ws + xb_base, 0, xb_total, s));
        bwd_acc_clean = false;
        return HLMC_OK;
    }

    virtual void plan(Arena& A, int64_t B) = 0;
    size_t ws_bytes(int64_t B) override {
        if (B != planned_B) {
            Arena A;
            scratch_bytes = 0;
            xf_total = xb_total = 0;
            plan(A, B);
            scratch_off = A.take(scratch_bytes + 256);
            scratch2_off = A.take(scratch_bytes + 256);
            xf_base = A.take(xf_total);  // xb directly after xf (one memset covers both: 256-aligned sizes)
            xb_base = A.take(xb_total);
            ws_total = A.used;
            planned_B = B;
        }
        return ws_total;
    }
    void set_ws(void* w) {
        ws = reinterpret_cast<char*>(w);
        scratch = Ws{reinterpret_cast<float*>(ws + scratch_off), scratch_bytes + 256};
        scratch2 = Ws{reinterpret_cast<float*>(ws + scratch2_off), scratch_bytes + 256};
    }

    // ---------------------------------------------------------------- weight-gradient stream
    // Weight and bias gradients have no consumer before Adam.  backward() forks them onto a second stream
    // (own split-K scratch) right after the data gradient they read is written, so the critical path stays
    // dgrad -> BN-backward -> dgrad and the wgrad GEMMs / reduces fill the CUs it leaves idle.  Every buffer
    // a forked op reads is written once per backward; backward() joins the stream before returning.
    // HLMC_SIDE_STREAM=0 keeps everything on the caller's stream (A/B measurement aid).
    hipStream_t s2 = nullptr;
    std::vector<hipEvent_t> evs;
    int ev_next = 0;
    bool use_side = true;
    hipEvent_t prelate_ev = nullptr;  // side stream passed every weight gradient except the late ones
    bool join_pending = false;         // backward left the side stream running (NetBase::overlap_adam)
    ~NetT() override {
        if (s2) (void)hipStreamDestroy(s2);
        for (auto e : evs) (void)hipEventDestroy(e);
        for (auto e : this->bucket_ev) (void)hipEventDestroy(e);
        if (prelate_ev) (void)hipEventDestroy(prelate_ev);
    }
    bool tail_overlap() const { return use_side && this->overlap_adam && !this->bucket_sync && this->late_params > 0; }
    // called in backward once every non-late weight gradient has been issued
    int prelate(hipStream_t s) {
        if (!tail_overlap()) return HLMC_OK;
        HLMC_TRY(flush_side(s));
        HLMC_TRY(fork(s));
        HLMC_HIP(hipEventRecord(prelate_ev, s2));
        return HLMC_OK;
    }
    // end of backward: join the weight-gradient stream, or leave it to adam_step (tail overlap)
    // a pending tail (backward without the adam_step that joins it) is joined before anything else runs
    int settle(hipStream_t s) override {
        if (!join_pending) return HLMC_OK;
        join_pending = false;
        return join(s);
    }
    int finish_backward(hipStream_t s) {
        if (tail_overlap()) {
            join_pending = true;
            return HLMC_OK;
        }
        return join(s);
    }
    int side_init() {
        static const bool env_off = [] {
            const char* e = std::getenv("HLMC_SIDE_STREAM");
            return e && e[0] == '0';
        }();
        use_side = !env_off;
        if (use_side && !s2) {
            // (default priority: the lowest priority removed the main queue's resource waits in the profile,
            // 322 -> 108 us per step, but the step was 0.4% slower, 3 alternating rounds)
            HLMC_HIP(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
            evs.resize(32);
            const unsigned fl = hipEventDisableTiming | fork_event_scope();
            for (auto& e : evs) HLMC_HIP(hipEventCreateWithFlags(&e, fl));
            HLMC_HIP(hipEventCreateWithFlags(&prelate_ev, fl));
        }
        if (this->bucket_sync && this->bucket_ev.size() != this->bucket_starts.size()) {
            for (auto e : this->bucket_ev) (void)hipEventDestroy(e);
            this->bucket_ev.assign(this->bucket_starts.size(), nullptr);
            for (auto& e : this->bucket_ev) HLMC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        return HLMC_OK;
    }
    // fence of the fork / join events.  Both streams run on this device: the kernels' own device-scope
    // release / acquire order every cross-stream hand-off, and the system-scope fence HIP adds to an event by
    // default (host visibility, which no fork needs) is what made every fork a main-stream bubble.  Measured (3
    // alternating rounds): hipEventDisableSystemFence 126.7k vs 125.1k clips/s with HIP's default and 125.0k with
    // hipEventReleaseToDevice
    static unsigned fork_event_scope() { return (unsigned)hipEventDisableSystemFence; }
    hipEvent_t next_ev() {
        hipEvent_t e = evs[ev_next];
        ev_next = (ev_next + 1) % (int)evs.size();
        return e;
    }
    // the weight-gradient stream continues after everything issued so far on s
    int fork(hipStream_t s) {
        hipEvent_t e = next_ev();
        HLMC_HIP(hipEventRecord(e, s));
        HLMC_HIP(hipStreamWaitEvent(s2, e, 0));
        return HLMC_OK;
    }
    int join(hipStream_t s) {
        if (!use_side || !s2) return HLMC_OK;
        HLMC_TRY(flush_side(s));
        hipEvent_t e = next_ev();
        HLMC_HIP(hipEventRecord(e, s2));
        HLMC_HIP(hipStreamWaitEvent(s, e, 0));
        return HLMC_OK;
    }
    // Weight-gradient work queued for the second stream.  A fork (event record on s, wait on s2) costs the main
    // stream a ~6 us bubble (measured: scripts/step_gaps.py), so queued work is issued in batches behind one
    // fork: the queue is flushed once it holds `batch` items (and by join / mark / prelate).  Every buffer a
    // queued op reads is written once per backward, so issuing it later is safe; it only waits longer.
    using SideFn = std::function<int(hipStream_t, Ws)>;
    std::vector<SideFn> side_q;
    int issue_side() {
        int rc = HLMC_OK;
        for (auto& f : side_q)
            if (rc == HLMC_OK) rc = f(s2, scratch2);
        side_q.clear();
        return rc;
    }
    int flush_side(hipStream_t s) {
        if (side_q.empty()) return HLMC_OK;
        HLMC_TRY(fork(s));
        return issue_side();
    }
    // queue f(stream, scratch) for the weight-gradient stream (ordered after the work issued so far on s);
    // inline on s without the second stream
    int defer_side(hipStream_t s, SideFn f, int batch) {
        if (!use_side) return f(s, scratch);
        side_q.push_back(std::move(f));
        return (int)side_q.size() >= batch ? flush_side(s) : HLMC_OK;
    }
    // conv layers / dense layers per fork.  Measured on the bench step (scripts/gpu_r3_knobs.sh, 3 alternating
    // rounds): conv 1 / dense 1 108.4k, 2 / 1 109.7k, 2 / 2 110.3k, 3 / 1 108.2k, 6 / 1 104.3k (the weight-gradient
    // stream starts too late), 2 / 9 108.1k
    static constexpr int side_batch() { return 2; }
    static constexpr int dense_batch() { return 2; }
    // run f on the weight-gradient stream now (with everything queued before it)
    int side(hipStream_t s, SideFn f) { return defer_side(s, std::move(f), 1); }
    // weight gradients of the dense layers: on the second stream (measured round 1: 93.3k vs 86.5k clips/s inline)
    bool dense_side_on() const { return use_side; }
    // bucket k of the data-parallel all-reduce is final once both streams pass this point
    int mark(hipStream_t s, int k) {
        if (!this->bucket_sync) return HLMC_OK;
        HLMC_CHECK_ARG(k >= 0 && k < (int)this->bucket_ev.size(), "bucket index");
        if (use_side && k + 1 < (int)this->bucket_ev.size()) {
            if (side_q.empty()) HLMC_TRY(fork(s));
            else HLMC_TRY(flush_side(s));
            HLMC_HIP(hipEventRecord(this->bucket_ev[k], s2));
        } else {  // the last bucket: the caller has joined the weight-gradient stream
            HLMC_HIP(hipEventRecord(this->bucket_ev[k], s));
        }
        return HLMC_OK;
    }

    // ---------------------------------------------------------------- reparameterisation
    // z = mu + eps * exp(0.5 logvar): eps from the caller (copied to eps_keep by the same launch) or,
    // when the caller passes none, drawn on the device from the net's Philox stream (hlmc_net_set_rng) straight
    // into eps_keep (the backward's copy) — no host / torch launch for the noise
    // mu_out / lv_out (nullable): the caller's latent outputs, written by the same launch
    int reparam(hipStream_t s, const float* eps_in, const float* mu, const float* lv, float* eps_keep, int B, int L,
                T* z, int ldz, float* mu_out, float* lv_out) {
        if (eps_in) return ops::reparam_fwd<T>(s, mu, lv, eps_in, B, L, z, ldz, mu_out, lv_out, eps_keep);
        const uint64_t off = this->rng_offset;
        this->rng_offset += ((uint64_t)B * L + 3) & ~uint64_t(3);
        return ops::reparam_rng<T>(s, mu, lv, this->rng_seed, off, B, L, eps_keep, z, ldz, mu_out, lv_out);
    }
    // encode only: the latent outputs
    int latent_out(hipStream_t s, const ForwardArgs& a, const float* mu, const float* lv, int64_t nl) {
        const ops::CopySeg cs[2] = {{a.mu, mu, nl}, {a.logvar, lv, nl}};
        return ops::copy_segments(s, cs, 2);
    }

    // ---------------------------------------------------------------- layer helpers
    // y = act(x W^T + b)
    template <typename OutT>
    int lin_fwd(hipStream_t s, const T* x, int ldx, int B, int w, int b, OutT* y, int ldy, int act, int acc = 0) {
        const int N = (int)params[w].shape[0], K = (int)params[w].shape[1];
        return ops::linear<T, OutT>(s, x, ldx, B, K, P0(w), ld0(w), b >= 0 ? P[b] : nullptr, N, y, ldy, act, acc, scratch);
    }
    void lin_need(int B, int w) {
        const int N = (int)params[w].shape[0], K = (int)params[w].shape[1];
        need(ops::linear_ws<T>(B, K, N));
        need(ops::linear_ws<T>(B, N, K));
        need(ops::linear_wgrad_ws<T>(B, N, K));
    }
    // grads of a linear layer from dy (pre-activation grad).  The dense middle of the backward is bound by the
    // host's launch rate (measured: 40-100 us main-stream gaps per layer, scripts/step_gaps.py), so per layer:
    // the fork's event first, then dx (+=) on s — the critical path, with the ReLU backward of the layer below
    // (relu_ref: its post-ReLU output) in the epilogue — then dW and db as ONE weight-gradient GEMM (a ones
    // column on x gives db) on the weight-gradient stream: 2-3 launches where there were 6-7.
    int lin_bwd(hipStream_t s, const T* dy, int lddy, const T* x, int ldx, int B, int w, int b, T* dx, int lddx,
                int acc = 0, const T* relu_ref = nullptr) {
        const int N = (int)params[w].shape[0], K = (int)params[w].shape[1];
        float* gw = G[w];
        float* gb = b >= 0 ? G[b] : nullptr;
        SideFn wg = [=](hipStream_t q, Ws sc) { return ops::linear_wgrad<T>(q, dy, lddy, x, ldx, B, N, K, gw, gb, sc); };
        if (!dense_side_on()) {
            if (dx)
                HLMC_TRY(ops::linear<T, T>(s, dy, lddy, B, N, P1(w), ld1(w), nullptr, K, dx, lddx, 0, acc, scratch, relu_ref));
            return wg(s, scratch);
        }
        side_q.push_back(std::move(wg));
        const bool go = (int)side_q.size() >= dense_batch();
        if (go) HLMC_TRY(fork(s));
        if (dx)
            HLMC_TRY(ops::linear<T, T>(s, dy, lddy, B, N, P1(w), ld1(w), nullptr, K, dx, lddx, 0, acc, scratch, relu_ref));
        return go ? issue_side() : HLMC_OK;
    }

    struct BnBufs {
        size_t mean = 0, inv = 0, sums = 0;
        size_t xf = 0, xb = 0, xbias = 0;  // offsets in the forward / backward accumulator regions
        int C = 0;
    };
    static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }
    BnBufs bn_plan(Arena& A, int C) {
        BnBufs b;
        b.C = C;
        b.mean = A.take(C * 4);
        b.inv = A.take(C * 4);
        b.sums = A.take(2 * C * 4);
        b.xf = xf_total;
        xf_total += al256(ops::bn_acc_bytes(C));
        b.xb = xb_total;
        xb_total += al256(ops::bn_acc_bytes(C));
        b.xbias = xb_total;
        xb_total += al256(ops::bias_acc_bytes(C));
        return b;
    }
    XAcc acc_at(size_t off, int C, int ncols) const {
        return XAcc{reinterpret_cast<unsigned long long*>(ws + off), xacc_shards(C), ncols};
    }
    XAcc acc_fwd(const BnBufs& b) const { return acc_at(xf_base + b.xf, b.C, 2 * b.C); }
    XAcc acc_mom(const BnBufs& b) const { return acc_at(xb_base + b.xb, b.C, 2 * b.C); }
    XAcc acc_bias(const BnBufs& b) const { return acc_at(xb_base + b.xbias, b.C, b.C); }
    // st: statistics already delivered by the producing kernel (st->done), else a moments pass first
    int bn_fwd(hipStream_t s, bool train, const T* y, int64_t R, int C, int bn, const BnBufs& bb, int g, int beta, int act,
               const uint8_t* mask, float mscale, T* a, int lda, const ops::ColStats* st = nullptr) {
        float* mean = AF(bb.mean);
        float* inv = AF(bb.inv);
        if (train)  // statistics finalized inside the activation kernel
            return ops::bn_act_train<T>(s, y, R, C, acc_fwd(bb), st && st->done, mean, inv, RM[bn], RV[bn], NBT[bn],
                                        kBnMomentum, kBnEps, P[g], P[beta], act, mask, mscale, a, lda);
        HLMC_TRY(ops::bn_eval_stats(s, RM[bn], RV[bn], C, kBnEps, mean, inv));
        return ops::bn_act<T>(s, y, R, C, mean, inv, P[g], P[beta], act, mask, mscale, a, lda);
    }
    // fused: moments delivered by the kernel that wrote da (nullable); bias_side: the conv bias column sums are
    // reduced into the gradient on the weight-gradient stream (else here)
    // defer_bias: leave the bias reduction to the next side_bias() call (one fork for it and the layer's weight
    // gradient: every fork puts an event marker on the main stream, measured as a ~10 us bubble)
    int bn_bwd(hipStream_t s, const T* da, int lda, const T* y, int64_t R, int C, const BnBufs& bb, int g, int beta,
               int act, const uint8_t* mask, float mscale, T* dy, int bias, const ops::BnBwdFuse* fused = nullptr,
               bool bias_side = false, bool defer_bias = false) {
        const bool on_side = bias >= 0 && use_side && bias_side;
        const XAcc bacc = bias >= 0 ? acc_bias(bb) : XAcc{};
        HLMC_TRY(ops::bn_act_bwd<T>(s, da, lda, y, R, C, AF(bb.mean), AF(bb.inv), P[g], P[beta], act, mask, mscale, dy,
                                    G[g], G[beta], acc_mom(bb), fused, bacc,
                                    (bias >= 0 && !on_side) ? G[bias] : nullptr, AF(bb.sums)));
        if (on_side) {
            float* gb = G[bias];
            if (defer_bias)
                pend_bias = PendingBias{bacc, C, gb};
            else
                HLMC_TRY(side(s, [=](hipStream_t q, Ws) { return ops::colsum_finalize(q, bacc, C, gb); }));
        }
        return HLMC_OK;
    }
    struct PendingBias {
        XAcc acc;
        int C = 0;
        float* gb = nullptr;
    };
    PendingBias pend_bias;
    PendingBias take_bias() {
        const PendingBias pb = pend_bias;
        pend_bias = PendingBias{};
        return pb;
    }
    // f on the weight-gradient stream, after the bias reduction a preceding bn_bwd(defer_bias) left pending
    // (queued: flushed every side_batch() layers)
    int side_bias(hipStream_t s, SideFn f) {
        const PendingBias pb = pend_bias;
        pend_bias = PendingBias{};
        return defer_side(s, [pb, f](hipStream_t q, Ws sc) {
            if (pb.gb) HLMC_TRY(ops::colsum_finalize(q, pb.acc, pb.C, pb.gb));
            return f(q, sc);
        }, side_batch());
    }
    ops::BnBwdFuse fuse4{};  // the decoder's last BN layer: moments from the output convT's data gradient

    // ---------------------------------------------------------------- conv encoder (6 x conv-BN-LReLU)
    struct Enc {
        int w[6], b[6], g[6], beta[6], bn[6];
        int H = 0, W = 0;
        size_t y[6], a[6], dy[6];  // dy: grad wrt the conv output (read by the forked wgrad)
        // the caller's input of the last full forward: the first conv's weight gradient reads it in backward (the
        // ABI contract keeps in0 alive and unchanged until then: hlmc.h hlmc_net_forward)
        const float* audio = nullptr;
        BnBufs bb[6];
    };
    Enc enc;
    void enc_register(const std::string& prefix) {
        for (int l = 0; l < 6; ++l) {
            const int ci = ENC_CH[l], co = ENC_CH[l + 1];
            enc.w[l] = add_param(prefix + "." + std::to_string(3 * l) + ".weight", {co, ci, 3, 3});
            enc.b[l] = add_param(prefix + "." + std::to_string(3 * l) + ".bias", {co});
            enc.g[l] = add_param(prefix + "." + std::to_string(3 * l + 1) + ".weight", {co});
            enc.beta[l] = add_param(prefix + "." + std::to_string(3 * l + 1) + ".bias", {co});
            enc.bn[l] = add_bn();
            if (l > 0) register_pack(enc.w[l], 9);
        }
    }
    void enc_plan(Arena& A, int64_t B) {
        int h = enc.H, w = enc.W;
        for (int l = 0; l < 6; ++l) {
            const int ci = ENC_CH[l], co = ENC_CH[l + 1];
            if (l > 0) {
                need(ops::conv_s2_ws<T>((int)B, h, w, ci, co));
                need(ops::subpixel_ws<T>((int)B, h / 2, w / 2, co, ci));
                need(ops::wgrad_s2_ws<T>((int)B, h / 2, w / 2, co, ci));
            } else {
                need(ops::wgrad_c1_ws((int)B, h / 2, w / 2, co));
            }
            h /= 2;
            w /= 2;
            const size_t n = (size_t)B * h * w * co;
            enc.y[l] = A.take(n * sizeof(T));
            enc.a[l] = A.take(n * sizeof(T));
            enc.dy[l] = A.take(n * sizeof(T));
            enc.bb[l] = bn_plan(A, co);
        }
    }
    size_t enc_max_elems(int64_t B) const { return (size_t)B * (enc.H / 2) * (enc.W / 2) * 32; }
    // train-mode BatchNorm + LeakyReLU of layer l's output applied by the next conv while it stages its input
    // (ops::BnInput: the LDS halo-tile kernels) instead of a bn_act pass; the activation is written by that kernel
    ops::BnInput bn_input(const BnBufs& bb, int bn, int g, int beta, int64_t R, size_t a_off) {
        return ops::BnInput{acc_fwd(bb), R, AF(bb.mean), AF(bb.inv), RM[bn], RV[bn], NBT[bn], kBnMomentum, kBnEps,
                            P[g], P[beta], ws + a_off};
    }
    int enc_fwd(hipStream_t s, bool train, const float* audio_in, int B) {
        int h = enc.H, w = enc.W;
        HLMC_CHECK_ARG(audio_in, "audio input required");
        const float* audio = audio_in;
        enc.audio = audio_in;
        bool fused_prev = false;  // layer l-1's BatchNorm + activation is applied inside layer l's conv
        ops::BnInput xin{};
        for (int l = 0; l < 6; ++l) {
            const int ci = ENC_CH[l], co = ENC_CH[l + 1];
            T* y = AT(enc.y[l]);
            // train mode: BN statistics from the producing conv's epilogue
            ops::ColStats st{train ? acc_fwd(enc.bb[l]) : XAcc{}, false};
            if (l == 0)  // BN statistics from the edge conv itself (no col_moments pass)
                HLMC_TRY(ops::conv_c1_s2<T>(s, audio, B, h, w, P[enc.w[0]], P[enc.b[0]], co, y, &st));
            else
                HLMC_TRY(ops::conv_s2<T>(s, fused_prev ? AT(enc.y[l - 1]) : AT(enc.a[l - 1]), B, h, w, ci, P0(enc.w[l]),
                                         P[enc.b[l]], co, y, scratch, &st, fused_prev ? &xin : nullptr));
            h /= 2;
            w /= 2;
            const int64_t R = (int64_t)B * h * w;
            fused_prev = train && l + 1 < 6 && ops::conv_s2_takes_input_bn<T>(B, h, w, co, ENC_CH[l + 2]);
            if (fused_prev) {
                if (!st.done) HLMC_TRY(ops::bn_moments<T>(s, y, R, co, acc_fwd(enc.bb[l])));  // e.g. a split-K producer
                xin = bn_input(enc.bb[l], enc.bn[l], enc.g[l], enc.beta[l], R, enc.a[l]);
            } else
                HLMC_TRY(bn_fwd(s, train, y, R, co, enc.bn[l], enc.bb[l], enc.g[l], enc.beta[l], 0, nullptr, 1.f,
                                AT(enc.a[l]), co, &st));
        }
        return HLMC_OK;
    }
    // gA: grad of the last activation on entry (overwritten: data-gradient chain buffer).  Bucket
    // `bucket_hi` (layers 3..5) is marked final after layer 3 (-1: no mark).
    int enc_bwd(hipStream_t s, int B, T* gA, int bucket_hi = -1) {
        const float* audio = enc.audio;
        HLMC_CHECK_ARG(audio, "backward: no forward input recorded");
        int hs[7], ws_[7];
        hs[0] = enc.H;
        ws_[0] = enc.W;
        for (int l = 0; l < 6; ++l) { hs[l + 1] = hs[l] / 2; ws_[l + 1] = ws_[l] / 2; }
        for (int l = 5; l >= 0; --l) {
            const int ci = ENC_CH[l], co = ENC_CH[l + 1];
            const int ho = hs[l + 1], wo = ws_[l + 1];
            const int64_t R = (int64_t)B * ho * wo;
            T* dy = AT(enc.dy[l]);
            HLMC_TRY(bn_bwd(s, gA, co, AT(enc.y[l]), R, co, enc.bb[l], enc.g[l], enc.beta[l], 0, nullptr, 1.f, dy, enc.b[l],
                            nullptr, true, true));
            float* gw = G[enc.w[l]];
            if (l == 0) {
                // the last weight gradient of backward: on the main stream, which would otherwise only wait for
                // the weight-gradient stream here (that stream is still reducing layer 1's gradient)
                const PendingBias pb = pend_bias;
                pend_bias = PendingBias{};
                if (pb.gb) HLMC_TRY(ops::colsum_finalize(s, pb.acc, pb.C, pb.gb));
                HLMC_TRY(ops::wgrad_c1<T>(s, dy, B, ho, wo, co, audio, gw, scratch));
            } else if (l == 0) {
                HLMC_TRY(side_bias(s, [=](hipStream_t q, Ws sc) { return ops::wgrad_c1<T>(q, dy, B, ho, wo, co, audio, gw, sc); }));
            } else {
                const T* xin = AT(enc.a[l - 1]);
                const PendingBias pb = take_bias();  // written by the weight gradient's reduce launch
                HLMC_TRY(side_bias(s, [=](hipStream_t q, Ws sc) {
                    return ops::wgrad_s2<T>(q, dy, B, ho, wo, co, xin, ci, gw, sc, pb.acc, pb.gb);
                }));
                if (l == 1) HLMC_TRY(flush_side(s));  // nothing queued may wait for the join behind the main tail
                // grad of layer l-1's activation
                HLMC_TRY(ops::subpixel<T>(s, dy, B, ho, wo, co, P1(enc.w[l]), nullptr, ci, gA, scratch));
            }
            if (l == 3 && bucket_hi >= 0) HLMC_TRY(mark(s, bucket_hi));
            if (l == 2) HLMC_TRY(prelate(s));  // layers 0-1 (late_params) remain
        }
        return HLMC_OK;
    }

    // ---------------------------------------------------------------- conv decoder (5 x convT-BN-LReLU + convT)
    struct Dec {
        int w[6], b[6], g[5], beta[5], bn[5];
        int h0 = 0, w0 = 0;  // low-res input grid (H/64, W/64)
        size_t y[5], a[5], dy[5];
        BnBufs bb[5];
    };
    Dec dec;
    // first_index: module index of the first ConvTranspose2d (1 for HybridVAE's Unflatten-led Sequential, 0 for CVAE)
    void dec_register(const std::string& prefix, int first_index) {
        for (int l = 0; l < 6; ++l) {
            const int ci = DEC_CH[l], co = DEC_CH[l + 1];
            const int mi = first_index + 3 * l;
            dec.w[l] = add_param(prefix + "." + std::to_string(mi) + ".weight", {ci, co, 3, 3});
            dec.b[l] = add_param(prefix + "." + std::to_string(mi) + ".bias", {co});
            if (l < 5) {
                dec.g[l] = add_param(prefix + "." + std::to_string(mi + 1) + ".weight", {co});
                dec.beta[l] = add_param(prefix + "." + std::to_string(mi + 1) + ".bias", {co});
                dec.bn[l] = add_bn();
                register_pack(dec.w[l], 9);
            }
        }
    }
    void dec_plan(Arena& A, int64_t B) {
        int h = dec.h0, w = dec.w0;
        for (int l = 0; l < 6; ++l) {
            const int ci = DEC_CH[l], co = DEC_CH[l + 1];
            if (l < 5) {
                need(ops::subpixel_ws<T>((int)B, h, w, ci, co));
                need(ops::conv_s2_ws<T>((int)B, 2 * h, 2 * w, co, ci));
                need(ops::wgrad_s2_ws<T>((int)B, h, w, ci, co));
                const size_t n = (size_t)B * 4 * h * w * co;
                dec.y[l] = A.take(n * sizeof(T));
                dec.a[l] = A.take(n * sizeof(T));
                dec.dy[l] = A.take(n * sizeof(T));
                dec.bb[l] = bn_plan(A, co);
            } else {
                need(ops::wgrad_c1_ws((int)B, h, w, ci));
                need(ops::colsum_ws((int)(B * 4 * h * w), 1));
            }
            h *= 2;
            w *= 2;
        }
    }
    size_t dec_max_elems(int64_t B) const { return (size_t)B * dec.h0 * 32 * dec.w0 * 32 * 32; }
    // u: NHWC [B, h0, w0, 512]; recon f32 [B, 64 h0, 64 w0]
    int dec_fwd(hipStream_t s, bool train, const T* u, int B, float* recon) {
        int h = dec.h0, w = dec.w0;
        const T* x = u;
        bool fused_prev = false;  // layer l-1's BatchNorm + activation is applied inside layer l's sub-pixel conv
        ops::BnInput xin{};
        for (int l = 0; l < 6; ++l) {
            const int ci = DEC_CH[l], co = DEC_CH[l + 1];
            if (l < 5) {
                T* y = AT(dec.y[l]);
                const int64_t R = (int64_t)B * 4 * h * w;
                ops::ColStats st{train ? acc_fwd(dec.bb[l]) : XAcc{}, false};
                HLMC_TRY(ops::subpixel<T>(s, fused_prev ? AT(dec.y[l - 1]) : x, B, h, w, ci, P1(dec.w[l]), P[dec.b[l]], co,
                                          y, scratch, &st, fused_prev ? &xin : nullptr));
                fused_prev = train && l + 1 < 5 && ops::subpixel_takes_input_bn<T>(B, 2 * h, 2 * w, co, DEC_CH[l + 2]);
                if (fused_prev) {
                    if (!st.done) HLMC_TRY(ops::bn_moments<T>(s, y, R, co, acc_fwd(dec.bb[l])));  // split-K producer
                    xin = bn_input(dec.bb[l], dec.bn[l], dec.g[l], dec.beta[l], R, dec.a[l]);
                } else
                    HLMC_TRY(bn_fwd(s, train, y, R, co, dec.bn[l], dec.bb[l], dec.g[l], dec.beta[l], 0, nullptr, 1.f,
                                    AT(dec.a[l]), co, &st));
                x = AT(dec.a[l]);
            } else {
                HLMC_TRY(ops::convT_c1<T>(s, x, B, h, w, ci, P[dec.w[5]], P[dec.b[5]], recon));
            }
            h *= 2;
            w *= 2;
        }
        return HLMC_OK;
    }
    // gA: data-gradient chain buffer; returns the grad wrt u in *out (= gA)
    int dec_bwd(hipStream_t s, const T* u, int B, const float* d_recon, T* gA, T** out) {
        int hs[7], ws_[7];
        hs[0] = dec.h0;
        ws_[0] = dec.w0;
        for (int l = 0; l < 6; ++l) { hs[l + 1] = hs[l] * 2; ws_[l + 1] = ws_[l] * 2; }
        // last layer (1 output channel): input a4 [B, hs5, ws5, 32]
        {
            const int hl = hs[5], wl = ws_[5];
            const T* a4 = AT(dec.a[4]);
            float* gw = G[dec.w[5]];
            float* gb = G[dec.b[5]];
            const int npix = B * hs[6] * ws_[6];
            HLMC_TRY(side(s, [=](hipStream_t q, Ws sc) {
                HLMC_TRY(ops::wgrad_c1<T>(q, a4, B, hl, wl, DEC_CH[5], d_recon, gw, sc));
                return ops::colsum<float>(q, d_recon, 1, npix, 1, gb, sc);
            }));
            // layer 4's BN-backward moments come with the edge conv that writes its output gradient
            fuse4 = ops::BnBwdFuse{AT(dec.y[4]), AF(dec.bb[4].mean), AF(dec.bb[4].inv), P[dec.g[4]], P[dec.beta[4]],
                                   acc_mom(dec.bb[4]), false};
            HLMC_TRY(ops::conv_c1_s2<T>(s, d_recon, B, hs[6], ws_[6], P[dec.w[5]], nullptr, DEC_CH[5], gA, nullptr,
                                        &fuse4));
        }
        ops::BnBwdFuse fuse = fuse4;
        for (int l = 4; l >= 0; --l) {
            const int ci = DEC_CH[l], co = DEC_CH[l + 1];
            const int hl = hs[l], wl = ws_[l];
            const int64_t R = (int64_t)B * 4 * hl * wl;
            T* dy = AT(dec.dy[l]);
            HLMC_TRY(bn_bwd(s, gA, co, AT(dec.y[l]), R, co, dec.bb[l], dec.g[l], dec.beta[l], 0, nullptr, 1.f, dy, dec.b[l],
                            &fuse, true, true));
            const T* xin = l == 0 ? u : AT(dec.a[l - 1]);
            float* gw = G[dec.w[l]];
            const PendingBias pb = take_bias();  // written by the weight gradient's reduce launch
            HLMC_TRY(side_bias(s, [=](hipStream_t q, Ws sc) {
                return ops::wgrad_s2<T>(q, xin, B, hl, wl, ci, dy, co, gw, sc, pb.acc, pb.gb);
            }));
            HLMC_TRY(ops::conv_s2<T>(s, dy, B, 2 * hl, 2 * wl, co, P0(dec.w[l]), nullptr, ci, gA, scratch));
            fuse = ops::BnBwdFuse{};  // the stride-2 conv data gradients carry no moments: a separate pass
        }
        *out = gA;
        return HLMC_OK;
    }
};

// ============================================================================ HybridVAE
template <typename T>
class HybridNet : public NetT<T> {
    using Base = NetT<T>;
    using typename Base::BnBufs;
    using Base::AT;
    using Base::AF;
    using Base::AU8;
    using Base::P;
    using Base::G;

  public:
    int L = 128, TD = 768, H = 128, W = 128, F = 0;
    bool text = true;
    int afc_w, afc_b, te_w[2], te_b[2], te_g[2], te_beta[2], te_bn[2];
    int fus_w, fus_b, mu_w, mu_b, lv_w, lv_b, di_w, di_b, ds_w, ds_b, adf_w, adf_b;
    int td_w[2], td_b[2], td_g, td_beta, td_bn;
    int FU = 1024, SP = 1024;  // fusion / split widths
    // workspace
    size_t flat_, fuse_, tin_, te_y[2], te_a0, h_, mu_, lv_, eps_, z_, d1_, s_, ah_, u_, td_y, td_a, rt_;
    BnBufs te_bb[2], td_bb;
    size_t gA_, gflat_, gfuse_, gh_, gz_, gd1_, gs_, gah_, gte_, gte1_, gte2_, gtd_, gtd2_, gmuT_, glvT_, grt_;
    int ldF = 0, ldT = 0, ldFU = 0, ldSP = 0;

    HybridNet(int latent, int text_dim, int h, int w) : L(latent), TD(text_dim), H(h), W(w) {
        text = text_dim > 0;
        F = 512 * (H / 64) * (W / 64);
        FU = text ? 1152 : 1024;
        SP = FU;
        this->enc.H = H;
        this->enc.W = W;
        this->dec.h0 = H / 64;
        this->dec.w0 = W / 64;
        this->enc_register("audio_encoder");
        afc_w = this->add_param("audio_fc.weight", {1024, F});
        afc_b = this->add_param("audio_fc.bias", {1024});
        this->register_pack(afc_w, 1);
        if (text) {
            const int dims[3] = {TD, 256, 128};
            for (int i = 0; i < 2; ++i) {
                te_w[i] = this->add_param("text_encoder." + std::to_string(3 * i) + ".weight", {dims[i + 1], dims[i]});
                te_b[i] = this->add_param("text_encoder." + std::to_string(3 * i) + ".bias", {dims[i + 1]});
                te_g[i] = this->add_param("text_encoder." + std::to_string(3 * i + 1) + ".weight", {dims[i + 1]});
                te_beta[i] = this->add_param("text_encoder." + std::to_string(3 * i + 1) + ".bias", {dims[i + 1]});
                te_bn[i] = this->add_bn();
                this->register_pack(te_w[i], 1);
            }
        }
        fus_w = this->add_param("fc_fusion.weight", {512, FU});
        fus_b = this->add_param("fc_fusion.bias", {512});
        mu_w = this->add_param("fc_mu.weight", {L, 512});
        mu_b = this->add_param("fc_mu.bias", {L});
        lv_w = this->add_param("fc_logvar.weight", {L, 512});
        lv_b = this->add_param("fc_logvar.bias", {L});
        di_w = this->add_param("decoder_input.weight", {512, L});
        di_b = this->add_param("decoder_input.bias", {512});
        ds_w = this->add_param("decoder_split.weight", {SP, 512});
        ds_b = this->add_param("decoder_split.bias", {SP});
        adf_w = this->add_param("audio_decoder_fc.weight", {F, 1024});
        adf_b = this->add_param("audio_decoder_fc.bias", {F});
        for (int w : {fus_w, mu_w, lv_w, di_w, ds_w, adf_w}) this->register_pack(w, 1);
        this->dec_register("audio_decoder", 1);
        if (text) {
            td_w[0] = this->add_param("text_decoder.0.weight", {256, 128});
            td_b[0] = this->add_param("text_decoder.0.bias", {256});
            td_g = this->add_param("text_decoder.1.weight", {256});
            td_beta = this->add_param("text_decoder.1.bias", {256});
            td_bn = this->add_bn();
            td_w[1] = this->add_param("text_decoder.3.weight", {TD, 256});
            td_b[1] = this->add_param("text_decoder.3.bias", {TD});
            this->register_pack(td_w[0], 1);
            this->register_pack(td_w[1], 1);
        }
        this->finalize_state();
        // backward finishes: audio + text decoder | audio_fc .. audio_decoder_fc | encoder layers 3-5 | layers 0-2
        this->bucket_starts = {this->dec.w[0], afc_w, this->enc.w[3], 0};
        this->late_params = this->enc.w[2];  // encoder layers 0-1: the last weight gradients of backward
    }

    void plan(Arena& A, int64_t B) override {
        ldF = pad8(F);
        ldT = pad8(TD);
        ldFU = pad8(FU);
        ldSP = pad8(SP);
        this->enc_plan(A, B);
        this->dec_plan(A, B);
        const size_t t = sizeof(T);
        flat_ = A.take(B * ldF * t);
        fuse_ = A.take(B * ldFU * t);
        h_ = A.take(B * 512 * t);
        mu_ = A.take(B * L * 4);
        lv_ = A.take(B * L * 4);
        eps_ = A.take(B * L * 4);
        z_ = A.take(B * L * t);
        d1_ = A.take(B * 512 * t);
        s_ = A.take(B * ldSP * t);
        ah_ = A.take(B * ldF * t);
        u_ = A.take(B * ldF * t);
        if (text) {
            tin_ = A.take(B * ldT * t);
            te_y[0] = A.take(B * 256 * t);
            te_a0 = A.take(B * 256 * t);
            te_y[1] = A.take(B * 128 * t);
            te_bb[0] = this->bn_plan(A, 256);
            te_bb[1] = this->bn_plan(A, 128);
            td_y = A.take(B * 256 * t);
            td_a = A.take(B * 256 * t);
            td_bb = this->bn_plan(A, 256);
            rt_ = A.take(B * ldT * t);
            gte_ = A.take(B * 256 * t);
            gte1_ = A.take(B * 128 * t);
            gte2_ = A.take(B * 256 * t);
            gtd_ = A.take(B * 256 * t);
            gtd2_ = A.take(B * 256 * t);
            grt_ = A.take(B * ldT * t);
            for (int i = 0; i < 2; ++i) this->lin_need((int)B, te_w[i]);
            this->lin_need((int)B, td_w[0]);
            this->lin_need((int)B, td_w[1]);
        }
        const size_t gmax = std::max(this->enc_max_elems(B), this->dec_max_elems(B));
        gA_ = A.take(gmax * t);
        gflat_ = A.take(B * ldF * t);
        gfuse_ = A.take(B * ldFU * t);
        gh_ = A.take(B * 512 * t);
        gz_ = A.take(B * L * t);
        gd1_ = A.take(B * 512 * t);
        gs_ = A.take(B * ldSP * t);
        gah_ = A.take(B * ldF * t);
        gmuT_ = A.take(B * L * t);
        glvT_ = A.take(B * L * t);
        for (int w : {afc_w, fus_w, mu_w, lv_w, di_w, ds_w, adf_w}) this->lin_need((int)B, w);
    }

    int encode(hipStream_t s, const ForwardArgs& a, int B) {
        const bool tr = a.train != 0;
        HLMC_TRY(this->enc_fwd(s, tr, a.in0, B));
        const int hh = H / 64, ww = W / 64;
        HLMC_TRY(ops::nhwc_to_flat<T>(s, AT(this->enc.a[5]), B, hh, ww, 512, AT(flat_), ldF));
        HLMC_TRY(this->template lin_fwd<T>(s, AT(flat_), ldF, B, afc_w, afc_b, AT(fuse_), ldFU, 0));
        if (text) {
            HLMC_CHECK_ARG(a.in1, "text input required");
            HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in1, TD, AT(tin_), ldT, B, TD));
            HLMC_TRY(this->template lin_fwd<T>(s, AT(tin_), ldT, B, te_w[0], te_b[0], AT(te_y[0]), 256, 0));
            HLMC_TRY(this->bn_fwd(s, tr, AT(te_y[0]), B, 256, te_bn[0], te_bb[0], te_g[0], te_beta[0], 0, nullptr, 1.f,
                                  AT(te_a0), 256));
            HLMC_TRY(this->template lin_fwd<T>(s, AT(te_a0), 256, B, te_w[1], te_b[1], AT(te_y[1]), 128, 0));
            HLMC_TRY(this->bn_fwd(s, tr, AT(te_y[1]), B, 128, te_bn[1], te_bb[1], te_g[1], te_beta[1], 0, nullptr, 1.f,
                                  AT(fuse_) + 1024, ldFU));
        }
        HLMC_TRY(this->template lin_fwd<T>(s, AT(fuse_), ldFU, B, fus_w, fus_b, AT(h_), 512, 1));
        HLMC_TRY(this->template lin_fwd<float>(s, AT(h_), 512, B, mu_w, mu_b, AF(mu_), L, 0));
        HLMC_TRY(this->template lin_fwd<float>(s, AT(h_), 512, B, lv_w, lv_b, AF(lv_), L, 0));
        return HLMC_OK;
    }

    int forward(hipStream_t s, const ForwardArgs& a) override {
        const int B = (int)a.B;
        HLMC_CHECK_ARG(B >= 2 || !a.train, "BatchNorm in train mode needs batch >= 2");
        this->ws_bytes(B);
        this->set_ws(a.ws);
        HLMC_TRY(this->settle(s));
        HLMC_TRY(this->pack_all(s));
        if (a.train) HLMC_TRY(this->zero_acc_fwd(s));
        this->last_full_forward = !a.encode_only && !a.decode_only;
        if (a.decode_only) {  // decode(z), src/Convolutional_VAE.py:167-179
            HLMC_CHECK_ARG(a.in0 && a.recon, "z and recon required");
            HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in0, L, AT(z_), L, B, L));
        } else {
            HLMC_TRY(encode(s, a, B));
            if (a.encode_only) return this->latent_out(s, a, AF(mu_), AF(lv_), (int64_t)B * L);
            HLMC_CHECK_ARG(a.recon, "recon required");
            // z, the kept eps and the caller's mu / logvar outputs in one launch
            HLMC_TRY(this->reparam(s, a.eps, AF(mu_), AF(lv_), AF(eps_), B, L, AT(z_), L, a.mu, a.logvar));
        }
        HLMC_TRY(this->template lin_fwd<T>(s, AT(z_), L, B, di_w, di_b, AT(d1_), 512, 1));
        HLMC_TRY(this->template lin_fwd<T>(s, AT(d1_), 512, B, ds_w, ds_b, AT(s_), ldSP, 1));
        HLMC_TRY(this->template lin_fwd<T>(s, AT(s_), ldSP, B, adf_w, adf_b, AT(ah_), ldF, 1));
        HLMC_TRY(ops::flat_to_nhwc<T>(s, AT(ah_), ldF, B, H / 64, W / 64, 512, AT(u_)));
        HLMC_TRY(this->dec_fwd(s, a.train != 0, AT(u_), B, a.recon));
        if (text) {
            HLMC_CHECK_ARG(a.recon_text, "recon_text required");
            HLMC_TRY(this->template lin_fwd<T>(s, AT(s_) + 1024, ldSP, B, td_w[0], td_b[0], AT(td_y), 256, 0));
            HLMC_TRY(this->bn_fwd(s, a.train != 0, AT(td_y), B, 256, td_bn, td_bb, td_g, td_beta, 0, nullptr, 1.f,
                                  AT(td_a), 256));
            HLMC_TRY(this->template lin_fwd<float>(s, AT(td_a), 256, B, td_w[1], td_b[1], a.recon_text, TD, 0));
        }
        return HLMC_OK;
    }

    int backward(hipStream_t s, const BackwardArgs& a) override {
        const int B = (int)a.B;
        HLMC_CHECK_ARG(B == this->planned_B, "backward batch differs from the last forward");
        HLMC_CHECK_ARG(this->last_full_forward, "backward needs a full hlmc_net_forward (not encode / decode)");
        this->set_ws(a.ws);
        HLMC_TRY(this->side_init());
        HLMC_TRY(this->settle(s));
        HLMC_TRY(this->zero_acc_bwd(s));
        T* gA = AT(gA_);
        // ---- text decoder
        if (text) {
            HLMC_CHECK_ARG(a.d_recon_text, "d_recon_text required");
            HLMC_TRY(ops::cast2d_from_f32<T>(s, a.d_recon_text, TD, AT(grt_), ldT, B, TD));
            HLMC_TRY(this->lin_bwd(s, AT(grt_), ldT, AT(td_a), 256, B, td_w[1], td_b[1], AT(gtd_), 256));
            HLMC_TRY(this->bn_bwd(s, AT(gtd_), 256, AT(td_y), B, 256, td_bb, td_g, td_beta, 0, nullptr, 1.f,
                                  AT(gtd2_), td_b[0]));
            HLMC_TRY(this->lin_bwd(s, AT(gtd2_), 256, AT(s_) + 1024, ldSP, B, td_w[0], -1, AT(gs_) + 1024, ldSP, 0,
                                   AT(s_) + 1024));
        }
        // ---- audio decoder
        T* gu = nullptr;
        HLMC_TRY(this->dec_bwd(s, AT(u_), B, a.d_recon, gA, &gu));
        HLMC_TRY(this->mark(s, 0));
        // (each ReLU backward rides in the epilogue of the GEMM / relayout that writes the gradient)
        HLMC_TRY(ops::nhwc_to_flat<T>(s, gu, B, H / 64, W / 64, 512, AT(gah_), ldF, AT(ah_)));
        HLMC_TRY(this->lin_bwd(s, AT(gah_), ldF, AT(s_), ldSP, B, adf_w, adf_b, AT(gs_), ldSP, 0, AT(s_)));
        HLMC_TRY(this->lin_bwd(s, AT(gs_), ldSP, AT(d1_), 512, B, ds_w, ds_b, AT(gd1_), 512, 0, AT(d1_)));
        HLMC_TRY(this->lin_bwd(s, AT(gd1_), 512, AT(z_), L, B, di_w, di_b, AT(gz_), L));
        // ---- reparameterisation + heads: one pass to the heads' T gradients (the caller's d_mu / d_logvar added)
        HLMC_TRY(ops::reparam_bwd<T>(s, AT(gz_), L, AF(lv_), AF(eps_), a.d_mu, a.d_logvar, B, L, AT(gmuT_), AT(glvT_)));
        HLMC_TRY(this->lin_bwd(s, AT(gmuT_), L, AT(h_), 512, B, mu_w, mu_b, AT(gh_), 512, 0));
        HLMC_TRY(this->lin_bwd(s, AT(glvT_), L, AT(h_), 512, B, lv_w, lv_b, AT(gh_), 512, 1, AT(h_)));
        HLMC_TRY(this->lin_bwd(s, AT(gh_), 512, AT(fuse_), ldFU, B, fus_w, fus_b, AT(gfuse_), ldFU));
        // ---- text encoder
        if (text) {
            HLMC_TRY(this->bn_bwd(s, AT(gfuse_) + 1024, ldFU, AT(te_y[1]), B, 128, te_bb[1], te_g[1], te_beta[1], 0,
                                  nullptr, 1.f, AT(gte1_), te_b[1]));
            HLMC_TRY(this->lin_bwd(s, AT(gte1_), 128, AT(te_a0), 256, B, te_w[1], -1, AT(gte_), 256));
            HLMC_TRY(this->bn_bwd(s, AT(gte_), 256, AT(te_y[0]), B, 256, te_bb[0], te_g[0], te_beta[0], 0, nullptr, 1.f,
                                  AT(gte2_), te_b[0]));
            HLMC_TRY(this->lin_bwd(s, AT(gte2_), 256, AT(tin_), ldT, B, te_w[0], -1, nullptr, 0));
        }
        // ---- audio encoder
        HLMC_TRY(this->lin_bwd(s, AT(gfuse_), ldFU, AT(flat_), ldF, B, afc_w, afc_b, AT(gflat_), ldF));
        HLMC_TRY(this->mark(s, 1));
        HLMC_TRY(ops::flat_to_nhwc<T>(s, AT(gflat_), ldF, B, H / 64, W / 64, 512, gA));
        HLMC_TRY(this->enc_bwd(s, B, gA, 2));
        HLMC_TRY(this->finish_backward(s));
        return this->mark(s, 3);
    }
};

// ============================================================================ ConditionalVAE
template <typename T>
class CvaeNet : public NetT<T> {
    using Base = NetT<T>;
    using typename Base::BnBufs;
    using Base::AT;
    using Base::AF;
    using Base::AU8;
    using Base::P;
    using Base::G;

  public:
    int L = 64, TD = 768, C = 10, H = 128, W = 128, F = 0;
    int te_w, te_b, te_g, te_beta, te_bn, mu_w, mu_b, lv_w, lv_b, dfc_w, dfc_b;
    int td_w[2], td_b[2], td_g, td_beta, td_bn;
    int ldF = 0, ldT = 0, ldX = 0, ldZ = 0, ldS = 0;
    size_t tin_, te_y, X_, mu_, lv_, eps_, Z_, S_, u_, td_y, td_a;
    BnBufs te_bb, td_bb;
    size_t gA_, grt_, gtd_, gt2_, gt3_, gS_, gZ_, gX_, gmuT_, glvT_;

    CvaeNet(int latent, int text_dim, int ncls, int h, int w) : L(latent), TD(text_dim), C(ncls), H(h), W(w) {
        F = 512 * (H / 64) * (W / 64);
        this->enc.H = H;
        this->enc.W = W;
        this->dec.h0 = H / 64;
        this->dec.w0 = W / 64;
        this->enc_register("audio_encoder");
        te_w = this->add_param("text_encoder.0.weight", {256, TD});
        te_b = this->add_param("text_encoder.0.bias", {256});
        te_g = this->add_param("text_encoder.1.weight", {256});
        te_beta = this->add_param("text_encoder.1.bias", {256});
        te_bn = this->add_bn();
        const int fusion = F + 256 + C;
        mu_w = this->add_param("fc_mu.weight", {L, fusion});
        mu_b = this->add_param("fc_mu.bias", {L});
        lv_w = this->add_param("fc_logvar.weight", {L, fusion});
        lv_b = this->add_param("fc_logvar.bias", {L});
        dfc_w = this->add_param("decoder_fc.weight", {F + 256, L + C});
        dfc_b = this->add_param("decoder_fc.bias", {F + 256});
        td_w[0] = this->add_param("text_decoder.0.weight", {512, 256});
        td_b[0] = this->add_param("text_decoder.0.bias", {512});
        td_g = this->add_param("text_decoder.1.weight", {512});
        td_beta = this->add_param("text_decoder.1.bias", {512});
        td_bn = this->add_bn();
        td_w[1] = this->add_param("text_decoder.3.weight", {TD, 512});
        td_b[1] = this->add_param("text_decoder.3.bias", {TD});
        for (int w_ : {te_w, mu_w, lv_w, dfc_w, td_w[0], td_w[1]}) this->register_pack(w_, 1);
        this->dec_register("audio_decoder", 0);
        this->finalize_state();
        // backward finishes: text + audio decoder | text_encoder .. decoder_fc | encoder layers 3-5 | layers 0-2
        this->bucket_starts = {td_w[0], te_w, this->enc.w[3], 0};
        this->late_params = this->enc.w[2];
    }

    void plan(Arena& A, int64_t B) override {
        const size_t t = sizeof(T);
        ldF = pad8(F);
        ldT = pad8(TD);
        ldX = pad8(F + 256 + C);
        ldZ = pad8(L + C);
        ldS = pad8(F + 256);
        this->enc_plan(A, B);
        this->dec_plan(A, B);
        tin_ = A.take(B * ldT * t);
        te_y = A.take(B * 256 * t);
        te_bb = this->bn_plan(A, 256);
        X_ = A.take(B * ldX * t);
        mu_ = A.take(B * L * 4);
        lv_ = A.take(B * L * 4);
        eps_ = A.take(B * L * 4);
        Z_ = A.take(B * ldZ * t);
        S_ = A.take(B * ldS * t);
        u_ = A.take(B * ldF * t);
        td_y = A.take(B * 512 * t);
        td_a = A.take(B * 512 * t);
        td_bb = this->bn_plan(A, 512);
        const size_t gmax = std::max(this->enc_max_elems(B), this->dec_max_elems(B));
        gA_ = A.take(gmax * t);
        grt_ = A.take(B * ldT * t);
        gtd_ = A.take(B * 512 * t);
        gt2_ = A.take(B * 512 * t);
        gt3_ = A.take(B * 256 * t);
        gS_ = A.take(B * ldS * t);
        gZ_ = A.take(B * ldZ * t);
        gX_ = A.take(B * ldX * t);
        gmuT_ = A.take(B * L * t);
        glvT_ = A.take(B * L * t);
        for (int w_ : {te_w, mu_w, lv_w, dfc_w, td_w[0], td_w[1]}) this->lin_need((int)B, w_);
    }

    int encode(hipStream_t s, const ForwardArgs& a, int B) {
        const bool tr = a.train != 0;
        HLMC_CHECK_ARG(a.in1 && a.in2, "text and condition inputs required");
        HLMC_TRY(this->enc_fwd(s, tr, a.in0, B));
        HLMC_TRY(ops::nhwc_to_flat<T>(s, AT(this->enc.a[5]), B, H / 64, W / 64, 512, AT(X_), ldX));
        HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in1, TD, AT(tin_), ldT, B, TD));
        HLMC_TRY(this->template lin_fwd<T>(s, AT(tin_), ldT, B, te_w, te_b, AT(te_y), 256, 0));
        HLMC_TRY(this->bn_fwd(s, tr, AT(te_y), B, 256, te_bn, te_bb, te_g, te_beta, 0, nullptr, 1.f, AT(X_) + F, ldX));
        HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in2, C, AT(X_) + F + 256, ldX, B, C));
        HLMC_TRY(this->template lin_fwd<float>(s, AT(X_), ldX, B, mu_w, mu_b, AF(mu_), L, 0));
        HLMC_TRY(this->template lin_fwd<float>(s, AT(X_), ldX, B, lv_w, lv_b, AF(lv_), L, 0));
        return HLMC_OK;
    }

    int forward(hipStream_t s, const ForwardArgs& a) override {
        const int B = (int)a.B;
        HLMC_CHECK_ARG(B >= 2 || !a.train, "BatchNorm in train mode needs batch >= 2");
        this->ws_bytes(B);
        this->set_ws(a.ws);
        HLMC_TRY(this->settle(s));
        HLMC_TRY(this->pack_all(s));
        if (a.train) HLMC_TRY(this->zero_acc_fwd(s));
        this->last_full_forward = !a.encode_only && !a.decode_only;
        if (a.decode_only) {  // decode(z, condition), src/Conditional_VAE.py:206-225
            HLMC_CHECK_ARG(a.in0 && a.in2 && a.recon && a.recon_text, "z / condition / recon / recon_text required");
            HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in0, L, AT(Z_), ldZ, B, L));
        } else {
            HLMC_TRY(encode(s, a, B));
            if (a.encode_only) return this->latent_out(s, a, AF(mu_), AF(lv_), (int64_t)B * L);
            HLMC_CHECK_ARG(a.recon && a.recon_text, "recon / recon_text required");
            // z, the kept eps and the caller's mu / logvar outputs in one launch
            HLMC_TRY(this->reparam(s, a.eps, AF(mu_), AF(lv_), AF(eps_), B, L, AT(Z_), ldZ, a.mu, a.logvar));
        }
        HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in2, C, AT(Z_) + L, ldZ, B, C));
        HLMC_TRY(this->template lin_fwd<T>(s, AT(Z_), ldZ, B, dfc_w, dfc_b, AT(S_), ldS, 0));
        HLMC_TRY(ops::flat_to_nhwc<T>(s, AT(S_), ldS, B, H / 64, W / 64, 512, AT(u_)));
        HLMC_TRY(this->dec_fwd(s, a.train != 0, AT(u_), B, a.recon));
        HLMC_TRY(this->template lin_fwd<T>(s, AT(S_) + F, ldS, B, td_w[0], td_b[0], AT(td_y), 512, 0));
        HLMC_TRY(this->bn_fwd(s, a.train != 0, AT(td_y), B, 512, td_bn, td_bb, td_g, td_beta, 0, nullptr, 1.f, AT(td_a), 512));
        HLMC_TRY(this->template lin_fwd<float>(s, AT(td_a), 512, B, td_w[1], td_b[1], a.recon_text, TD, 0));
        return HLMC_OK;
    }

    int backward(hipStream_t s, const BackwardArgs& a) override {
        const int B = (int)a.B;
        HLMC_CHECK_ARG(B == this->planned_B, "backward batch differs from the last forward");
        HLMC_CHECK_ARG(this->last_full_forward, "backward needs a full hlmc_net_forward (not encode / decode)");
        HLMC_CHECK_ARG(a.d_recon_text, "d_recon_text required");
        this->set_ws(a.ws);
        HLMC_TRY(this->side_init());
        HLMC_TRY(this->settle(s));
        HLMC_TRY(this->zero_acc_bwd(s));
        T* gA = AT(gA_);
        // text decoder
        HLMC_TRY(ops::cast2d_from_f32<T>(s, a.d_recon_text, TD, AT(grt_), ldT, B, TD));
        HLMC_TRY(this->lin_bwd(s, AT(grt_), ldT, AT(td_a), 512, B, td_w[1], td_b[1], AT(gtd_), 512));
        HLMC_TRY(this->bn_bwd(s, AT(gtd_), 512, AT(td_y), B, 512, td_bb, td_g, td_beta, 0, nullptr, 1.f, AT(gt2_), td_b[0]));
        HLMC_TRY(this->lin_bwd(s, AT(gt2_), 512, AT(S_) + F, ldS, B, td_w[0], -1, AT(gS_) + F, ldS));
        // audio decoder
        T* gu = nullptr;
        HLMC_TRY(this->dec_bwd(s, AT(u_), B, a.d_recon, gA, &gu));
        HLMC_TRY(this->mark(s, 0));
        HLMC_TRY(ops::nhwc_to_flat<T>(s, gu, B, H / 64, W / 64, 512, AT(gS_), ldS));
        // decoder_fc (no activation)
        HLMC_TRY(this->lin_bwd(s, AT(gS_), ldS, AT(Z_), ldZ, B, dfc_w, dfc_b, AT(gZ_), ldZ));
        // reparameterisation
        HLMC_TRY(ops::reparam_bwd<T>(s, AT(gZ_), ldZ, AF(lv_), AF(eps_), a.d_mu, a.d_logvar, B, L, AT(gmuT_), AT(glvT_)));
        HLMC_TRY(this->lin_bwd(s, AT(gmuT_), L, AT(X_), ldX, B, mu_w, mu_b, AT(gX_), ldX, 0));
        HLMC_TRY(this->lin_bwd(s, AT(glvT_), L, AT(X_), ldX, B, lv_w, lv_b, AT(gX_), ldX, 1));
        // text encoder
        HLMC_TRY(this->bn_bwd(s, AT(gX_) + F, ldX, AT(te_y), B, 256, te_bb, te_g, te_beta, 0, nullptr, 1.f, AT(gt3_), te_b));
        HLMC_TRY(this->lin_bwd(s, AT(gt3_), 256, AT(tin_), ldT, B, te_w, -1, nullptr, 0));
        HLMC_TRY(this->mark(s, 1));
        // audio encoder
        HLMC_TRY(ops::flat_to_nhwc<T>(s, AT(gX_), ldX, B, H / 64, W / 64, 512, gA));
        HLMC_TRY(this->enc_bwd(s, B, gA, 2));
        HLMC_TRY(this->finish_backward(s));
        return this->mark(s, 3);
    }
};

// ============================================================================ Simple VAE (MLP)
template <typename T>
class SimpleNet : public NetT<T> {
    using Base = NetT<T>;
    using typename Base::BnBufs;
    using Base::AT;
    using Base::AF;
    using Base::AU8;
    using Base::P;
    using Base::G;

  public:
    int D = 370, L = 32;
    std::vector<int> hid;
    struct Blk {
        int w, b, g, beta, bn, din, dout;
        size_t y, a, dy;
        BnBufs bb;
        int64_t mask_off;
    };
    std::vector<Blk> encb, decb;
    int mu_w, mu_b, lv_w, lv_b, out_w, out_b;
    int ldD = 0;
    size_t x_, mu_, lv_, eps_, z_, gx1_, gmuT_, glvT_, gz_, grec_, mask_;
    int64_t mask_total = 0;

    SimpleNet(int input_dim, int latent, std::vector<int> hidden) : D(input_dim), L(latent), hid(std::move(hidden)) {
        int prev = D, mi = 0;
        for (int h : hid) {
            Blk b{};
            b.din = prev;
            b.dout = h;
            b.w = this->add_param("encoder." + std::to_string(mi) + ".weight", {h, prev});
            b.b = this->add_param("encoder." + std::to_string(mi) + ".bias", {h});
            b.g = this->add_param("encoder." + std::to_string(mi + 1) + ".weight", {h});
            b.beta = this->add_param("encoder." + std::to_string(mi + 1) + ".bias", {h});
            b.bn = this->add_bn();
            this->register_pack(b.w, 1);
            encb.push_back(b);
            prev = h;
            mi += 4;
        }
        mu_w = this->add_param("fc_mu.weight", {L, prev});
        mu_b = this->add_param("fc_mu.bias", {L});
        lv_w = this->add_param("fc_logvar.weight", {L, prev});
        lv_b = this->add_param("fc_logvar.bias", {L});
        this->register_pack(mu_w, 1);
        this->register_pack(lv_w, 1);
        prev = L;
        mi = 0;
        for (int i = (int)hid.size() - 1; i >= 0; --i) {
            const int h = hid[i];
            Blk b{};
            b.din = prev;
            b.dout = h;
            b.w = this->add_param("decoder." + std::to_string(mi) + ".weight", {h, prev});
            b.b = this->add_param("decoder." + std::to_string(mi) + ".bias", {h});
            b.g = this->add_param("decoder." + std::to_string(mi + 1) + ".weight", {h});
            b.beta = this->add_param("decoder." + std::to_string(mi + 1) + ".bias", {h});
            b.bn = this->add_bn();
            this->register_pack(b.w, 1);
            decb.push_back(b);
            prev = h;
            mi += 4;
        }
        out_w = this->add_param("decoder." + std::to_string(mi) + ".weight", {D, prev});
        out_b = this->add_param("decoder." + std::to_string(mi) + ".bias", {D});
        this->register_pack(out_w, 1);
        this->finalize_state();
    }

    void plan(Arena& A, int64_t B) override {
        const size_t t = sizeof(T);
        ldD = pad8(D);
        x_ = A.take(B * ldD * t);
        int64_t moff = 0;
        int widest = ldD;
        for (auto* v : {&encb, &decb})
            for (auto& b : *v) {
                b.y = A.take(B * b.dout * t);
                b.a = A.take(B * b.dout * t);
                b.dy = A.take(B * b.dout * t);
                b.bb = this->bn_plan(A, b.dout);
                b.mask_off = moff;
                moff += B * b.dout;
                widest = std::max(widest, pad8(b.dout));
                this->lin_need((int)B, b.w);
            }
        mask_total = moff;
        mask_ = A.take((size_t)moff);
        mu_ = A.take(B * L * 4);
        lv_ = A.take(B * L * 4);
        eps_ = A.take(B * L * 4);
        z_ = A.take(B * pad8(L) * t);
        gx1_ = A.take(B * widest * t);
        gmuT_ = A.take(B * L * t);
        glvT_ = A.take(B * L * t);
        gz_ = A.take(B * pad8(L) * t);
        grec_ = A.take(B * ldD * t);
        for (int w_ : {mu_w, lv_w, out_w}) this->lin_need((int)B, w_);
    }

    const uint8_t* mask_of(const Blk& b) const { return dropout ? dropout + b.mask_off : nullptr; }
    const uint8_t* dropout = nullptr;
    static constexpr float kKeepScale = 1.f / 0.8f;  // Dropout(0.2)

    int encode(hipStream_t s, const ForwardArgs& a, int B) {
        const bool tr = a.train != 0;
        dropout = nullptr;
        if (tr && a.dropout) {
            HLMC_HIP(hipMemcpyAsync(AU8(mask_), a.dropout, (size_t)mask_total, hipMemcpyDeviceToDevice, s));
            dropout = AU8(mask_);
        }
        HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in0, D, AT(x_), ldD, B, D));
        const T* x = AT(x_);
        int ldx = ldD;
        for (auto& b : encb) {
            HLMC_TRY(this->template lin_fwd<T>(s, x, ldx, B, b.w, b.b, AT(b.y), b.dout, 0));
            HLMC_TRY(this->bn_fwd(s, tr, AT(b.y), B, b.dout, b.bn, b.bb, b.g, b.beta, 1, mask_of(b), kKeepScale,
                                  AT(b.a), b.dout));
            x = AT(b.a);
            ldx = b.dout;
        }
        HLMC_TRY(this->template lin_fwd<float>(s, x, ldx, B, mu_w, mu_b, AF(mu_), L, 0));
        HLMC_TRY(this->template lin_fwd<float>(s, x, ldx, B, lv_w, lv_b, AF(lv_), L, 0));
        return HLMC_OK;
    }

    int forward(hipStream_t s, const ForwardArgs& a) override {
        const int B = (int)a.B;
        HLMC_CHECK_ARG(B >= 2 || !a.train, "BatchNorm in train mode needs batch >= 2");
        this->ws_bytes(B);
        this->set_ws(a.ws);
        HLMC_TRY(this->settle(s));
        HLMC_TRY(this->pack_all(s));
        if (a.train) HLMC_TRY(this->zero_acc_fwd(s));
        this->last_full_forward = !a.encode_only && !a.decode_only;
        if (a.decode_only) {  // decode(z), src/Simple_VAE.py:95-96 (decoder blocks' dropout from the same mask layout)
            HLMC_CHECK_ARG(a.in0 && a.recon, "z and recon required");
            dropout = nullptr;
            if (a.train && a.dropout) {
                HLMC_HIP(hipMemcpyAsync(AU8(mask_), a.dropout, (size_t)mask_total, hipMemcpyDeviceToDevice, s));
                dropout = AU8(mask_);
            }
            HLMC_TRY(ops::cast2d_from_f32<T>(s, a.in0, L, AT(z_), pad8(L), B, L));
        } else {
            HLMC_TRY(encode(s, a, B));
            if (a.encode_only) return this->latent_out(s, a, AF(mu_), AF(lv_), (int64_t)B * L);
            HLMC_CHECK_ARG(a.recon, "recon required");
            // z, the kept eps and the caller's mu / logvar outputs in one launch
            HLMC_TRY(this->reparam(s, a.eps, AF(mu_), AF(lv_), AF(eps_), B, L, AT(z_), pad8(L), a.mu, a.logvar));
            if (a.z) HLMC_TRY(ops::reparam_fwd<float>(s, AF(mu_), AF(lv_), AF(eps_), B, L, a.z, L));
        }
        const T* x = AT(z_);
        int ldx = pad8(L);
        for (auto& b : decb) {
            HLMC_TRY(this->template lin_fwd<T>(s, x, ldx, B, b.w, b.b, AT(b.y), b.dout, 0));
            HLMC_TRY(this->bn_fwd(s, a.train != 0, AT(b.y), B, b.dout, b.bn, b.bb, b.g, b.beta, 1, mask_of(b), kKeepScale,
                                  AT(b.a), b.dout));
            x = AT(b.a);
            ldx = b.dout;
        }
        HLMC_TRY(this->template lin_fwd<float>(s, x, ldx, B, out_w, out_b, a.recon, D, 0));
        return HLMC_OK;
    }

    int backward(hipStream_t s, const BackwardArgs& a) override {
        const int B = (int)a.B;
        HLMC_CHECK_ARG(B == this->planned_B, "backward batch differs from the last forward");
        HLMC_CHECK_ARG(this->last_full_forward, "backward needs a full hlmc_net_forward (not encode / decode)");
        this->set_ws(a.ws);
        HLMC_TRY(this->side_init());
        HLMC_TRY(this->settle(s));
        HLMC_TRY(this->zero_acc_bwd(s));
        T* g1 = AT(gx1_);
        HLMC_TRY(ops::cast2d_from_f32<T>(s, a.d_recon, D, AT(grec_), ldD, B, D));
        const Blk& last = decb.back();
        HLMC_TRY(this->lin_bwd(s, AT(grec_), ldD, AT(last.a), last.dout, B, out_w, out_b, g1, last.dout));
        for (int i = (int)decb.size() - 1; i >= 0; --i) {
            const Blk& b = decb[i];
            T* dy = AT(b.dy);
            HLMC_TRY(this->bn_bwd(s, g1, b.dout, AT(b.y), B, b.dout, b.bb, b.g, b.beta, 1, mask_of(b), kKeepScale, dy, b.b));
            const T* xin = i == 0 ? AT(z_) : AT(decb[i - 1].a);
            const int ldx = i == 0 ? pad8(L) : decb[i - 1].dout;
            T* gin = i == 0 ? AT(gz_) : g1;
            const int ldg = i == 0 ? pad8(L) : b.din;
            HLMC_TRY(this->lin_bwd(s, dy, b.dout, xin, ldx, B, b.w, -1, gin, ldg));
        }
        HLMC_TRY(ops::reparam_bwd<T>(s, AT(gz_), pad8(L), AF(lv_), AF(eps_), a.d_mu, a.d_logvar, B, L, AT(gmuT_),
                                     AT(glvT_)));
        const Blk& top = encb.back();
        HLMC_TRY(this->lin_bwd(s, AT(gmuT_), L, AT(top.a), top.dout, B, mu_w, mu_b, g1, top.dout, 0));
        HLMC_TRY(this->lin_bwd(s, AT(glvT_), L, AT(top.a), top.dout, B, lv_w, lv_b, g1, top.dout, 1));
        for (int i = (int)encb.size() - 1; i >= 0; --i) {
            const Blk& b = encb[i];
            T* dy = AT(b.dy);
            HLMC_TRY(this->bn_bwd(s, g1, b.dout, AT(b.y), B, b.dout, b.bb, b.g, b.beta, 1, mask_of(b), kKeepScale, dy, b.b));
            const T* xin = i == 0 ? AT(x_) : AT(encb[i - 1].a);
            const int ldx = i == 0 ? ldD : encb[i - 1].dout;
            HLMC_TRY(this->lin_bwd(s, dy, b.dout, xin, ldx, B, b.w, -1, i == 0 ? nullptr : g1, b.din));
        }
        HLMC_TRY(this->join(s));
        return this->mark(s, 0);
    }
};

template <template <typename> class NetTpl, typename... A>
std::unique_ptr<NetBase> make_typed(int dtype, A... args) {
    if (dtype == HLMC_BF16) return std::unique_ptr<NetBase>(new NetTpl<bf16>(args...));
    return std::unique_ptr<NetBase>(new NetTpl<float>(args...));
}

}  // namespace

int make_net(int kind, const int64_t* cfg, int ncfg, int dtype, std::unique_ptr<NetBase>* out) {
    HLMC_CHECK_ARG(dtype == HLMC_F32 || dtype == HLMC_BF16, "dtype must be HLMC_F32 or HLMC_BF16");
    HLMC_CHECK_ARG(cfg != nullptr, "cfg is NULL");
    std::unique_ptr<NetBase> n;
    if (kind == HLMC_NET_HYBRID) {
        HLMC_CHECK_ARG(ncfg == 4, "hybrid cfg = {latent, text_dim, H, W}");
        HLMC_CHECK_ARG(cfg[2] % 64 == 0 && cfg[3] % 64 == 0 && cfg[2] >= 64 && cfg[3] >= 64, "H, W must be multiples of 64");
        HLMC_CHECK_ARG(cfg[0] > 0 && cfg[1] >= 0, "latent > 0, text_dim >= 0");
        n = make_typed<HybridNet>(dtype, (int)cfg[0], (int)cfg[1], (int)cfg[2], (int)cfg[3]);
    } else if (kind == HLMC_NET_CVAE) {
        HLMC_CHECK_ARG(ncfg == 5, "cvae cfg = {latent, text_dim, num_classes, H, W}");
        HLMC_CHECK_ARG(cfg[3] % 64 == 0 && cfg[4] % 64 == 0 && cfg[3] >= 64 && cfg[4] >= 64, "H, W must be multiples of 64");
        HLMC_CHECK_ARG(cfg[0] > 0 && cfg[1] > 0 && cfg[2] > 0, "latent, text_dim, num_classes > 0");
        n = make_typed<CvaeNet>(dtype, (int)cfg[0], (int)cfg[1], (int)cfg[2], (int)cfg[3], (int)cfg[4]);
    } else if (kind == HLMC_NET_SIMPLE) {
        HLMC_CHECK_ARG(ncfg >= 3 && cfg[2] >= 1 && ncfg == 3 + cfg[2], "simple cfg = {input_dim, latent, n, h_1..h_n}");
        std::vector<int> hid;
        for (int i = 0; i < cfg[2]; ++i) {
            const int v = dtype == HLMC_BF16 ? 8 : 4;
            HLMC_CHECK_ARG(cfg[3 + i] % v == 0, "hidden widths must be multiples of the vector width (8 bf16 / 4 f32)");
            hid.push_back((int)cfg[3 + i]);
        }
        n = make_typed<SimpleNet>(dtype, (int)cfg[0], (int)cfg[1], hid);
    } else {
        HLMC_CHECK_ARG(false, "unknown net kind");
    }
    n->kind = kind;
    n->dtype = dtype;
    *out = std::move(n);
    return HLMC_OK;
}

}  // namespace hlmc
