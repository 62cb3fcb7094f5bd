// Native VAE engine: the three reference model families as fixed kernel schedules.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "ops.hpp"

namespace hlmc {

struct ParamInfo {
    std::string name;
    std::vector<int64_t> shape;
    int64_t numel() const {
        int64_t n = 1;
        for (auto d : shape) n *= d;
        return n;
    }
};

// Bump allocator over a caller-provided device buffer (offsets only; 256-byte aligned).
struct Arena {
    size_t used = 0;
    size_t take(size_t bytes) {
        size_t o = used;
        used += (bytes + 255) & ~size_t(255);
        return o;
    }
};

struct ForwardArgs {
    int64_t B;
    int train;
    const float* in0;
    const float* in1;
    const float* in2;
    const float* eps;
    const uint8_t* dropout;
    float* recon;
    float* recon_text;
    float* mu;
    float* logvar;
    float* z;
    void* ws;
    bool encode_only;
    bool decode_only = false;  // in0 = z [B][latent] (cvae: in2 = condition); eps, mu, logvar unused
};

struct BackwardArgs {
    int64_t B;
    const float* d_recon;
    const float* d_recon_text;
    const float* d_mu;
    const float* d_logvar;
    void* ws;
};

class NetBase {
  public:
    virtual ~NetBase() = default;
    int kind = 0, dtype = 0;
    std::vector<ParamInfo> params;
    int n_bn = 0;

    // bound storage
    std::vector<float*> P, G, RM, RV;
    std::vector<int64_t*> NBT;
    char* state = nullptr;

    int add_param(const std::string& name, std::vector<int64_t> shape) {
        params.push_back({name, std::move(shape)});
        return (int)params.size() - 1;
    }
    int add_bn() { return n_bn++; }

    virtual size_t state_bytes() const = 0;
    virtual size_t ws_bytes(int64_t B) = 0;
    virtual int bind_state(hipStream_t s) = 0;  // upload pack jobs into state
    virtual int forward(hipStream_t s, const ForwardArgs& a) = 0;
    virtual int backward(hipStream_t s, const BackwardArgs& a) = 0;
    // Adam over all bound parameters with the packed GEMM weights refreshed in the same pass
    // coef_dev (nullable): device coefficients (ops::adam_coef_host layout) instead of a's step-dependent ones
    virtual int adam_step(hipStream_t s, float* const* m, float* const* v, const ops::AdamArgs& a,
                          const float* coef_dev = nullptr) = 0;
    bool trust_packs = false;  // forward skips re-packing when packs are known current
    bool packs_valid = false;

    // Gradient buckets of the data-parallel all-reduce, in the order backward() finishes them:
    // bucket k = params[bucket_starts[k] .. bucket_starts[k-1]) (bucket_starts[-1] = params.size();
    // strictly decreasing, last = 0).  With bucket_sync set, backward() records bucket_ev[k] once every
    // gradient of bucket k is written (on any stream), so an all-reduce can start before backward ends.
    std::vector<int> bucket_starts{0};
    std::vector<hipEvent_t> bucket_ev;
    bool bucket_sync = false;

    // Tail overlap (single process): the gradients of params [0, late_params) are the last the weight-gradient
    // stream writes.  With overlap_adam set (and no bucket sync), backward() leaves that stream running and
    // adam_step() updates every other parameter first, joins, then updates the late ones — the first part of
    // Adam runs under the tail of the backward pass.
    int late_params = 0;
    bool overlap_adam = false;
    bool last_full_forward = false;  // the workspace holds a full forward (backward's precondition)
    // reparameterisation noise drawn on the device when the caller passes no eps (ops::reparam_rng): Philox
    // stream `rng_seed`, next element rng_offset (advanced by each such forward, kept a multiple of 4)
    uint64_t rng_seed = 0, rng_offset = 0;
    virtual int settle(hipStream_t s) = 0;  // make every gradient of the last backward final on s
};

// factory: kind 0 hybrid, 1 cvae, 2 simple; cfg per hlmc.h
int make_net(int kind, const int64_t* cfg, int ncfg, int dtype, std::unique_ptr<NetBase>* out);

}  // namespace hlmc
