// MFMA GEMM main loops for the VAE hot path (gfx950).
//
//   gemm_nt : C[m][n] = sum_k A(m,k) * B(n,k)   A gathered by a loader policy (conv stride-2 window,
//             transposed-conv sub-pixel phase, dense row-major), B = packed weight [N][K] (K contiguous).
//   gemm_tn : C[m][n] = sum_k L(k,m) * H(k,n)   both operands k-major (weight gradients); fragments are
//             read with ds_read_b64_tr_b16 (bf16) so no transposed staging is needed.
//
// T = bf16 -> v_mfma_f32_16x16x32_bf16 (f32 accumulate), BK = 32
// T = float -> v_mfma_f32_16x16x4_f32 (exact f32 fma chain), BK = 16
// Every k-row of a tile is 64 bytes (4 x 16-byte chunks); LDS rows are padded to 80 bytes.
// 256 threads = 4 waves; each wave owns a WM x WN sub-tile of 16x16 MFMA tiles.
#pragma once
#include "common.hpp"

namespace hlmc {

// ============================================================================ helpers
// Largest K-step of both GEMM families: 8 16-byte chunks per tile row (64 bf16 / 32 f32).  Kernels
// take the chunk count KCH (4 or 8) as a template parameter; split-K ranges are multiples of this.
constexpr int kKCH = 8;
template <typename T>
constexpr int gemm_bk() { return kKCH * Vec16<T>::N; }

// XCD-aware block order (cdna_hip_programming.md T1): the dispatcher deals linear block ids round-robin over
// the 8 XCDs (ids b and b+8 share an L2), so map them to logical ids that run consecutively on one XCD; blocks
// that share operand rows (the N-tiles / phases of one M-tile, the tiles of one K-split) then share an L2.
// Bijective for any total (q = total / 8 logical ids per XCD, the first total % 8 XCD labels get one more).
// Placement is a speed hint only: every logical id is still computed exactly once.
__device__ __forceinline__ int xcd_logical_block(int lin, int total) {
    const int xcd = lin & 7, idx = lin >> 3;
    const int q = total >> 3, r = total & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// 16 zero bytes: the source of every out-of-range / padding chunk of the LDS-DMA (global_load_lds) loaders
static __device__ __attribute__((aligned(16))) uint4 g_zero16 = {0u, 0u, 0u, 0u};
// a 16-byte chunk whose first element is 1 (the ones column of a weight-gradient operand)
template <typename T> __device__ __attribute__((aligned(16))) uint4 g_one16 = {sizeof(T) == 2 ? 0x3F80u : 0x3F800000u, 0u, 0u, 0u};

// ============================================================================ A / B loaders (NT)
// Loader contract: set_phase(p); int K() const;
//   Row prep(int m)  — once per tile row, outside the K loop;
//   Ctx ctx(int k)   — once per (thread, K-step): everything that depends only on this thread's k;
//   uint4 load(const Row&, const Ctx&)        — 16 bytes = V consecutive k, zero outside the operand;
//   const void* addr(const Row&, const Ctx&)  — the same chunk's global address or g_zero16 (LDS-DMA path).
// A thread's 16-byte chunk column is fixed for the whole kernel, so per row and step a load costs one
// flag test and one 64-bit add.

template <typename T>
struct DenseLoader {  // X[m * ld + k], m < M, k < K
    const T* p;
    int ld, M, Kd;
    bool vec;  // ld % VEC == 0 and p 16B aligned
    struct Row {
        const T* r;
    };
    struct Ctx {
        int k;
    };
    __device__ void set_phase(int) {}
    __device__ int K() const { return Kd; }
    __device__ Row prep(int m) const { return Row{m < M ? p + (int64_t)m * ld : nullptr}; }
    __device__ Ctx ctx(int k) const { return Ctx{k}; }
    __device__ const void* addr(const Row& rw, const Ctx& cx) const {  // DMA path: Kd % V == 0, 16-byte rows
        return (rw.r && cx.k < Kd) ? static_cast<const void*>(rw.r + cx.k) : static_cast<const void*>(&g_zero16);
    }
    // whole-chunk operand (Kd % V == 0, aligned rows: every conv weight): the kernel takes the unconditional
    // load from addr() for all its chunks (one uniform branch around the whole K-step's loads: a per-chunk branch
    // makes hipcc wait for every outstanding load at its join)
    __host__ __device__ bool vec_ok() const { return vec && (Kd % Vec16<T>::N) == 0; }
    __device__ uint4 load(const Row& rw, const Ctx& cx) const {
        constexpr int V = Vec16<T>::N;
        const int k = cx.k;
        if (vec && (Kd % V) == 0) return *reinterpret_cast<const uint4*>(addr(rw, cx));
        if (!rw.r) return make_uint4(0, 0, 0, 0);
        if (vec && k + V <= Kd) return *reinterpret_cast<const uint4*>(rw.r + k);
        union { uint4 u; T e[V]; } x;
#pragma unroll
        for (int i = 0; i < V; ++i) x.e[i] = (k + i < Kd) ? rw.r[k + i] : from_f32<T>(0.f);
        return x.u;
    }
};

// Stride-2, pad-1, 3x3 window gather over an NHWC map: A(m = (b,oh,ow), k = (kh,kw,ci))
//   = X[b, 2oh-1+kh, 2ow-1+kw, ci].  Requires C % VEC == 0 (a 16-byte chunk never straddles taps);
// chunks past K = 9C read as zeros.  Row flags: bit0 row out of range, bit1 top row (oh = 0), bit2 left
// column (ow = 0), bit3 always set; the step's Ctx rejects the rows whose flags meet its mask.
template <typename T>
struct ConvS2Loader {
    const T* x;
    int Hi, Wi, C, Ho, Wo, M;
    int cshift;  // log2(C) when C is a power of two, else -1
    FastDiv dWo, dHo;
    struct Row {
        int64_t base;  // element offset of (b, 2oh-1, 2ow-1, 0)
        int flags;
    };
    struct Ctx {
        int64_t off;  // (kh*Wi + kw)*C + ci
        int reject;   // bit0 always; bit1 if kh == 0; bit2 if kw == 0; bit3 if tap >= 9
    };
    __device__ void set_phase(int) {}
    __device__ int K() const { return 9 * C; }
    __device__ Row prep(int m) const {
        if (m >= M) return Row{0, 1 | 8};
        const int t = (int)dWo.div((uint32_t)m), ow = m - t * Wo;
        const int b = (int)dHo.div((uint32_t)t), oh = t - b * Ho;
        return Row{(((int64_t)b * Hi + 2 * oh - 1) * Wi + 2 * ow - 1) * C, 8 | (oh == 0 ? 2 : 0) | (ow == 0 ? 4 : 0)};
    }
    __device__ Ctx ctx(int k) const {
        const int tap = cshift >= 0 ? (k >> cshift) : k / C;
        const int ci = k - tap * C;
        const int kh = tap / 3, kw = tap - kh * 3;
        return Ctx{((int64_t)kh * Wi + kw) * C + ci, 1 | (kh == 0 ? 2 : 0) | (kw == 0 ? 4 : 0) | (tap >= 9 ? 8 : 0)};
    }
    __host__ __device__ bool vec_ok() const { return true; }
    // unconditional load from a selected address (no branch around the load: hipcc would wait per chunk)
    __device__ uint4 load(const Row& rw, const Ctx& cx) const { return *reinterpret_cast<const uint4*>(addr(rw, cx)); }
    __device__ const void* addr(const Row& rw, const Ctx& cx) const {
        if (rw.flags & cx.reject) return &g_zero16;
        return x + rw.base + cx.off;
    }
};

// Sub-pixel phase of a stride-2 transposed 3x3 conv (pad 1, output_padding 1) / of the stride-2
// conv's data gradient.  Output pixel (2r+py, 2c+px) gathers low-res X[b, r+dr, c+dc, ci] over taps:
//   parity 0 -> {kh=1, dr=0};  parity 1 -> {kh=0, dr=+1}, {kh=2, dr=0}.
__device__ __forceinline__ int sp_ntaps(int par) { return par ? 2 : 1; }
__device__ __forceinline__ int sp_kidx(int par, int t) { return par ? (t ? 2 : 0) : 1; }
__device__ __forceinline__ int sp_delta(int par, int t) { return (par && t == 0) ? 1 : 0; }

// Row flags: bit0 row out of range, bit1 last low-res row (r+1 outside), bit2 last column, bit3 always.
template <typename T>
struct SubpixelLoader {
    const T* x;  // low-res NHWC [B, Hi, Wi, C]
    int Hi, Wi, C, M;  // M = B*Hi*Wi
    int cshift;
    int py, px, ntx, Kd;
    FastDiv dWi, dHi;
    struct Row {
        int64_t base;  // offset of (b, r, c, 0)
        int flags;
    };
    struct Ctx {
        int64_t off;  // (dr*Wi + dc)*C + ci
        int reject;   // bit0 always; bit1 if dr; bit2 if dc; bit3 if k >= K
    };
    __device__ void set_phase(int p) {
        py = p >> 1; px = p & 1;
        ntx = sp_ntaps(px);
        Kd = sp_ntaps(py) * ntx * C;
    }
    __device__ int K() const { return Kd; }
    __device__ Row prep(int m) const {
        if (m >= M) return Row{0, 1 | 8};
        const int t = (int)dWi.div((uint32_t)m), c = m - t * Wi;
        const int b = (int)dHi.div((uint32_t)t), r = t - b * Hi;
        return Row{(((int64_t)b * Hi + r) * Wi + c) * C, 8 | (r == Hi - 1 ? 2 : 0) | (c == Wi - 1 ? 4 : 0)};
    }
    __device__ Ctx ctx(int k) const {
        const int tt = cshift >= 0 ? (k >> cshift) : k / C;
        const int ci = k - tt * C;
        const int ty = ntx == 2 ? (tt >> 1) : tt, tx = ntx == 2 ? (tt & 1) : 0;
        const int dr = sp_delta(py, ty), dc = sp_delta(px, tx);
        return Ctx{((int64_t)dr * Wi + dc) * C + ci, 1 | (dr ? 2 : 0) | (dc ? 4 : 0) | (k >= Kd ? 8 : 0)};
    }
    __host__ __device__ bool vec_ok() const { return true; }
    // unconditional load from a selected address (no branch around the load: hipcc would wait per chunk)
    __device__ uint4 load(const Row& rw, const Ctx& cx) const { return *reinterpret_cast<const uint4*>(addr(rw, cx)); }
    __device__ const void* addr(const Row& rw, const Ctx& cx) const {
        if (rw.flags & cx.reject) return &g_zero16;
        return x + rw.base + cx.off;
    }
};

// B operand for a sub-pixel phase: packed P[n][kh][kw][C]; k = (ty,tx,ci) -> tap (kh,kw) of the phase.
template <typename T>
struct SubpixelWeight {
    const T* w;
    int C, N;
    int cshift;
    int py, px, ntx, Kd;
    struct Row {
        const T* r;
    };
    struct Ctx {
        int off;  // (kh*3 + kw)*C + ci, or -1 past K
    };
    __device__ void set_phase(int p) {
        py = p >> 1; px = p & 1;
        ntx = sp_ntaps(px);
        Kd = sp_ntaps(py) * ntx * C;
    }
    __device__ int K() const { return Kd; }
    __device__ Row prep(int n) const { return Row{n < N ? w + (int64_t)n * 9 * C : nullptr}; }
    __device__ Ctx ctx(int k) const {
        if (k >= Kd) return Ctx{-1};
        const int tt = cshift >= 0 ? (k >> cshift) : k / C;
        const int ci = k - tt * C;
        const int ty = ntx == 2 ? (tt >> 1) : tt, tx = ntx == 2 ? (tt & 1) : 0;
        return Ctx{(sp_kidx(py, ty) * 3 + sp_kidx(px, tx)) * C + ci};
    }
    __host__ __device__ bool vec_ok() const { return true; }
    __device__ uint4 load(const Row& rw, const Ctx& cx) const { return *reinterpret_cast<const uint4*>(addr(rw, cx)); }
    __device__ const void* addr(const Row& rw, const Ctx& cx) const {
        if (!rw.r || cx.off < 0) return &g_zero16;
        return rw.r + cx.off;
    }
};

// ============================================================================ epilogues
// Epilogue contract (two access forms):
//   GEMM tiles:  float colbias(n) (hoisted per column); Quad quad(m) once per 4 consecutive rows m..m+3
//                (m % 4 == 0, the MFMA C/D row group of a lane); float put(const Quad&, r, n, v) stores
//                row m+r, column n of v (= accumulator + colbias) and returns the stored value as float.
//   split-K reduce (per element): set_phase(p); Row row(int m); store(const Row&, int n, float v).
// 4 consecutive outputs rounded to OutT and stored with one 8-byte (bf16) / 16-byte (f32) store; v <- the stored values
template <typename OutT>
__device__ __forceinline__ void store4_round(OutT* p, float (&v)[4]) {
    if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        unsigned h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bf16 t = __float2bfloat16(v[k]);
            h[k] = *reinterpret_cast<unsigned short*>(&t);
            v[k] = __uint_as_float(h[k] << 16);
        }
        *reinterpret_cast<uint2*>(p) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    }
}

// Row-major store with bias, activation, optional accumulate:  out[m*ld + n] (+)= act(v + bias[n])
// act: 0 none, 1 relu
template <typename OutT>
struct StoreRM {
    static constexpr int kStatMode = 0;
    static constexpr bool kDirectTn = true;  // gemm_tn_kernel may store through it directly (TnDirect)
    OutT* out;
    const float* bias;
    int ld, act, accumulate;
    struct Row {
        OutT* r;
    };
    struct Quad {
        int64_t off;  // element offset of row m
    };
    __device__ void set_split(int) {}
    __device__ float colbias(int n) const { return bias ? bias[n] : 0.f; }
    __device__ Quad quad(int m) const { return Quad{(int64_t)m * ld}; }
    __device__ int64_t row_off(const Quad& q, int r) const { return q.off + (int64_t)r * ld; }
    __device__ float put(int64_t ro, int n, float v) const {
        if (act == 1) v = v > 0.f ? v : 0.f;
        OutT* o = out + ro + n;
        if (accumulate) v += to_f32<OutT>(*o);
        const OutT t = from_f32<OutT>(v);
        *o = t;
        return to_f32<OutT>(t);
    }
    // columns n..n+3 of row offset ro in one vector store (v: accumulators + bias; <- the stored values)
    __device__ void put4(int64_t ro, int n, float (&v)[4]) const {
        OutT* o = out + ro + n;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (act == 1) v[k] = v[k] > 0.f ? v[k] : 0.f;
            if (accumulate) v[k] += to_f32<OutT>(o[k]);
        }
        store4_round<OutT>(o, v);
    }
    // put / put4 without the accumulate read (kernels whose output is never accumulated into: no global loads)
    __device__ float put_na(int64_t ro, int n, float v) const {
        if (act == 1) v = v > 0.f ? v : 0.f;
        const OutT t = from_f32<OutT>(v);
        out[ro + n] = t;
        return to_f32<OutT>(t);
    }
    __device__ void put4_na(int64_t ro, int n, float (&v)[4]) const {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (act == 1) v[k] = v[k] > 0.f ? v[k] : 0.f;
        store4_round<OutT>(out + ro + n, v);
    }
    // the value store() writes (without accumulate), as float: for the fused column statistics
    __device__ float stored(int n, float v) const {
        if (bias) v += bias[n];
        if (act == 1) v = v > 0.f ? v : 0.f;
        return to_f32<OutT>(from_f32<OutT>(v));
    }
    __device__ void set_phase(int) {}
    __device__ Row row(int m) const { return Row{out + (int64_t)m * ld}; }
    __device__ void store(const Row& rw, int n, float v) const {
        if (bias) v += bias[n];
        if (act == 1) v = v > 0.f ? v : 0.f;
        OutT* o = rw.r + n;
        if (accumulate) v += to_f32<OutT>(*o);
        *o = from_f32<OutT>(v);
    }
};

// StoreRM followed by the ReLU backward mask of the layer below: the stored (accumulated) value is zeroed where
// relu_ref (that layer's post-ReLU activation, same row stride ld) is not positive.  Replaces a relu_bwd pass over
// the data gradient (one launch and a read-modify-write of the map per dense layer).
template <typename OutT>
struct StoreReluBwd : StoreRM<OutT> {
    const OutT* relu_ref;
    __device__ bool live(int64_t e) const { return to_f32<OutT>(relu_ref[e]) > 0.f; }
    __device__ float put(int64_t ro, int n, float v) const {
        OutT* o = this->out + ro + n;
        if (this->accumulate) v += to_f32<OutT>(*o);
        if (!live(ro + n)) v = 0.f;
        const OutT t = from_f32<OutT>(v);
        *o = t;
        return to_f32<OutT>(t);
    }
    __device__ void put4(int64_t ro, int n, float (&v)[4]) const {
        OutT* o = this->out + ro + n;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (this->accumulate) v[k] += to_f32<OutT>(o[k]);
            if (!live(ro + n + k)) v[k] = 0.f;
        }
        store4_round<OutT>(o, v);
    }
    __device__ void store(const typename StoreRM<OutT>::Row& rw, int n, float v) const {
        if (this->bias) v += this->bias[n];
        OutT* o = rw.r + n;
        if (this->accumulate) v += to_f32<OutT>(*o);
        if (!live(o - this->out)) v = 0.f;
        *o = from_f32<OutT>(v);
    }
};

// Sub-pixel phase store into a high-res NHWC map [B, 2Hi, 2Wi, N]; m = (b, r, c) over the low grid.
template <typename OutT>
struct StoreSubpixel {
    static constexpr int kStatMode = 0;
    OutT* out;
    const float* bias;
    int Hi, Wi, N;
    int py, px;
    FastDiv dWi, dHi;
    struct Row {
        OutT* r;
    };
    struct Quad {
        int64_t off;  // element offset of row m (Wi % 4 == 0: rows m+1..m+3 are the next low-res columns)
        int m;
    };
    __device__ int64_t pix_off(int m) const {
        const int t = (int)dWi.div((uint32_t)m), c = m - t * Wi;
        const int b = (int)dHi.div((uint32_t)t), r = t - b * Hi;
        return (((int64_t)b * 2 * Hi + 2 * r + py) * (2 * Wi) + 2 * c + px) * N;
    }
    __device__ void set_split(int) {}
    __device__ float colbias(int n) const { return bias ? bias[n] : 0.f; }
    __device__ Quad quad(int m) const { return Quad{pix_off(m), m}; }
    __device__ int64_t row_off(const Quad& q, int r) const {
        return (Wi & 3) == 0 ? q.off + (int64_t)2 * r * N : pix_off(q.m + r);
    }
    __device__ float put(int64_t ro, int n, float v) const {
        const OutT t = from_f32<OutT>(v);
        out[ro + n] = t;
        return to_f32<OutT>(t);
    }
    __device__ void put4(int64_t ro, int n, float (&v)[4]) const { store4_round<OutT>(out + ro + n, v); }
    __device__ float put_na(int64_t ro, int n, float v) const { return put(ro, n, v); }
    __device__ void put4_na(int64_t ro, int n, float (&v)[4]) const { put4(ro, n, v); }
    __device__ float stored(int n, float v) const {
        if (bias) v += bias[n];
        return to_f32<OutT>(from_f32<OutT>(v));
    }
    __device__ void set_phase(int p) { py = p >> 1; px = p & 1; }
    __device__ Row row(int m) const {
        const int c = m % Wi, t = m / Wi;
        const int r = t % Hi, b = t / Hi;
        const int64_t pix = ((int64_t)b * 2 * Hi + 2 * r + py) * (2 * Wi) + 2 * c + px;
        return Row{out + pix * N};
    }
    __device__ void store(const Row& rw, int n, float v) const {
        if (bias) v += bias[n];
        rw.r[n] = from_f32<OutT>(v);
    }
};

// Any epilogue plus fused per-column statistics of the stored values (BatchNorm batch statistics): each block's
// column sums (f64, fixed-order reduction over its rows) go to the exact accumulator `acc` (2N columns: sum n,
// sum of squares N + n; common.hpp XAcc) -- the consumer reads the totals, no fold launch.
template <class Base>
struct WithStats : Base {
    static constexpr int kStatMode = 1;
    XAcc acc;
};

// Split-K partial slab: ws[((phase * S + split) * M + m) * N + n]
struct StorePartial {
    static constexpr int kStatMode = 0;
    float* ws;
    int M, N, S;
    int phase, split;
    struct Row {
        float* r;
    };
    __device__ void set_phase(int p) { phase = p; }
    __device__ Row row(int m) const { return Row{ws + (((int64_t)phase * S + split) * M + m) * N}; }
    __device__ void store(const Row& rw, int n, float v) const { rw.r[n] = v; }
    struct Quad {
        int64_t off;
    };
    __device__ void set_split(int z) { split = z; }
    __device__ float colbias(int) const { return 0.f; }
    __device__ Quad quad(int m) const { return Quad{(((int64_t)phase * S + split) * M + m) * N}; }
    __device__ int64_t row_off(const Quad& q, int r) const { return q.off + (int64_t)r * N; }
    __device__ float put(int64_t ro, int n, float v) const {
        ws[ro + n] = v;
        return v;
    }
    __device__ void put4(int64_t ro, int n, float (&v)[4]) const {
        *reinterpret_cast<float4*>(ws + ro + n) = make_float4(v[0], v[1], v[2], v[3]);
    }
};

// Store one wave's TM x TN grid of 16x16 accumulator tiles through the epilogue (C/D map: col = lane & 15,
// rows (lane >> 4) * 4 + 0..3), bias hoisted per column, one quad() per 4-row group.  EP::kStatMode 1: per-column
// sum / sum of squares of the stored values over this lane's rows into cs / cq (f64).
template <int TM, int TN, class EP>
__device__ __forceinline__ void epilogue_tile(const EP& ep, const f32x4_t (&acc)[TM][TN], int mb, int nb, int lane,
                                              int M, int N, double (&cs)[TN], double (&cq)[TN]) {
    float bias[TN];
    int ncol[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        ncol[j] = nb + j * 16 + (lane & 15);
        bias[j] = ncol[j] < N ? ep.colbias(ncol[j]) : 0.f;
        cs[j] = 0.0;
        cq[j] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + (lane >> 4) * 4;
        if (m >= M) continue;
        const typename EP::Quad q = ep.quad(m);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (m + r >= M) continue;
            const int64_t ro = ep.row_off(q, r);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if (ncol[j] >= N) continue;
                const float v = ep.put(ro, ncol[j], acc[i][j][r] + bias[j]);
                if constexpr (EP::kStatMode == 1) {
                    cs[j] += v;
                    cq[j] += (double)v * v;
                }
            }
        }
    }
}

// The same for accumulators computed with the operands swapped (mfma(B fragment, A fragment)): acc[i][j] holds the
// 16 x 16 tile (columns nb + j*16 .., rows mb + i*16 ..) TRANSPOSED, i.e. lane l has columns nb + j*16 + 4*(l >> 4)
// + 0..3 of row mb + i*16 + (l & 15).  Each lane stores its 4 consecutive columns with one vector store (put4: 8 bytes
// for bf16) instead of 4 scalar 2-byte stores, so an NHWC output tile costs a quarter of the store instructions.
// kStatMode 1: per-column sums / sums of squares of the stored values, reduced over the 16 rows of each lane group
// (xor shuffles) -> cs / cq [j][k] hold the totals of column nb + j*16 + 4*(lane >> 4) + k in every lane.
// F32RED: the per-lane sums (<= TM bf16-exact values and their squares) and the 16-lane shuffle tree in f32 (one
// DPP / swizzle step per value instead of two plus an f64 add), widened to f64 afterwards — bf16 outputs (the
// throughput mode); fp32 outputs (the parity mode) keep f64 throughout.
template <int TM, int TN, class EP, bool F32RED = false>
__device__ __forceinline__ void epilogue_tile_t(const EP& ep, const f32x4_t (&acc)[TM][TN], int mb, int nb, int lane,
                                                int M, int N, double (&cs)[TN][4], double (&cq)[TN][4]) {
    using Acc = typename std::conditional<F32RED, float, double>::type;
    Acc as[TN][4], aq[TN][4];
    float bias[TN][4];
    int n4[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        n4[j] = nb + j * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bias[j][k] = n4[j] + k < N ? ep.colbias(n4[j] + k) : 0.f;
            as[j][k] = Acc(0);
            aq[j][k] = Acc(0);
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + (lane & 15);
        if (m >= M) continue;
        const int64_t ro = ep.row_off(ep.quad(m), 0);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (n4[j] >= N) continue;  // N % 4 == 0 (checked by the launcher)
            float v[4] = {acc[i][j][0] + bias[j][0], acc[i][j][1] + bias[j][1], acc[i][j][2] + bias[j][2],
                          acc[i][j][3] + bias[j][3]};
            ep.put4(ro, n4[j], v);
            if constexpr (EP::kStatMode == 1) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    as[j][k] += Acc(v[k]);
                    aq[j][k] += Acc(v[k]) * Acc(v[k]);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (EP::kStatMode == 1) {
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    as[j][k] += __shfl_xor(as[j][k], o, 64);
                    aq[j][k] += __shfl_xor(aq[j][k], o, 64);
                }
            }
            cs[j][k] = (double)as[j][k];
            cq[j][k] = (double)aq[j][k];
        }
}

// A wave's per-column statistics (its rows) into the block scratch sred[(wmi * 2 + {0, 1}) * BN + column] for the
// column strip wn0 .. wn0 + 16 TN: TR = false from epilogue_tile's per-lane sums (xor over the 4 row groups),
// TR = true from epilogue_tile_t's already-reduced totals.
template <bool TR, int TN, int BN>
__device__ __forceinline__ void stats_to_lds(const double* cs, const double* cq, double* sred, int wmi, int wn0,
                                             int lane) {
    if constexpr (TR) {
        if ((lane & 15) == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    sred[(wmi * 2 + 0) * BN + wn0 + j * 16 + 4 * (lane >> 4) + k] = cs[j * 4 + k];
                    sred[(wmi * 2 + 1) * BN + wn0 + j * 16 + 4 * (lane >> 4) + k] = cq[j * 4 + k];
                }
        }
    } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            double a = cs[j], q = cq[j];
            a += __shfl_xor(a, 16, 64);
            q += __shfl_xor(q, 16, 64);
            a += __shfl_xor(a, 32, 64);
            q += __shfl_xor(q, 32, 64);
            if (lane < 16) {
                sred[(wmi * 2 + 0) * BN + wn0 + j * 16 + lane] = a;
                sred[(wmi * 2 + 1) * BN + wn0 + j * 16 + lane] = q;
            }
        }
    }
}
// one MFMA step of a wave's TM x TN tile grid: TR = true swaps the operands (transposed accumulators,
// epilogue_tile_t), else the row-per-lane-group layout of epilogue_tile
template <bool TR>
__device__ __forceinline__ f32x4_t mfma_bf16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
    if constexpr (TR) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <bool TR>
__device__ __forceinline__ f32x4_t mfma_f32(float a, float b, const f32x4_t& c) {
    if constexpr (TR) return __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Block coordinates of the NT kernels after the XCD remap: logical id -> (phase fastest, then tile, then
// K-split), so the phases and N-tiles of one M-tile (which gather the same A rows) run on one XCD.
#define NT_BLOCK_COORDS()                                                                                  \
    const int gx_ = (int)gridDim.x, gy_ = (int)gridDim.y;                                                  \
    const int lin_ = (int)blockIdx.x + gx_ * ((int)blockIdx.y + gy_ * (int)blockIdx.z);                     \
    const int lg_ = remap ? xcd_logical_block(lin_, gx_ * gy_ * (int)gridDim.z) : 0;                       \
    const int phase = remap ? lg_ % gy_ : (int)blockIdx.y;                                                 \
    const int tile_ = remap ? (lg_ / gy_) % gx_ : (int)blockIdx.x;                                         \
    const int bz = remap ? lg_ / (gx_ * gy_) : (int)blockIdx.z;                                            \
    const int m0 = (tile_ / tiles_n) * BM, n0 = (tile_ % tiles_n) * BN;                                     \
    const int tile_m_ = tile_ / tiles_n

// Physical 16-byte chunk of logical chunk c in LDS tile row `row` (rows of KCH chunks, unpadded).  The bf16
// A/B fragment read (ds_read_b128: lane l -> row l & 15, chunk 4s + (l >> 4)) is then conflict-free in all
// four 16-lane bank groups (cdna_hip_programming.md §2 bank rule): 128-B rows XOR the chunk with row & 7;
// 64-B rows (4 per 256-B bank row) XOR it with f((row >> 2) & 3), f = {0, 2, 3, 1}.  The ds_write_b128 fill
// (8 consecutive lanes = 2 or 1 whole rows) stays conflict-free under any per-row chunk permutation.
template <int KCH>
__device__ __forceinline__ int nt_lds_chunk(int row, int c) {
    if constexpr (KCH == 8) return c ^ (row & 7);
    else return c ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3);
}

// ============================================================================ NT main loop
// ploop > 1: the grid has one y-slice and every block runs all ploop phases of its tile in turn (the sub-pixel
// phases of one M-tile gather overlapping low-res rows: the later phases find them in L2 instead of every
// phase's blocks streaming the whole input again).
template <typename T, int BM, int BN, int WM, int WN, int KCH, class AL, class BL, class EP, bool TR = false>
__global__ __launch_bounds__(256) void gemm_nt_kernel(AL al, BL bl, EP ep, int M, int N, int ksplit_len, int remap,
                                                      int ploop) {
    constexpr int V = Vec16<T>::N;
    constexpr int BK = KCH * V;  // LDS rows of KCH 16-byte chunks, chunk positions swizzled (nt_lds_chunk)
    constexpr int WAVES_N = BN / WN;
    static_assert((BM / WM) * WAVES_N == 4, "4 waves per block");
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ACH = BM * KCH, BCH = BN * KCH;     // 16-byte chunks per tile
    constexpr int AR = (ACH + 255) / 256, BR = (BCH + 255) / 256;
    __shared__ __attribute__((aligned(16))) T As[2][BM * BK];
    __shared__ __attribute__((aligned(16))) T Bs[2][BN * BK];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
    const int tiles_n = (N + BN - 1) / BN;
    NT_BLOCK_COORDS();
    typename AL::Row arow[AR];   // row preparation does not depend on the phase
    typename BL::Row brow[BR];
#pragma unroll
    for (int i = 0; i < AR; ++i) arow[i] = al.prep(m0 + ((tid + i * 256) / KCH));
#pragma unroll
    for (int i = 0; i < BR; ++i) brow[i] = bl.prep(n0 + ((tid + i * 256) / KCH));
    const int ph0 = ploop > 1 ? 0 : phase, ph1 = ploop > 1 ? ploop : phase + 1;
    for (int ph = ph0; ph < ph1; ++ph) {
    al.set_phase(ph); bl.set_phase(ph); ep.set_phase(ph); ep.set_split(bz);
    const int K = al.K();
    const int kb = bz * ksplit_len;
    const int ke = min(K, kb + ksplit_len);

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    struct Regs {
        uint4 a[AR], b[BR];
    };
    Regs r0;  // staging set: one K-step of global loads in flight (measured: a second set, two steps in
              // flight, was 1.2-1.6x slower on every short-K layer — lower occupancy)
    const int kc = (tid % KCH) * V;  // this thread's chunk column (256 % KCH == 0: the same for every i)
    const bool vec = al.vec_ok() && bl.vec_ok();  // uniform: every chunk from addr() (DenseLoader::vec_ok)
    auto gload = [&](Regs& rg, int k0) {
        const typename AL::Ctx ax = al.ctx(k0 + kc);
        const typename BL::Ctx bx = bl.ctx(k0 + kc);
        if (vec) {
#pragma unroll
            for (int i = 0; i < AR; ++i) {
                int c = tid + i * 256;
                if (ACH % 256 == 0 || c < ACH) rg.a[i] = *reinterpret_cast<const uint4*>(al.addr(arow[i], ax));
            }
#pragma unroll
            for (int i = 0; i < BR; ++i) {
                int c = tid + i * 256;
                if (BCH % 256 == 0 || c < BCH) rg.b[i] = *reinterpret_cast<const uint4*>(bl.addr(brow[i], bx));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            int c = tid + i * 256;
            if (ACH % 256 == 0 || c < ACH) rg.a[i] = al.load(arow[i], ax);
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            int c = tid + i * 256;
            if (BCH % 256 == 0 || c < BCH) rg.b[i] = bl.load(brow[i], bx);
        }
    };
    auto lstore = [&](const Regs& rg, int buf) {
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            int c = tid + i * 256;
            if (ACH % 256 == 0 || c < ACH)
                *reinterpret_cast<uint4*>(&As[buf][(c / KCH) * BK + nt_lds_chunk<KCH>(c / KCH, c % KCH) * V]) = rg.a[i];
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            int c = tid + i * 256;
            if (BCH % 256 == 0 || c < BCH)
                *reinterpret_cast<uint4*>(&Bs[buf][(c / KCH) * BK + nt_lds_chunk<KCH>(c / KCH, c % KCH) * V]) = rg.b[i];
        }
    };

    auto mma_step = [&](int cur) {
        const T* A = As[cur];
        const T* B = Bs[cur];
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int s = 0; s < BK / 32; ++s) {
                bf16x8_t af[TM], bfr[TN];
                const int c = s * 4 + (lane >> 4);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm0 + i * 16 + (lane & 15);
                    af[i] = *reinterpret_cast<const bf16x8_t*>(&A[row * BK + nt_lds_chunk<KCH>(row, c) * 8]);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn0 + j * 16 + (lane & 15);
                    bfr[j] = *reinterpret_cast<const bf16x8_t*>(&B[row * BK + nt_lds_chunk<KCH>(row, c) * 8]);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = mfma_bf16<TR>(af[i], bfr[j], acc[i][j]);
            }
        } else {
#pragma unroll
            for (int s = 0; s < BK / 4; ++s) {
                float af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm0 + i * 16 + (lane & 15);
                    af[i] = A[row * BK + nt_lds_chunk<KCH>(row, s) * 4 + (lane >> 4)];
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn0 + j * 16 + (lane & 15);
                    bfr[j] = B[row * BK + nt_lds_chunk<KCH>(row, s) * 4 + (lane >> 4)];
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = mfma_f32<TR>(af[i], bfr[j], acc[i][j]);
            }
        }
    };
    if (kb < ke) {
        gload(r0, kb);
        lstore(r0, 0);
        __syncthreads();
        int it = 0;
        for (int k0 = kb; k0 < ke; k0 += BK, ++it) {
            const int cur = it & 1;
            const bool more = k0 + BK < ke;
            if (more) gload(r0, k0 + BK);
            mma_step(cur);
            if (more) lstore(r0, cur ^ 1);
            __syncthreads();
        }
    }
    double cs[TR ? TN * 4 : TN], cq[TR ? TN * 4 : TN];
    if constexpr (TR)
        epilogue_tile_t<TM, TN, EP, sizeof(T) == 2>(ep, acc, m0 + wm0, n0 + wn0, lane, M, N,
                                *reinterpret_cast<double(*)[TN][4]>(cs), *reinterpret_cast<double(*)[TN][4]>(cq));
    else
        epilogue_tile<TM, TN>(ep, acc, m0 + wm0, n0 + wn0, lane, M, N, cs, cq);
    if constexpr (EP::kStatMode != 0) {
        // per-column sum / sum of squares of the stored values over the block's rows: the wave's column totals
        // (stats_to_lds), then the waves of one column strip in order
        constexpr int WAVES_M = BM / WM;
        __shared__ double sred[WAVES_M][2][BN];
        const int wmi = wave / WAVES_N;
        stats_to_lds<TR, TN, BN>(cs, cq, &sred[0][0][0], wmi, wn0, lane);
        __syncthreads();
        const int shard = (int)((blockIdx.x + gridDim.x * blockIdx.y) % (unsigned)ep.acc.shards);
        for (int c = tid; c < BN; c += 256) {
            const int n = n0 + c;
            if (n >= N) continue;
            double a = 0.0, q = 0.0;
#pragma unroll
            for (int w = 0; w < WAVES_M; ++w) {
                a += sred[w][0][c];
                q += sred[w][1][c];
            }
            xacc_add_shard(ep.acc, shard, n, a);
            xacc_add_shard(ep.acc, shard, N + n, q);
        }
    }
    if (ph + 1 < ph1) __syncthreads();  // the next phase's LDS fills / statistics scratch
    }
}

// ============================================================================ NT main loop, LDS-DMA pipeline
// NS-stage ring of [rows][8 x 16-byte chunks] tiles in LDS, filled by global_load_lds_dwordx4 (no register
// staging): one wave-instruction writes 1 KB = 8 rows; lane l of it writes physical chunk l & 7 of row l >> 3
// and fetches logical chunk (l & 7) ^ (row & 7) (XOR swizzle on the SOURCE address keeps the LDS image
// lane-linear and makes the MFMA fragment reads bank-conflict-free).  Per K-step: counted vmcnt wait for this
// stage's DMA, raw barrier, issue the stage NS-1 ahead into the buffer everyone just finished, MFMAs.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int GPW, int NS>
__device__ __forceinline__ void wait_stage(int ahead) {  // ahead = stages still allowed in flight (< NS-1)
    if constexpr (NS >= 4) {
        if (ahead >= 2) { wait_vmcnt<2 * GPW>(); return; }
    }
    if constexpr (NS >= 3) {
        if (ahead >= 1) { wait_vmcnt<GPW>(); return; }
    }
    wait_vmcnt<0>();
}
__device__ __forceinline__ void glds16(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// WPE: waves per SIMD the register allocation targets (2 with the 2-stage ring: two blocks per CU)
template <typename T, int BM, int BN, int WM, int WN, int NS, class AL, class BL, class EP, bool TR = false, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void gemm_nt_glds_kernel(
    AL al, BL bl, EP ep, int M, int N, int ksplit_len, int remap) {
    constexpr int V = Vec16<T>::N;
    constexpr int BK = 8 * V;                       // 128-byte tile rows
    constexpr int ASZ = BM * 128, BSZ = BN * 128, STG = ASZ + BSZ;
    constexpr int AI = BM / 8, BI = BN / 8;         // 1 KB DMA instructions per stage
    static_assert(AI % 4 == 0 && BI >= 4 && BI % 4 == 0, "tile rows per stage must split over 4 waves");
    constexpr int AIW = AI / 4, BIW = BI / 4, GPW = AIW + BIW;
    constexpr int WAVES_N = BN / WN;
    static_assert((BM / WM) * WAVES_N == 4, "4 waves per block");
    constexpr int TM = WM / 16, TN = WN / 16;
    __shared__ __attribute__((aligned(1024))) char smem[NS * STG];  // the only LDS object (see vmcnt traps)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
    const int tiles_n = (N + BN - 1) / BN;
    NT_BLOCK_COORDS();
    al.set_phase(phase); bl.set_phase(phase); ep.set_phase(phase); ep.set_split(bz);
    const int K = al.K();
    const int kb = bz * ksplit_len;
    const int ke = min(K, kb + ksplit_len);
    const int nsteps = kb < ke ? (ke - kb + BK - 1) / BK : 0;

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int lrow = lane >> 3;
    const int lchunk = (lane & 7) ^ (lrow & 7);  // logical chunk fetched by this lane (row & 7 == lrow)
    typename AL::Row arow[AIW];
    typename BL::Row brow[BIW];
#pragma unroll
    for (int i = 0; i < AIW; ++i) arow[i] = al.prep(m0 + (wave * AIW + i) * 8 + lrow);
#pragma unroll
    for (int i = 0; i < BIW; ++i) brow[i] = bl.prep(n0 + (wave * BIW + i) * 8 + lrow);
    auto issue = [&](int slot, int k0) {
        char* sb = smem + slot * STG;
        const int k = k0 + lchunk * V;
        const typename AL::Ctx ax = al.ctx(k);
        const typename BL::Ctx bx = bl.ctx(k);
#pragma unroll
        for (int i = 0; i < AIW; ++i) glds16(al.addr(arow[i], ax), sb + (wave * AIW + i) * 1024);
#pragma unroll
        for (int i = 0; i < BIW; ++i) glds16(bl.addr(brow[i], bx), sb + ASZ + (wave * BIW + i) * 1024);
    };

#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
        if (p < nsteps) issue(p, kb + p * BK);
    for (int t = 0; t < nsteps; ++t) {
        wait_stage<GPW, NS>(min(NS - 2, nsteps - 1 - t));
        __builtin_amdgcn_s_barrier();
        if (t + NS - 1 < nsteps) issue((t + NS - 1) % NS, kb + (t + NS - 1) * BK);
        const char* sa = smem + (t % NS) * STG;
        const char* sbb = sa + ASZ;
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int s = 0; s < BK / 32; ++s) {
                const int c = 4 * s + (lane >> 4);
                bf16x8_t af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm0 + i * 16 + (lane & 15);
                    af[i] = *reinterpret_cast<const bf16x8_t*>(sa + row * 128 + ((c ^ (row & 7)) << 4));
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn0 + j * 16 + (lane & 15);
                    bfr[j] = *reinterpret_cast<const bf16x8_t*>(sbb + row * 128 + ((c ^ (row & 7)) << 4));
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = mfma_bf16<TR>(af[i], bfr[j], acc[i][j]);
            }
        } else {
#pragma unroll
            for (int s = 0; s < BK / 4; ++s) {
                float af[TM], bfr[TN];
                const int q = lane >> 4;  // k = 4 s + q: chunk s, word q
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm0 + i * 16 + (lane & 15);
                    af[i] = *reinterpret_cast<const float*>(sa + row * 128 + ((s ^ (row & 7)) << 4) + q * 4);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn0 + j * 16 + (lane & 15);
                    bfr[j] = *reinterpret_cast<const float*>(sbb + row * 128 + ((s ^ (row & 7)) << 4) + q * 4);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = mfma_f32<TR>(af[i], bfr[j], acc[i][j]);
            }
        }
    }
    double cs[TR ? TN * 4 : TN], cq[TR ? TN * 4 : TN];
    if constexpr (TR)
        epilogue_tile_t<TM, TN, EP, sizeof(T) == 2>(ep, acc, m0 + wm0, n0 + wn0, lane, M, N,
                                *reinterpret_cast<double(*)[TN][4]>(cs), *reinterpret_cast<double(*)[TN][4]>(cq));
    else
        epilogue_tile<TM, TN>(ep, acc, m0 + wm0, n0 + wn0, lane, M, N, cs, cq);
    if constexpr (EP::kStatMode != 0) {
        constexpr int WAVES_M = BM / WM;
        static_assert(WAVES_M * 2 * BN * 8 <= NS * STG, "stats scratch fits the staging ring");
        __syncthreads();  // every wave is done with the ring: reuse it for the column-sum scratch
        double* sred = reinterpret_cast<double*>(smem);  // [WAVES_M][2][BN]
        const int wmi = wave / WAVES_N;
        stats_to_lds<TR, TN, BN>(cs, cq, sred, wmi, wn0, lane);
        __syncthreads();
        const int shard = (int)((blockIdx.x + gridDim.x * blockIdx.y) % (unsigned)ep.acc.shards);
        for (int c = tid; c < BN; c += 256) {
            const int n = n0 + c;
            if (n >= N) continue;
            double a = 0.0, q = 0.0;
#pragma unroll
            for (int w = 0; w < WAVES_M; ++w) {
                a += sred[(w * 2 + 0) * BN + c];
                q += sred[(w * 2 + 1) * BN + c];
            }
            xacc_add_shard(ep.acc, shard, n, a);
            xacc_add_shard(ep.acc, shard, N + n, q);
        }
    }
}

// Split-K wrapper epilogue: the z-index of the grid selects the partial slab.
struct StorePartialZ : StorePartial {
    __device__ void set_split(int z) { split = z; }  // the block's (XCD-remapped) K-split index
};

// Reduce split-K partials (fixed order => deterministic) then apply the final epilogue.
template <class EP>
__global__ void splitk_reduce_kernel(const float* ws, EP ep, int M, int N, int S, int phases) {
    int64_t total = (int64_t)phases * M * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int n = (int)(i % N);
        int64_t t = i / N;
        int m = (int)(t % M);
        int ph = (int)(t / M);
        const float* p = ws + ((int64_t)ph * S * M + m) * N + n;
        const int64_t st = (int64_t)M * N;
        // fixed summation order (k ascending) with 4 slab loads in flight
        float s = 0.f;
        int k = 0;
        for (; k + 4 <= S; k += 4) {
            const float a0 = p[k * st], a1 = p[(k + 1) * st], a2 = p[(k + 2) * st], a3 = p[(k + 3) * st];
            s += a0; s += a1; s += a2; s += a3;
        }
        for (; k < S; ++k) s += p[k * st];
        EP e = ep;
        e.set_phase(ph);
        e.store(e.row(m), n, s);
    }
}

// The same with one float4 of outputs per thread (N % 4 == 0, phases * S * M * N < 2^31, 16-byte aligned slabs):
// 16-byte slab loads and 32-bit index math (the 64-bit divisions above cost more than the loads); each output's
// additions in the same order as above (the same bits)
template <class EP>
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float* __restrict__ ws, EP ep, int M, int N, int S,
                                                             int phases, FastDiv dN, FastDiv dM) {
    const uint32_t e = (blockIdx.x * 256u + threadIdx.x) * 4u;
    if (e >= (uint32_t)phases * (uint32_t)M * (uint32_t)N) return;
    const uint32_t t = dN.div(e), n = e - t * (uint32_t)N;
    const uint32_t ph = dM.div(t), m = t - ph * (uint32_t)M;
    const uint32_t st = (uint32_t)M * (uint32_t)N;
    const float* p = ws + ((ph * (uint32_t)S) * (uint32_t)M + m) * (uint32_t)N + n;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [](float4& x, const float4& y) { x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w; };
    int k = 0;
    for (; k + 4 <= S; k += 4) {
        const float4 a0 = *reinterpret_cast<const float4*>(p + k * st);
        const float4 a1 = *reinterpret_cast<const float4*>(p + (k + 1) * st);
        const float4 a2 = *reinterpret_cast<const float4*>(p + (k + 2) * st);
        const float4 a3 = *reinterpret_cast<const float4*>(p + (k + 3) * st);
        add(a, a0); add(a, a1); add(a, a2); add(a, a3);
    }
    for (; k < S; ++k) add(a, *reinterpret_cast<const float4*>(p + k * st));
    EP o = ep;
    o.set_phase((int)ph);
    const auto rw = o.row((int)m);
    o.store(rw, (int)n, a.x);
    o.store(rw, (int)n + 1, a.y);
    o.store(rw, (int)n + 2, a.z);
    o.store(rw, (int)n + 3, a.w);
}

// The same reduction for a launch whose output feeds a train-mode BatchNorm: block = a tile of 4 * RU output rows
// (phase-major) x 64 columns; it also delivers the column sums / sums of squares of the values it stored to `acc`
// (2N columns, common.hpp XAcc) -- no separate moments pass over the output.  Thread (column tid % 64, row group
// tid / 64) owns rows g, g + 4, ...; every row is loaded before the adds (two slabs at a time, k ascending: the sums
// equal splitk_reduce_kernel's).  Tall tiles keep the accumulator adds per output element low (6 per column per
// tile: measured, 16-row tiles were atomic-bound at 3x the plain reduce's time).  Needs N % 64 == 0 and
// phases * S * M * N < 2^31 (32-bit offsets).
template <class EP, int RU>
__global__ __launch_bounds__(256) void splitk_reduce_stats_kernel(const float* ws, EP ep, int M, int N, int S,
                                                                  int phases, XAcc acc) {
    __shared__ double red[2][256];
    const int tid = threadIdx.x, c = tid & 63, g = tid >> 6;
    const int ntc = N >> 6;
    const int tr = (int)(blockIdx.x / (unsigned)ntc);
    const int col = ((int)blockIdx.x - tr * ntc) * 64 + c;
    const int rows = phases * M;
    const unsigned st = (unsigned)M * (unsigned)N;
    const int r0 = tr * 4 * RU + g;
    unsigned off[RU];
    float s[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
        const int r = min(r0 + 4 * u, rows - 1);  // clamped: in bounds, skipped below
        const int ph = r / M, m = r - ph * M;
        off[u] = ((unsigned)(ph * S) * (unsigned)M + (unsigned)m) * (unsigned)N + (unsigned)col;
        s[u] = 0.f;
    }
    int k = 0;
    for (; k + 2 <= S; k += 2) {
        float x0[RU], x1[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            x0[u] = ws[off[u] + (unsigned)k * st];
            x1[u] = ws[off[u] + (unsigned)(k + 1) * st];
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            s[u] += x0[u];
            s[u] += x1[u];
        }
    }
    if (k < S)
#pragma unroll
        for (int u = 0; u < RU; ++u) s[u] += ws[off[u] + (unsigned)k * st];
    double a = 0.0, q = 0.0;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
        const int r = r0 + 4 * u;
        if (r >= rows) break;
        const int ph = r / M, m = r - ph * M;
        EP e = ep;
        e.set_phase(ph);
        e.store(e.row(m), col, s[u]);
        const float v = e.stored(col, s[u]);
        a += v;
        q += (double)v * v;
    }
    red[0][tid] = a;
    red[1][tid] = q;
    __syncthreads();
    if (tid < 64) {
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            a += red[0][j * 64 + tid];
            q += red[1][j * 64 + tid];
        }
        xacc_add(acc, col, a);
        xacc_add(acc, N + col, q);
    }
}

// ============================================================================ TN (weight-gradient) loaders
// Contract: Col prep(int col) (once per chunk column, outside the K loop); uint4 load(int k, const Col&)
// returns V consecutive columns of k-row k.
template <typename T>
struct KRowDense {
    const T* p;
    int ld, Kd, Md;  // rows (k) and columns (m/n)
    bool vec;        // rows 16-byte aligned (ld % V == 0)
    bool ones;       // a virtual column Md of ones: column Md of the product is the row sum of the other operand
                     // (a linear layer's bias gradient from its weight-gradient GEMM; register path only)
    struct Col {
        int m;
    };
    __device__ Col prep(int m) const { return Col{m}; }
    // LDS-DMA path (vec, Md % V == 0, no ones column): the 16-byte chunk's address or g_zero16 outside the operand
    __device__ const void* addr(int k, const Col& cl) const {
        return (k < Kd && cl.m < Md) ? static_cast<const void*>(p + (int64_t)k * ld + cl.m) : &g_zero16;
    }
    // branch-free path (vec_ok: 16-byte rows, Md % V == 0): one 16-byte load from a selected address -- the chunk,
    // g_zero16 outside the operand, g_one16 for the ones column's chunk.  (The per-element fallback inside the
    // K loop made the compiler wait for every outstanding load at its join: the loads issued one at a time.)
    __host__ bool vec_ok() const { return vec && Md % Vec16<T>::N == 0; }
    __device__ uint4 vload(int k, const Col& cl) const {
        // every candidate address formed, then selected (a conditional expression over them compiled to divergent
        // branches around the index math)
        const bool in = k < Kd && cl.m < Md, one = k < Kd && ones && cl.m == Md;
        const uintptr_t pa = reinterpret_cast<uintptr_t>(p + (int64_t)k * ld + cl.m);
        const uintptr_t po = reinterpret_cast<uintptr_t>(&g_one16<T>), pz = reinterpret_cast<uintptr_t>(&g_zero16);
        const uintptr_t a = in ? pa : (one ? po : pz);
        return *reinterpret_cast<const uint4*>(a);
    }
    __device__ uint4 load(int k, const Col& cl) const {
        constexpr int V = Vec16<T>::N;
        const int m = cl.m;
        if (k >= Kd) return make_uint4(0, 0, 0, 0);
        const T* r = p + (int64_t)k * ld;
        if (vec && m + V <= Md) return *reinterpret_cast<const uint4*>(r + m);
        union { uint4 u; T e[V]; } x;
#pragma unroll
        for (int i = 0; i < V; ++i)
            x.e[i] = (m + i < Md) ? r[m + i] : from_f32<T>((ones && m + i == Md) ? 1.f : 0.f);
        return x.u;
    }    // stepped form (gemm_tn_kernel): the chunk's row j of the K-step and its column, the step's first row k0
    struct Pre {
        Col cl;
        int j;
    };
    __device__ Pre pre(int j, int m) const { return Pre{prep(m), j}; }
    __device__ int step(int k0) const { return k0; }
    template <bool VEC>
    __device__ uint4 sload(int k0, const Pre& p) const { return VEC ? vload(k0 + p.j, p.cl) : load(k0 + p.j, p.cl); }
};

// H loader for stride-2 conv / transposed conv weight gradient: k = (b, r, c) over the LOW-res grid,
// n = (kh, kw, ci): H(k, n) = Xh[b, 2r-1+kh, 2c-1+kw, ci] over the HIGH-res NHWC map [B, 2Hl, 2Wl, C].
template <typename T>
struct KRowConvS2 {
    const T* x;
    int Hl, Wl, C, Kd;  // Kd = B*Hl*Wl
    FastDiv dW, dH;     // division by Wl and Hl
    struct Col {
        int off;  // (kh*Wh + kw)*C + ci relative to pixel (2r-1, 2c-1)
        int kh, kw;
        bool ok;
    };
    __device__ Col prep(int n) const {
        if (n >= 9 * C) return Col{0, 0, 0, false};
        const int tap = n / C, ci = n - tap * C;
        const int kh = tap / 3, kw = tap - kh * 3;
        return Col{(kh * 2 * Wl + kw) * C + ci, kh, kw, true};
    }
    // branch-free: every term computed for every lane and the zero chunk chosen by a select (early returns compiled
    // to divergent branches around the index math, and the joins cost the weight-gradient loop its exact wait counts:
    // it waited for every outstanding load at the LDS store of the oldest)
    __device__ const void* addr(int k, const Col& cl) const {
        const uint32_t t = dW.div((uint32_t)k);
        const int c = k - (int)t * Wl;
        const uint32_t b = dH.div(t);
        const int r = (int)t - (int)b * Hl;
        const bool zero = k >= Kd || !cl.ok || (r == 0 && cl.kh == 0) || (c == 0 && cl.kw == 0);
        const int64_t pix = ((int64_t)b * 2 * Hl + 2 * r - 1) * (2 * Wl) + 2 * c - 1;
        const uintptr_t a = reinterpret_cast<uintptr_t>(x + pix * C + cl.off);
        return reinterpret_cast<const void*>(zero ? reinterpret_cast<uintptr_t>(&g_zero16) : a);
    }
    __host__ bool vec_ok() const { return true; }
    __device__ uint4 vload(int k, const Col& cl) const { return *reinterpret_cast<const uint4*>(addr(k, cl)); }
    __device__ uint4 load(int k, const Col& cl) const {
        if (k >= Kd || !cl.ok) return make_uint4(0, 0, 0, 0);
        const uint32_t t = dW.div((uint32_t)k);
        const int c = k - (int)t * Wl;
        const uint32_t b = dH.div(t);
        const int r = (int)t - (int)b * Hl;
        if ((r == 0 && cl.kh == 0) || (c == 0 && cl.kw == 0)) return make_uint4(0, 0, 0, 0);
        const int64_t pix = ((int64_t)b * 2 * Hl + 2 * r - 1) * (2 * Wl) + 2 * c - 1;
        return *reinterpret_cast<const uint4*>(x + pix * C + cl.off);
    }    // stepped form (gemm_tn_kernel): the chunk's row j of the K-step and its column, the step's first row k0
    struct Pre {
        Col cl;
        int j;
    };
    __device__ Pre pre(int j, int m) const { return Pre{prep(m), j}; }
    __device__ int step(int k0) const { return k0; }
    template <bool VEC>
    __device__ uint4 sload(int k0, const Pre& p) const { return VEC ? vload(k0 + p.j, p.cl) : load(k0 + p.j, p.cl); }
};

// Buffer-descriptor forms of the two weight-gradient loaders for power-of-two sizes (every layer of the model: image
// sides, channel counts and row strides are powers of two) and operands under 2 GB: one 32-bit byte offset per 16-byte
// chunk from shifts and adds, loaded with raw_buffer_load_b128 through a range-checked descriptor, so every zero chunk
// (padding taps, rows past K, columns past N) is an offset past the descriptor's end that the hardware returns as zeros
// -- no select between addresses, no 64-bit products.  The general loaders above spent ~1,700 VALU cycles per K-step
// and wave on their index math (28 v_mul_lo_u32 / 16 v_mad_u64_u32 / 8 v_mul_hi_u32 among 243 vector instructions, the
// quarter-rate ones 16 cycles each) against 512 cycles of MFMA, with one wave per SIMD to issue both.
constexpr int kBufOut = 0x7FFFFFF0;  // a byte offset past every descriptor's end: the load returns zeros
template <typename T>
struct KRowDenseP2 {  // X[k * 2^lld + m], k < Kd, m < Md (Md % V == 0)
    const T* p;
    int lld, Kd, Md;
    uint32_t bytes;   // Kd << lld elements, in bytes
    struct Col {
        int m;
    };
    __device__ Col prep(int m) const { return Col{m}; }
    __host__ bool vec_ok() const { return true; }
    __device__ uint4 vload(int k, const Col& cl) const {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(p), (short)0, (int)bytes, 0x00020000);
        const int off = (k < Kd && cl.m < Md) ? ((k << lld) + cl.m) * (int)sizeof(T) : kBufOut;
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
    __device__ uint4 load(int k, const Col& cl) const { return vload(k, cl); }
    // stepped form: byte offset of (row j, column m) -- kBufOut past the columns -- plus the step's k0 rows; rows
    // past Kd land past the descriptor's end (Kd << lld elements) and read as zeros with no test
    struct Pre {
        uint32_t v;
    };
    __device__ Pre pre(int j, int m) const { return Pre{m < Md ? (uint32_t)(((j << lld) + m) * (int)sizeof(T)) : (uint32_t)kBufOut}; }
    __device__ uint32_t step(int k0) const { return (uint32_t)(k0 << lld) * (uint32_t)sizeof(T); }
    template <bool VEC>
    __device__ uint4 sload(uint32_t s, const Pre& pr) const {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(p), (short)0, (int)bytes, 0x00020000);
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(pr.v + s), 0, 0));
    }
};
template <typename T>
struct KRowConvS2P2 {  // KRowConvS2 with Hl = 2^lh, Wl = 2^lw, C = 2^lc
    const T* x;
    int lh, lw, lc, Kd;
    uint32_t bytes;   // the high-res map [B, 2Hl, 2Wl, C] in bytes
    struct Col {
        int off;  // (kh * 2Wl + kw) * C + ci relative to pixel (2r-1, 2c-1)
        int kh, kw;
        bool ok;
    };
    __device__ Col prep(int n) const {
        const int C = 1 << lc;
        if (n >= 9 * C) return Col{0, 0, 0, false};
        const int tap = n >> lc, ci = n & (C - 1);
        const int kh = tap / 3, kw = tap - kh * 3;
        return Col{((kh << (lw + 1)) + kw) * C + ci, kh, kw, true};
    }
    __host__ bool vec_ok() const { return true; }
    __device__ uint4 vload(int k, const Col& cl) const {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(x), (short)0, (int)bytes, 0x00020000);
        const int c = k & ((1 << lw) - 1), t = k >> lw;
        const int r = t & ((1 << lh) - 1), b = t >> lh;
        const bool zero = k >= Kd || !cl.ok || (r == 0 && cl.kh == 0) || (c == 0 && cl.kw == 0);
        // pixel (2r - 1, 2c - 1) of image b in the [2Hl][2Wl] map, then the tap / channel offset
        const int pix = ((((b << lh) + r) * 2 - 1) << (lw + 1)) + 2 * c - 1;
        const int off = zero ? kBufOut : ((pix << lc) + cl.off) * (int)sizeof(T);
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
    __device__ uint4 load(int k, const Col& cl) const { return vload(k, cl); }
    // stepped form.  With k0 % 64 == 0, j < 64 and power-of-two sides, k0 + j splits into (b, r, c) without carries:
    // c = c0 + cj, r = r0 + rj, b = b0 + bj, each first term from k0 alone (wave-uniform), each second from j alone
    // (fixed per chunk), so the pixel offset is a per-step scalar plus a per-chunk constant and the padding tests
    // (r == 0 with kh == 0, c == 0 with kw == 0) are a uniform flag AND a per-chunk flag.  Rows past Kd (b >= B)
    // land past the descriptor's end.
    struct Pre {
        int v;       // byte offset of the chunk at k0 = 0: pixel (2rj - 1 + kh, 2cj - 1 + kw) of image bj, its channels
        bool zr, zc;  // rj == 0 and kh == 0 / cj == 0 and kw == 0
    };
    struct Step {
        uint32_t s;  // byte offset of the step's (b0, r0, c0) pixel block
        bool r0, c0;  // r0 == 0 / c0 == 0
    };
    __device__ Pre pre(int j, int n) const {
        const Col cl = prep(n);
        const int cj = j & ((1 << lw) - 1), tj = j >> lw, rj = tj & ((1 << lh) - 1), bj = tj >> lh;
        const int pix = ((((bj << lh) + rj) * 2 - 1) << (lw + 1)) + 2 * cj - 1;
        if (!cl.ok) return Pre{kBufOut, false, false};  // a column past N: kBufOut + any step offset is past the end
        return Pre{((pix << lc) + cl.off) * (int)sizeof(T), rj == 0 && cl.kh == 0, cj == 0 && cl.kw == 0};
    }
    __device__ Step step(int k0) const {
        const int c0 = k0 & ((1 << lw) - 1), t0 = k0 >> lw, r0 = t0 & ((1 << lh) - 1), b0 = t0 >> lh;
        const uint32_t pix = ((uint32_t)((b0 << lh) + r0) << (lw + 2)) + 2u * (uint32_t)c0;
        return Step{(pix << lc) * (uint32_t)sizeof(T), r0 == 0, c0 == 0};
    }
    template <bool VEC>
    __device__ uint4 sload(const Step& st, const Pre& pr) const {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(x), (short)0, (int)bytes, 0x00020000);
        const bool zero = (st.r0 && pr.zr) || (st.c0 && pr.zc);
        const int off = zero ? kBufOut : (int)((uint32_t)pr.v + st.s);
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
};

#ifdef HLMC_TN_TS  // diagnostic build only: per-block phase timestamps of gemm_tn_kernel (100 MHz wall clock)
__device__ unsigned long long g_tn_ts[8192][4];
#define TN_TS(i)                                                                                   \
    do {                                                                                           \
        const unsigned b_ = blockIdx.x + gridDim.x * blockIdx.z;                                    \
        if (threadIdx.x == 0 && b_ < 8192u) g_tn_ts[b_][i] = wall_clock64();                        \
    } while (0)
#else
#define TN_TS(i)
#endif

// ============================================================================ TN main loop
// XOR swizzle of the 16-byte chunks of a bf16 k-row (CPR chunks per row, 8 or 16) for the ds_read_b64_tr_b16
// fragment reads: the 8 k-rows one 32-lane half reads (q = 0..3, g = 0..1) land on disjoint bank groups.
template <int CPR>
__device__ __forceinline__ int tn_swz(int row) {
    if constexpr (CPR == 16) return 2 * ((row & 3) | (((row >> 3) & 1) << 2));
    else return 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
}

// Output of gemm_tn_kernel: the split's fp32 slab ws[(split * M + m) * N + n], reduced by a split-K reduce launch
struct TnSlab {
    float* ws;
    __device__ void put(int bz, int m, int n, int M, int N, float v) const { ws[((int64_t)bz * M + m) * N + n] = v; }
};
// ... or, when the grid has one split, the final epilogue itself (no slab, no reduce launch): epilogues that flag
// kDirectTn (a store(row(m), n, v) with no once-per-launch side task)
template <class EP>
struct TnDirect {
    EP ep;
    __device__ void put(int, int m, int n, int, int, float v) const {
        EP e = ep;
        e.set_phase(0);
        e.store(e.row(m), n, v);
    }
};
template <class E, class = void>
struct tn_direct : std::false_type {};
template <class E>
struct tn_direct<E, std::void_t<decltype(E::kDirectTn)>> : std::bool_constant<E::kDirectTn> {};

// One K-step of global loads in flight in one register set, double-buffered LDS images.  (Two register sets -- loads
// two K-steps ahead -- measured no faster, round 6, nor did 8-wave blocks or 256-wide tiles: per-block timestamps
// put the K loop at ~0.86 us per 64-deep K-step on the deep layers, bound by the per-CU load throughput.)
template <typename T, int BM, int BN, int WM, int WN, int KCH, class LL, class HL, bool VEC = false, class OUT = TnSlab>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void gemm_tn_kernel(LL ll, HL hl, OUT out, int M, int N, int K,
                                                                             int ksplit_len, int remap) {
    constexpr int V = Vec16<T>::N;
    constexpr int BK = KCH * V;            // k rows per tile (KCH 16-byte chunks of one column)
    constexpr int ACPR = BM / V, BCPR = BN / V;  // chunks per k-row
    // bf16 rows of 8 / 16 chunks: unpadded, XOR-swizzled chunks (tn_swz); otherwise one chunk of padding
    // (measured: the padded 136-element rows put 2-way bank conflicts on a third of the LDS cycles)
    constexpr bool SWA = sizeof(T) == 2 && (ACPR == 8 || ACPR == 16);
    constexpr bool SWB = sizeof(T) == 2 && (BCPR == 8 || BCPR == 16);
    constexpr int LDA = SWA ? BM : BM + V;  // LDS row (elements)
    constexpr int LDB = SWB ? BN : BN + V;
    constexpr int WAVES_N = BN / WN;
    constexpr int NTH = 64 * (BM / WM) * WAVES_N;  // 4 or 8 waves
    static_assert(NTH == 256 || NTH == 512, "4 or 8 waves per block");
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ACH = BK * BM / V, BCH = BK * BN / V;
    constexpr int AR = (ACH + NTH - 1) / NTH, BR = (BCH + NTH - 1) / NTH;
    constexpr int LSZ = BK * LDA, HSZ = BK * LDB;
    __shared__ __attribute__((aligned(16))) T tn_sm[2 * (LSZ + HSZ)];

    TN_TS(0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    T* const Lg = tn_sm;  // L0 H0 L1 H1
    auto Lbuf = [&](int buf) { return Lg + buf * (LSZ + HSZ); };
    auto Hbuf = [&](int buf) { return Lg + buf * (LSZ + HSZ) + LSZ; };
    const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
    const int tiles_n = (N + BN - 1) / BN;
    // XCD remap: the tiles of one K-split (which share L and H rows) run consecutively on one XCD
    const int gx_ = (int)gridDim.x;
    const int lg_ = remap ? xcd_logical_block((int)blockIdx.x + gx_ * (int)blockIdx.z, gx_ * (int)gridDim.z) : 0;
    const int tile_ = remap ? lg_ % gx_ : (int)blockIdx.x, bz = remap ? lg_ / gx_ : (int)blockIdx.z;
    const int m0 = (tile_ / tiles_n) * BM, n0 = (tile_ % tiles_n) * BN;
    const int kb = bz * ksplit_len;
    const int ke = min(K, kb + ksplit_len);

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    struct Regs {
        uint4 a[AR], b[BR];
    };
    // each chunk's K-step row and column are fixed for the whole kernel: the loaders' per-chunk constants once
    // (pre), the per-K-step part once per step (step: wave-uniform), one select / add per chunk and step (sload)
    typename LL::Pre apre[AR];
    typename HL::Pre bpre[BR];
#pragma unroll
    for (int i = 0; i < AR; ++i) {
        const int c = tid + i * NTH;
        apre[i] = ll.pre(c / ACPR, m0 + (c % ACPR) * V);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
        const int c = tid + i * NTH;
        bpre[i] = hl.pre(c / BCPR, n0 + (c % BCPR) * V);
    }
    auto gload = [&](Regs& rg, int k0) {
        const auto sa = ll.step(k0);
        const auto sb = hl.step(k0);
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            int c = tid + i * NTH;
            if (ACH % NTH == 0 || c < ACH)  // (a provable guard: a runtime one put every load in a branch)
                rg.a[i] = ll.template sload<VEC>(sa, apre[i]);
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            int c = tid + i * NTH;
            if (BCH % NTH == 0 || c < BCH) rg.b[i] = hl.template sload<VEC>(sb, bpre[i]);
        }
    };
    auto lstore = [&](const Regs& rg, int buf) {
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            int c = tid + i * NTH;
            if (ACH % NTH == 0 || c < ACH) {
                const int row = c / ACPR, cc = c % ACPR;
                const int pc = SWA ? (cc ^ tn_swz<ACPR>(row)) : cc;
                *reinterpret_cast<uint4*>(&Lbuf(buf)[row * LDA + pc * V]) = rg.a[i];
            }
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            int c = tid + i * NTH;
            if (BCH % NTH == 0 || c < BCH) {
                const int row = c / BCPR, cc = c % BCPR;
                const int pc = SWB ? (cc ^ tn_swz<BCPR>(row)) : cc;
                *reinterpret_cast<uint4*>(&Hbuf(buf)[row * LDB + pc * V]) = rg.b[i];
            }
        }
    };
    // element offset of (k-row, column col) in a tile image (the fragment reads stay inside one 16-byte chunk)
    auto aoff = [](int row, int col) {
        if constexpr (SWA) return row * LDA + (((col >> 3) ^ tn_swz<ACPR>(row)) << 3) + (col & 7);
        else return row * LDA + col;
    };
    auto boff = [](int row, int col) {
        if constexpr (SWB) return row * LDB + (((col >> 3) ^ tn_swz<BCPR>(row)) << 3) + (col & 7);
        else return row * LDB + col;
    };
    const int g = lane >> 4, li = lane & 15;
    auto mma_step = [&](int cur) {
        const T* A = Lbuf(cur);
        const T* B = Hbuf(cur);
        if constexpr (sizeof(T) == 2) {
            // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses row q, cols 4p..4p+3;
            // lane i receives column i of the 4 rows.
            const int q = li >> 2, p = li & 3;
#pragma unroll
            for (int s = 0; s < BK / 32; ++s) {
                bf16x8_t af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int col = wm0 + i * 16 + 4 * p;
                    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(A + aoff(32 * s + 8 * g + q, col)));
                    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(A + aoff(32 * s + 8 * g + q + 4, col)));
                    af[i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = wn0 + j * 16 + 4 * p;
                    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(B + boff(32 * s + 8 * g + q, col)));
                    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(B + boff(32 * s + 8 * g + q + 4, col)));
                    bfr[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int s = 0; s < BK / 4; ++s) {
                float af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = A[(s * 4 + g) * LDA + wm0 + i * 16 + li];
#pragma unroll
                for (int j = 0; j < TN; ++j) bfr[j] = B[(s * 4 + g) * LDB + wn0 + j * 16 + li];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    Regs r0;
    const int nsteps = kb < ke ? (ke - kb + BK - 1) / BK : 0;
    if (nsteps > 0) {
        gload(r0, kb);
        lstore(r0, 0);
        __syncthreads();
        TN_TS(1);
        for (int st = 0; st < nsteps; ++st) {
            const int cur = st & 1;
            const bool more = st + 1 < nsteps;
            if (more) gload(r0, kb + (st + 1) * BK);
            mma_step(cur);
            if (more) lstore(r0, cur ^ 1);
            __syncthreads();
        }
    }
    TN_TS(2);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int m = m0 + wm0 + i * 16 + (lane >> 4) * 4 + r;
                int n = n0 + wn0 + j * 16 + (lane & 15);
                if (m < M && n < N) out.put(bz, m, n, M, N, acc[i][j][r]);
            }
    TN_TS(3);
}

// Split-K reduction parallel over the splits as well as the outputs: a block holds 256 / G outputs x G split
// groups; thread (group g, output o) adds the slabs s = g, g + G, ... (loads issued 4 at a time) in order, then
// the G group sums are added in group order.  Fixed order => deterministic; G = 1 is the plain split-order sum.
// Deep split counts (the 16-262k-row weight gradients split 50-170 ways over 3-18 tiles) are latency chains
// otherwise: one thread per output walking S slabs waits S / 4 memory round trips.
// an epilogue's optional side task (E::extra(), e.g. StoreWgradConv's bias gradient), run once per reduce launch
template <class E>
__device__ __forceinline__ auto ep_extra(const E& e, int) -> decltype(e.extra(), void()) { e.extra(); }
template <class E>
__device__ __forceinline__ void ep_extra(const E&, long) {}

template <int G, class EP>
__global__ __launch_bounds__(256) void splitk_reduce_grouped_kernel(const float* __restrict__ ws, EP ep, int M, int N,
                                                                    int S) {
    ep_extra(ep, 0);
    constexpr int OPB = 256 / G;
    __shared__ float part[G][OPB];
    const int o = threadIdx.x % OPB, g = threadIdx.x / OPB;
    const int64_t idx = (int64_t)blockIdx.x * OPB + o;
    const int64_t total = (int64_t)M * N;
    const int64_t st = total;
    float acc = 0.f;
    if (idx < total) {
        const float* p = ws + idx;
        int k = g;
        for (; k + 3 * G < S; k += 4 * G) {
            const float a0 = p[k * st], a1 = p[(k + G) * st], a2 = p[(k + 2 * G) * st], a3 = p[(k + 3 * G) * st];
            acc += a0; acc += a1; acc += a2; acc += a3;
        }
        for (; k < S; k += G) acc += p[k * st];
    }
    if constexpr (G > 1) {
        part[g][o] = acc;
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int j = 1; j < G; ++j) acc += part[j][o];
    }
    if (idx < total) {
        const int m = (int)(idx / N), n = (int)(idx - (int64_t)m * N);
        EP e = ep;
        e.set_phase(0);
        e.store(e.row(m), n, acc);
    }
}
// The same with 4 consecutive outputs per thread (N % 4 == 0, 16-byte aligned slabs): 16-byte slab loads, 4x the
// bytes in flight per thread; each output's additions in the same order as above (the same bits)
template <int G, class EP>
__global__ __launch_bounds__(256) void splitk_reduce_grouped4_kernel(const float* __restrict__ ws, EP ep, int M, int N,
                                                                     int S) {
    ep_extra(ep, 0);
    constexpr int OPB = 256 / G;  // float4 outputs per block
    __shared__ float4 part[G][OPB];
    const int o = threadIdx.x % OPB, g = threadIdx.x / OPB;
    const int64_t idx = ((int64_t)blockIdx.x * OPB + o) * 4;
    const int64_t total = (int64_t)M * N;
    const int64_t st = total;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [](float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; };
    if (idx < total) {
        const float* p = ws + idx;
        int k = g;
        for (; k + 3 * G < S; k += 4 * G) {
            const float4 a0 = *reinterpret_cast<const float4*>(p + k * st);
            const float4 a1 = *reinterpret_cast<const float4*>(p + (k + G) * st);
            const float4 a2 = *reinterpret_cast<const float4*>(p + (k + 2 * G) * st);
            const float4 a3 = *reinterpret_cast<const float4*>(p + (k + 3 * G) * st);
            add(acc, a0); add(acc, a1); add(acc, a2); add(acc, a3);
        }
        for (; k < S; k += G) add(acc, *reinterpret_cast<const float4*>(p + k * st));
    }
    if constexpr (G > 1) {
        part[g][o] = acc;
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int j = 1; j < G; ++j) add(acc, part[j][o]);
    }
    if (idx < total) {
        const int m = (int)(idx / N), n = (int)(idx - (int64_t)m * N);  // N % 4 == 0: the 4 outputs share row m
        EP e = ep;
        e.set_phase(0);
        const auto rw = e.row(m);
        e.store(rw, n, acc.x);
        e.store(rw, n + 1, acc.y);
        e.store(rw, n + 2, acc.z);
        e.store(rw, n + 3, acc.w);
    }
}

}  // namespace hlmc
