// Launchers for the MFMA GEMM families (tile choice + deterministic split-K planning).
#include "gemm.hpp"
#include "ops.hpp"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace hlmc {
namespace {

// split-K grid targets (A/B on the bench step, scripts in DESIGN.md §8): NT (forward / data-gradient convs,
// linears) 512: 101.8k vs 101.2k at 256 (round 2, after the small split-K grids moved to the LDS-DMA ring;
// round 1 measured 256 ahead of 512 and 128); TN (weight gradients) 512: 93.2k vs 92.8k at 1024, 90.7k at 2048
constexpr int kNtTargetBlocks = 512;
constexpr int kTnTargetBlocks = 192;
constexpr int kTnLongK = 131072;
constexpr int kTnKch8Min = 1024;
// XCD-aware block order (gemm.hpp xcd_logical_block) for these op kinds: measured per layer (scripts/bench_gemm.py),
// it helps the TN (weight-gradient) family and slows the sub-pixel / conv NT families by 10-20 %
constexpr int kXcdRemapKinds = probe::kWgradS2 | probe::kLinearWgrad;

// Split-K plan shared by the launcher and the workspace query (must agree).
struct Plan {
    int S, ksl;
};
// BK = the largest K-step (split ranges are multiples of it); the minimum work per split is counted in
// steps of the short (BK/2) K-step the kernel uses for short ranges
inline Plan plan_nt(int tiles, int Kmax, int BK) {
    constexpr int target = kNtTargetBlocks;
    int S = 1;
    if (tiles < target / 2) {
        S = cdiv(target, tiles);
        S = std::min(S, std::max(1, Kmax / (2 * BK)));
    }
    int ksl = cdiv(cdiv(Kmax, S), BK) * BK;
    S = cdiv(Kmax, ksl);
    return {S, ksl};
}
inline Plan plan_tn(int tiles, int K, int BK) {
    // weight gradients: long K (= batch x pixels), tiny M x N: split K until the grid fills the chip
    // (>= 4 k-tiles per split); the slab reduction keeps 4 loads in flight.  The longest reductions (the
    // 32 / 64-channel layers, K = 262 144) take a 1024-block grid: per layer (scripts/gpu_wgrad_blocks.sh,
    // bench_gemm.py) 47 vs 60 us at 512, while every shorter layer is fastest at 512 (1024: +10-20 %).
    // Round 4 (with the NT GEMMs at two blocks per CU beside them): one 256-block target for every layer measured
    // 134.1k vs 132.9k clips/s at 512 / 1024 (128: 129.6k, 192: 133.6k, 320: 133.6k, 384: 132.1k, 768: 130.8k);
    // the long layers at 512 then 134.5k vs 134.0k (1024: 134.1k).  Round 6, with the cheap power-of-two loaders: 192
    // 142.5k vs 141.8k at 256, 384 139.2k vs 141.9k (3 pairs each; 384 is 7 % faster standalone: the side-stream grids
    // take CUs from the main stream).
    const int target = K >= kTnLongK ? 2 * kTnTargetBlocks : kTnTargetBlocks;
    int S = cdiv(target, tiles);
    S = std::max(1, std::min(S, K / (4 * BK)));
    int ksl = cdiv(cdiv(K, S), BK) * BK;
    S = cdiv(K, ksl);
    return {S, ksl};
}

// NT pipeline: 0 register-staged (gemm_nt_kernel), 2 = the 2-stage LDS-DMA ring (gemm_nt_glds_kernel).
// Measured (scripts/bench_gemm.py): the DMA ring wins when a block reduces >= 1024 (16 K-steps), the register path
// below that (short reductions: more co-resident blocks hide the pipeline prologue) -- except on split-K grids of
// <= 512 blocks, where the ring wins even on 9-step reductions (the 4x4x512 conv / its data gradient: 21.5 vs
// 31.8 us).  The ring's depth: 2 stages (64 KB of LDS, 176 VGPRs: two blocks per CU, each one K-step ahead)
// measured 131.9k vs 129.3k clips/s with 4 stages (128 KB, one block per CU, three K-steps ahead) and 129.7k with 3;
// split grids on the ring up to 1024 blocks 132.0k (3 rounds each; round 4).
constexpr int kGldsSplitMax = 512;
inline int nt_pipe_select(int ksl, int S, int blocks) {
    if (S > 1 && blocks <= kGldsSplitMax) return 2;
    return ksl >= 1024 ? 2 : 0;
}

inline int xcd_remap_for_site() { return (kXcdRemapKinds & probe::g_site.kind) ? 1 : 0; }

// Register-path launches with 4 sub-pixel phases and >= kPloopTiles M x N tiles (>= 4 blocks per CU without
// the phases) run the phases inside each block (gemm_nt_kernel ploop): the 64 x 64 / 32 x 32 layers' phases
// otherwise stream the low-res input from HBM once per phase (measured round 2: 105.2k vs 104.25k clips/s without,
// both the forward and the data-gradient launches gain).
constexpr int kPloopTiles = 1024;
inline bool use_ploop(int phases, int tmn, int pipe) { return phases >= 2 && pipe == 0 && tmn >= kPloopTiles; }

// TR: transposed accumulators + 4-column vector stores (epilogue_tile_t; needs N % 4 == 0 and 4-aligned row
// strides: the conv / sub-pixel NHWC outputs and their split-K slabs), else the per-element epilogue (linears)
template <typename T, int BM, int BN, int WM, int WN, bool TR, class AL, class BL, class E>
void nt_kernel_launch_tr(hipStream_t s, dim3 grid, const AL& al, const BL& bl, const E& ep, int M, int N, int ksl,
                         bool long_k, int pipe) {
    const int rm = xcd_remap_for_site();
    const int ploop = use_ploop((int)grid.y, (int)grid.x, pipe) ? (int)grid.y : 1;
    if (ploop > 1) grid.y = 1;
    HLMC_PROBE_BEGIN(s);
    if (pipe == 2)
        gemm_nt_glds_kernel<T, BM, BN, WM, WN, 2, AL, BL, E, TR, 2><<<grid, 256, 0, s>>>(al, bl, ep, M, N, ksl, rm);
    else if (long_k)
        gemm_nt_kernel<T, BM, BN, WM, WN, 8, AL, BL, E, TR><<<grid, 256, 0, s>>>(al, bl, ep, M, N, ksl, rm, ploop);
    else
        gemm_nt_kernel<T, BM, BN, WM, WN, 4, AL, BL, E, TR><<<grid, 256, 0, s>>>(al, bl, ep, M, N, ksl, rm, ploop);
    HLMC_PROBE_END(s);
}
// The transposed-accumulator epilogue for the conv families (N % 4 == 0).  Measured per layer (scripts/bench_gemm.py,
// round 3): it takes the split-K / LDS-DMA conv and sub-pixel GEMMs from 28-42 to 22-32 us (the 8 x 8 .. 2 x 2
// layers), but makes the LDS halo-tile kernels 4-15 % slower (their stores were not the bound; the swapped fragments
// cost LDS issue) -> halo kernels keep the per-element epilogue.

template <typename T, int BM, int BN, int WM, int WN, bool TR, class AL, class BL, class EP>
int launch_nt(hipStream_t s, const AL& al, const BL& bl, const EP& ep, int M, int N, int Kmax, int phases, Ws ws,
              ops::ColStats* st = nullptr, bool dma_ok = true) {
    constexpr int BK = gemm_bk<T>();
    const int tmn = cdiv(M, BM) * cdiv(N, BN);
    Plan pl = plan_nt(tmn * phases, Kmax, BK);
    dim3 grid(tmn, phases, pl.S);
    // register path: short reductions keep the 4-chunk K-step (more co-resident blocks), long ones 8 chunks
    const bool long_k = Kmax >= 1024;
    const int pipe = (dma_ok && BN >= 32 && BM >= 64) ? nt_pipe_select(pl.ksl, pl.S, tmn * phases * pl.S) : 0;
    const bool stats = st && st->acc.on();
    if (st) st->done = false;
    if (pl.S == 1 && stats) {  // single pass: the epilogue also emits the column statistics
        WithStats<EP> eps;
        static_cast<EP&>(eps) = ep;
        eps.acc = st->acc;
        nt_kernel_launch_tr<T, BM, BN, WM, WN, TR>(s, grid, al, bl, eps, M, N, pl.ksl, long_k, pipe);
        HLMC_LAUNCHED();
        st->done = true;
        return HLMC_OK;
    }
    if (pl.S == 1) {
        nt_kernel_launch_tr<T, BM, BN, WM, WN, TR>(s, grid, al, bl, ep, M, N, pl.ksl, long_k, pipe);
        HLMC_LAUNCHED();
        return HLMC_OK;
    }
    size_t need = (size_t)phases * pl.S * M * N * sizeof(float);
    HLMC_CHECK_ARG(ws.p && ws.bytes >= need, "split-K workspace too small");
    StorePartialZ part;
    part.ws = ws.p; part.M = M; part.N = N; part.S = pl.S; part.phase = 0; part.split = 0;
    nt_kernel_launch_tr<T, BM, BN, WM, WN, TR>(s, grid, al, bl, part, M, N, pl.ksl, long_k, pipe);
    HLMC_LAUNCHED();
    if (stats && N % 64 == 0 && (double)phases * pl.S * M * N < 2147483648.0) {  // the reduce delivers them
        const int rows = phases * M, ntc = N / 64;
        // the tallest tile (fewest accumulator adds) that still gives >= 1024 blocks (A/B: 128 / 256 / 512 / 1024)
        const int RU = cdiv(rows, 128) * ntc >= 1024 ? 32 : cdiv(rows, 64) * ntc >= 1024 ? 16 : 8;
        const unsigned nb = (unsigned)(cdiv(rows, 4 * RU) * ntc);
        switch (RU) {
            case 32: splitk_reduce_stats_kernel<EP, 32><<<nb, 256, 0, s>>>(ws.p, ep, M, N, pl.S, phases, st->acc); break;
            case 16: splitk_reduce_stats_kernel<EP, 16><<<nb, 256, 0, s>>>(ws.p, ep, M, N, pl.S, phases, st->acc); break;
            default: splitk_reduce_stats_kernel<EP, 8><<<nb, 256, 0, s>>>(ws.p, ep, M, N, pl.S, phases, st->acc); break;
        }
        HLMC_LAUNCHED();
        st->done = true;
        return HLMC_OK;
    }
    int64_t total = (int64_t)phases * M * N;
    if (N % 4 == 0 && (double)phases * pl.S * M * N < 2147483648.0 && ((uintptr_t)ws.p & 15) == 0) {
        const unsigned nb = (unsigned)((total / 4 + 255) / 256);
        splitk_reduce4_kernel<EP><<<nb, 256, 0, s>>>(ws.p, ep, M, N, pl.S, phases, FastDiv((uint32_t)N), FastDiv((uint32_t)M));
        HLMC_LAUNCHED();
        return HLMC_OK;
    }
    int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
    splitk_reduce_kernel<EP><<<blocks, 256, 0, s>>>(ws.p, ep, M, N, pl.S, phases);
    HLMC_LAUNCHED();
    return HLMC_OK;
}

template <int BM, int BN>
size_t nt_ws(int M, int N, int Kmax, int phases, int BK) {
    const int tmn = cdiv(M, BM) * cdiv(N, BN);
    Plan pl = plan_nt(tmn * phases, Kmax, BK);
    return pl.S == 1 ? 0 : (size_t)phases * pl.S * M * N * sizeof(float);
}

// Tile choice for the NT family by N: 128x128 / 128x64 / 128x32.  (Measured: stepping down to 64x64 to put
// two blocks on every CU doubles operand re-reads and is slower on every layer of the step.)
inline int nt_tile(int M, int N, int phases) {
    // 128 x 64 tiles where 128 x 128 tiles would give an unsplit grid of target/2 .. target blocks (one block per
    // CU where two fit: the 2-stage ring and the register path hold two): twice the blocks, no split-K slabs.
    // Measured: 133.1k vs 132.3k clips/s (3 rounds); also for target/4 .. target/2 (then split-K) 131.3k.
    if (N >= 128) {
        const int t = cdiv(M, 128) * cdiv(N, 128) * phases;
        if (t >= kNtTargetBlocks / 2 && t < kNtTargetBlocks) return 1;
    }
    if (N >= 128) return 0;
    if (N > 32) return 1;
    return 3;
}
template <typename T, class AL, class BL, class EP>
int dispatch_nt(hipStream_t s, const AL& al, const BL& bl, const EP& ep, int M, int N, int Kmax, int phases, Ws ws,
                ops::ColStats* st = nullptr) {
    // conv / sub-pixel outputs are NHWC rows of N (a multiple of 8) channels: transposed-accumulator epilogue
    if (N % 4 == 0) {
        switch (nt_tile(M, N, phases)) {
            case 0: return launch_nt<T, 128, 128, 64, 64, true>(s, al, bl, ep, M, N, Kmax, phases, ws, st);
            case 1: return launch_nt<T, 128, 64, 32, 64, true>(s, al, bl, ep, M, N, Kmax, phases, ws, st);
            default: return launch_nt<T, 128, 32, 32, 32, true>(s, al, bl, ep, M, N, Kmax, phases, ws, st);
        }
    }
    switch (nt_tile(M, N, phases)) {
        case 0: return launch_nt<T, 128, 128, 64, 64, false>(s, al, bl, ep, M, N, Kmax, phases, ws, st);
        case 1: return launch_nt<T, 128, 64, 32, 64, false>(s, al, bl, ep, M, N, Kmax, phases, ws, st);
        default: return launch_nt<T, 128, 32, 32, 32, false>(s, al, bl, ep, M, N, Kmax, phases, ws, st);
    }
}
template <typename T>
size_t dispatch_nt_ws(int M, int N, int Kmax, int phases) {
    constexpr int BK = gemm_bk<T>();
    switch (nt_tile(M, N, phases)) {
        case 0: return nt_ws<128, 128>(M, N, Kmax, phases, BK);
        case 1: return nt_ws<128, 64>(M, N, Kmax, phases, BK);
        case 2: return nt_ws<64, 64>(M, N, Kmax, phases, BK);
        default: return nt_ws<128, 32>(M, N, Kmax, phases, BK);
    }
}

// Linear layers have small M (= batch): 64x64 tiles so more blocks exist before split-K.
template <typename T, class AL, class BL, class EP>
int dispatch_linear(hipStream_t s, const AL& al, const BL& bl, const EP& ep, int M, int N, int K, Ws ws) {
    // register path: arbitrary ld / K (the DMA path needs 16-byte chunks that never straddle K)
    if (M >= 1024 && N >= 128) return launch_nt<T, 128, 128, 64, 64, false>(s, al, bl, ep, M, N, K, 1, ws, nullptr, false);
    return launch_nt<T, 64, 64, 32, 32, false>(s, al, bl, ep, M, N, K, 1, ws, nullptr, false);
}
template <typename T>
size_t dispatch_linear_ws(int M, int N, int K) {
    constexpr int BK = gemm_bk<T>();
    if (M >= 1024 && N >= 128) return nt_ws<128, 128>(M, N, K, 1, BK);
    return nt_ws<64, 64>(M, N, K, 1, BK);
}

// Final epilogue of a conv weight gradient: C[m][n = tap*C + ci] -> dW[m][ci][tap] (torch layout).
struct StoreWgradConv {
    float* dW;
    int C;
    // the layer's bias gradient (column totals of its exact accumulator) written by the reduce launch's first block
    // (splitk_reduce_grouped_kernel: ep_extra) instead of a separate launch on the weight-gradient stream
    XAcc bacc;
    float* gb = nullptr;
    __device__ void extra() const {
        if (gb && blockIdx.x == 0)
            for (int c = threadIdx.x; c < bacc.ncols; c += blockDim.x) gb[c] = (float)xacc_column(bacc, c);
    }
    struct Row {
        float* r;
    };
    __device__ void set_phase(int) {}
    __device__ Row row(int m) const { return Row{dW + (int64_t)m * C * 9}; }
    __device__ void store(const Row& rw, int n, float v) const {
        int tap = n / C, ci = n - tap * C;
        rw.r[ci * 9 + tap] = v;
    }
};

// Split-K reduction of a conv weight gradient into torch's [M][C][3][3] layout for few splits (S <= 4: the deep
// layers, whose 2-9 MB outputs dominate): one 288-thread block per (row m, 32 input channels) sums the 9 taps x 32
// channels in split order (the slab reads: 9 runs of 32 consecutive floats) and writes the block's 288 consecutive
// dW floats through LDS.  (splitk_reduce_grouped_kernel stores dW[m][ci][tap] from the GEMM's (tap, ci) column
// order: stride-9 scattered 4-byte stores, 10-13 us for these layers.)
__global__ __launch_bounds__(288) void splitk_reduce_wgrad_conv_kernel(const float* __restrict__ ws, StoreWgradConv ep,
                                                                       int M, int C, int S) {
    ep_extra(ep, 0);
    __shared__ float tile[288];
    const int cb = C / 32;
    const int m = blockIdx.x / cb, ci0 = (blockIdx.x - m * cb) * 32;
    const int t = threadIdx.x, tap = t >> 5, cl = t & 31;
    const int64_t N = 9LL * C, st = (int64_t)M * N;
    const float* p = ws + (int64_t)m * N + tap * C + ci0 + cl;
    float acc = 0.f;
    int k = 0;
    for (; k + 3 < S; k += 4) {
        const float a0 = p[k * st], a1 = p[(k + 1) * st], a2 = p[(k + 2) * st], a3 = p[(k + 3) * st];
        acc += a0; acc += a1; acc += a2; acc += a3;
    }
    for (; k < S; ++k) acc += p[k * st];
    tile[cl * 9 + tap] = acc;
    __syncthreads();
    ep.dW[(int64_t)m * N + (int64_t)ci0 * 9 + t] = tile[t];
}

// The same for C % 128 == 0 with 16-byte slab loads: a 288-thread block per (row m, 128 input channels), each thread
// summing 4 consecutive channels of one tap in split order (the same order, so the same bits, as the kernel above),
// the block's 1,152 consecutive dW floats written as float4 through LDS.  (Four-byte loads left too few bytes in
// flight: 2.6-3.5 TB/s on the 2- and 4-split layers.)
__global__ __launch_bounds__(288) void splitk_reduce_wgrad_conv4_kernel(const float* __restrict__ ws, StoreWgradConv ep,
                                                                        int M, int C, int S) {
    ep_extra(ep, 0);
    __shared__ __attribute__((aligned(16))) float tile[128 * 9];
    const int cb = C / 128;
    const int m = blockIdx.x / cb, ci0 = (blockIdx.x - m * cb) * 128;
    const int t = threadIdx.x, tap = t >> 5, cl = t & 31;
    const int64_t N = 9LL * C, st = (int64_t)M * N;
    const float* p = ws + (int64_t)m * N + tap * C + ci0 + 4 * cl;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = 0;
    for (; k + 3 < S; k += 4) {
        const float4 a0 = *reinterpret_cast<const float4*>(p + k * st), a1 = *reinterpret_cast<const float4*>(p + (k + 1) * st);
        const float4 a2 = *reinterpret_cast<const float4*>(p + (k + 2) * st), a3 = *reinterpret_cast<const float4*>(p + (k + 3) * st);
        acc.x += a0.x; acc.y += a0.y; acc.z += a0.z; acc.w += a0.w;
        acc.x += a1.x; acc.y += a1.y; acc.z += a1.z; acc.w += a1.w;
        acc.x += a2.x; acc.y += a2.y; acc.z += a2.z; acc.w += a2.w;
        acc.x += a3.x; acc.y += a3.y; acc.z += a3.z; acc.w += a3.w;
    }
    for (; k < S; ++k) {
        const float4 a = *reinterpret_cast<const float4*>(p + k * st);
        acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    tile[(4 * cl + 0) * 9 + tap] = acc.x;
    tile[(4 * cl + 1) * 9 + tap] = acc.y;
    tile[(4 * cl + 2) * 9 + tap] = acc.z;
    tile[(4 * cl + 3) * 9 + tap] = acc.w;
    __syncthreads();
    *reinterpret_cast<float4*>(ep.dW + (int64_t)m * N + (int64_t)ci0 * 9 + 4 * t) = *reinterpret_cast<const float4*>(&tile[4 * t]);
}

// S-way split-K reduction with the splits spread over G thread groups (splitk_reduce_grouped_kernel)
template <class EP>
void reduce_splits(hipStream_t s, const float* ws, const EP& ep, int M, int N, int S) {
    if constexpr (std::is_same<EP, StoreWgradConv>::value) {
        if (S <= 4 && ep.C % 128 == 0 && (((uintptr_t)ws | (uintptr_t)ep.dW) & 15) == 0) {
            splitk_reduce_wgrad_conv4_kernel<<<(unsigned)(M * (ep.C / 128)), 288, 0, s>>>(ws, ep, M, ep.C, S);
            return;
        }
        if (S <= 4 && ep.C % 32 == 0) {
            splitk_reduce_wgrad_conv_kernel<<<(unsigned)(M * (ep.C / 32)), 288, 0, s>>>(ws, ep, M, ep.C, S);
            return;
        }
    }
    const int64_t total = (int64_t)M * N;
    const bool v4 = N % 4 == 0 && ((uintptr_t)ws & 15) == 0;
    auto go = [&](auto gtag) {
        constexpr int G = decltype(gtag)::value;
        const int64_t per = v4 ? 4 * (256 / G) : 256 / G;  // outputs per block
        const int64_t blocks = (total + per - 1) / per;
        if (v4) splitk_reduce_grouped4_kernel<G, EP><<<(unsigned)blocks, 256, 0, s>>>(ws, ep, M, N, S);
        else splitk_reduce_grouped_kernel<G, EP><<<(unsigned)blocks, 256, 0, s>>>(ws, ep, M, N, S);
    };
    if (S >= 32) go(std::integral_constant<int, 8>{});
    else if (S >= 8) go(std::integral_constant<int, 4>{});
    else if (S >= 4) go(std::integral_constant<int, 2>{});
    else go(std::integral_constant<int, 1>{});
}

template <typename T, int BM, int BN, int WM, int WN, class LL, class HL, class EP>
int launch_tn(hipStream_t s, const LL& ll, const HL& hl, const EP& ep, int M, int N, int K, Ws ws) {
    constexpr int BK = gemm_bk<T>();
    const int tiles = cdiv(M, BM) * cdiv(N, BN);
    Plan pl = plan_tn(tiles, K, BK);
    size_t need = (size_t)pl.S * M * N * sizeof(float);
    HLMC_CHECK_ARG(ws.p && ws.bytes >= need, "wgrad workspace too small");
    dim3 grid(tiles, 1, pl.S);
    const int rm = xcd_remap_for_site();
    HLMC_PROBE_BEGIN(s);
    // the 64-deep K-step for splits of >= 1024 rows (measured: 490.9 vs 450.9 us for the 9 conv layers when
    // every split took it), the 32-deep one below; branch-free 16-byte loads where both operands allow them
    const bool vec = ll.vec_ok() && hl.vec_ok();
    constexpr int NTH = 64 * (BM / WM) * (BN / WN);
    auto go = [&](auto out) {
        using OUT = decltype(out);
        if (pl.ksl >= kTnKch8Min) {
            if (vec) gemm_tn_kernel<T, BM, BN, WM, WN, 8, LL, HL, true, OUT><<<grid, NTH, 0, s>>>(ll, hl, out, M, N, K, pl.ksl, rm);
            else gemm_tn_kernel<T, BM, BN, WM, WN, 8, LL, HL, false, OUT><<<grid, NTH, 0, s>>>(ll, hl, out, M, N, K, pl.ksl, rm);
        } else {
            if (vec) gemm_tn_kernel<T, BM, BN, WM, WN, 4, LL, HL, true, OUT><<<grid, NTH, 0, s>>>(ll, hl, out, M, N, K, pl.ksl, rm);
            else gemm_tn_kernel<T, BM, BN, WM, WN, 4, LL, HL, false, OUT><<<grid, NTH, 0, s>>>(ll, hl, out, M, N, K, pl.ksl, rm);
        }
    };
    if constexpr (tn_direct<EP>::value) {
        if (pl.S == 1) {  // one split (the dense layers' batch-long reductions): the epilogue stores from registers
            go(TnDirect<EP>{ep});
            HLMC_PROBE_END(s);
            HLMC_LAUNCHED();
            return HLMC_OK;
        }
    }
    go(TnSlab{ws.p});
    HLMC_PROBE_END(s);
    HLMC_LAUNCHED();
    reduce_splits(s, ws.p, ep, M, N, pl.S);
    HLMC_LAUNCHED();
    return HLMC_OK;
}
template <int BM, int BN>
size_t tn_ws(int M, int N, int K, int BK) {
    Plan pl = plan_tn(cdiv(M, BM) * cdiv(N, BN), K, BK);
    return (size_t)pl.S * M * N * sizeof(float);
}

// Weight-gradient tile choice.  Weight gradients reduce over K = B * pixels (16 k - 262 k) into a small
// M x N output; the grid is filled by split-K.  Conv weight gradients have N = 9 C: C = 32 gives N = 288,
// which 128-wide tiles cover with 25 % zero columns; 96-wide tiles cover it exactly (measured: 83 -> 72 us for
// the 64 x 288 x 262144 layers).  (Measured and rejected: 64 x 64 tiles everywhere, which cut the split-K slab
// bytes 3-4x but were 10-35 % slower per layer — the kernel is bound by per-block load latency, not slabs.)
inline bool tn_n96(int N) { return N % 128 != 0 && N % 96 == 0; }
// 0: 128x128, 1: 64x128, 2: 64x96, 3: 32x128
inline int tn_tile(int M, int N) {
    if (M >= 128) return 0;
    if (M > 32) return tn_n96(N) ? 2 : 1;
    return 3;
}
template <typename T, class LL, class HL, class EP>
int dispatch_tn(hipStream_t s, const LL& ll, const HL& hl, const EP& ep, int M, int N, int K, Ws ws) {
    switch (tn_tile(M, N)) {
        case 0: return launch_tn<T, 128, 128, 64, 64>(s, ll, hl, ep, M, N, K, ws);
        case 1: return launch_tn<T, 64, 128, 32, 64>(s, ll, hl, ep, M, N, K, ws);
        case 2: return launch_tn<T, 64, 96, 32, 48>(s, ll, hl, ep, M, N, K, ws);
        default: return launch_tn<T, 32, 128, 32, 32>(s, ll, hl, ep, M, N, K, ws);
    }
}
template <typename T>
size_t dispatch_tn_ws(int M, int N, int K) {
    constexpr int BK = gemm_bk<T>();
    size_t w = 0;
    switch (tn_tile(M, N)) {
        case 0: w = tn_ws<128, 128>(M, N, K, BK); break;
        case 1: w = tn_ws<64, 128>(M, N, K, BK); break;
        case 2: w = tn_ws<64, 96>(M, N, K, BK); break;
        default: w = tn_ws<32, 128>(M, N, K, BK); break;
    }
    return w;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline int log2_exact(int c) { return (c > 0 && (c & (c - 1)) == 0) ? __builtin_ctz(c) : -1; }

// The epilogue of the persistent halo kernels: the block's bias columns from an LDS table (filled once before the
// tile loop) and stores without the accumulate read, so the tile loop issues no global loads besides the prefetched
// input rows.  (With the per-tile bias / accumulate loads in the loop the compiler's wait-count merge at the loop
// head waited for ALL outstanding loads -- the prefetch included -- before the first MFMA of every tile.)
template <class EP>
struct HaloEp : EP {
    const float* lb;  // LDS: bias of columns nbase ..
    int nbase;
    __device__ float colbias(int n) const { return lb[n - nbase]; }
    __device__ float put(int64_t ro, int n, float v) const { return EP::put_na(ro, n, v); }
    __device__ void put4(int64_t ro, int n, float (&v)[4]) const { EP::put4_na(ro, n, v); }
};

// ---- train-mode BatchNorm + LeakyReLU(0.01) of a halo kernel's INPUT, applied while its rows are staged (XIN):
// the input pointer is the pre-BN map y of the layer below; the block folds that layer's statistics accumulator
// in its prologue (bn_act_train's consumer-side finalize, same arithmetic; block 0 stores mean / invstd / running
// statistics), transforms each staged 16-byte chunk (8 channels) in registers, and writes the activation a of the
// rows its tile owns (every input row exactly once over the grid, by the first channel-split block) for the weight
// gradient that reads it later.  Rows outside the image stay zero (padding).
struct BnIn {
    XAcc acc;                       // 2C columns
    int64_t R;                      // rows of the normalised map
    float *mean, *invstd, *rmean, *rvar;
    int64_t* nbt;
    float momentum, eps;
    const float *gamma, *beta;
    bf16* a_out;
};
template <int CI>
struct BnInLds {  // prologue scratch + per-channel parameters (LDS)
    double tot[2 * CI];
    long long red[3 * 256];
    float prm[4 * CI];  // mean | invstd | gamma | beta
};
template <int CI>
__device__ __forceinline__ void bn_in_prologue(const BnIn& f, BnInLds<CI>& L) {
    xacc_fold(f.acc, L.tot, L.red);
    for (int c = threadIdx.x; c < CI; c += 256) {
        const double m = L.tot[c] / (double)f.R;
        double var = L.tot[CI + c] / (double)f.R - m * m;
        if (var < 0.0) var = 0.0;
        const float mf = (float)m, inv = (float)(1.0 / sqrt(var + (double)f.eps));
        L.prm[c] = mf;
        L.prm[CI + c] = inv;
        L.prm[2 * CI + c] = f.gamma[c];
        L.prm[3 * CI + c] = f.beta[c];
        if (blockIdx.x == 0) {
            f.mean[c] = mf;
            f.invstd[c] = inv;
            if (f.rmean) {
                const double unb = f.R > 1 ? var * (double)f.R / (double)(f.R - 1) : var;
                f.rmean[c] = (float)((1.0 - f.momentum) * f.rmean[c] + f.momentum * m);
                f.rvar[c] = (float)((1.0 - f.momentum) * f.rvar[c] + f.momentum * unb);
            }
            if (c == 0 && f.nbt) f.nbt[0] += 1;
        }
    }
    __syncthreads();
}
// lrelu((x - mean) * invstd * gamma + beta) of 8 bf16 channels (the thread's parameters in registers)
__device__ __forceinline__ uint4 bn_in_apply(uint4 v, const float (&pr)[4][8]) {
    float x[8];
    cvt16_f32<bf16>(v, x);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float z = (x[k] - pr[0][k]) * pr[1][k] * pr[2][k] + pr[3][k];
        x[k] = z > 0.f ? z : 0.01f * z;
    }
    uint4 o;
    unsigned* w = reinterpret_cast<unsigned*>(&o);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bf16 lo = __float2bfloat16(x[2 * i]), hi = __float2bfloat16(x[2 * i + 1]);
        w[i] = (unsigned)(*reinterpret_cast<unsigned short*>(&lo)) | ((unsigned)(*reinterpret_cast<unsigned short*>(&hi)) << 16);
    }
    return o;
}

// ---- stride-2 3x3 conv over LDS halo tiles: Ci = 32, Wo = 32, bf16, Co = CO.
// Measured (scripts/bench_gemm.py): the 64x64x32 -> 64 conv and the matching decoder data gradient 46.3 / 44.1 ->
// 36.7 / 34.2 us; bench A/B 106.4k vs 105.0k clips/s (3 alternating rounds).
// A persistent block (one per CU) keeps the packed weights [CO][9 x 32] in LDS and walks 128-pixel M-tiles (4
// output rows of one image).  Each tile's 9 input rows (plus the zero column left of the image) are staged in
// LDS once, and every tap's A fragment is read from there: the input crosses L2 once per tile instead of once
// per (tap, 16-byte chunk) gather.  The next tile's rows are loaded into registers while this tile computes.
// Template: CI input channels, COB output channels per block (NSPL blocks share a tile's Co = NSPL * COB), WO
// output width, ROWS output rows per tile (TP = ROWS * WO pixels), DB: double-buffered halo (else one buffer and
// an extra barrier).  Shapes: 2 WO * CI / 8 == 256 (one 16-byte chunk per thread per input row).
template <int CI, int COB, int NSPL, int WO, int ROWS, bool DB, class EP, bool TR = true, bool XIN = false, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void conv_s2_halo_kernel(const bf16* __restrict__ x, int Hi, int ntiles,
                                                           const bf16* __restrict__ wp, EP ep, int M, BnIn xin) {
    constexpr int WI = 2 * WO, HR = 2 * ROWS + 1, HC = WI + 1, PS = CI + 8;  // halo rows / cols / pixel pitch
    constexpr int TP = ROWS * WO, CPP = CI / 8;                             // tile pixels, chunks per pixel
    static_assert(WI * CPP == 256 && (COB == 64 || COB == 32), "halo chunk map / wave tiling");
    constexpr int KP = 9 * CI + 8;      // weight row: 16 n-rows of a fragment read on distinct 16-byte slots
    constexpr int HS = HR * HC * PS;    // one halo buffer (bf16)
    constexpr int WAVES_N = COB / 32;   // 4 waves: 2 x 2 over (TP x 64) or 4 x 1 over (TP x 32)
    constexpr int WM = TP / (4 / WAVES_N), WN = 32, TM = WM / 16, TN = 2;
    static_assert(WM % 16 == 0, "wave rows");
    constexpr int CO = NSPL * COB;
    __shared__ __attribute__((aligned(16))) bf16 Bs[COB * KP];
    __shared__ __attribute__((aligned(16))) bf16 Hs[(DB ? 2 : 1) * HS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
    const int tpi = (Hi / 2) / ROWS;   // tiles per image
    const int nh = blockIdx.x % NSPL, n0 = nh * COB;
    const int bstep = gridDim.x / NSPL;
    __shared__ float bsh[COB];  // this block's bias columns
    if (tid < COB) bsh[tid] = n0 + tid < CO ? ep.colbias(n0 + tid) : 0.f;
    HaloEp<EP> hep;
    static_cast<EP&>(hep) = ep;
    hep.lb = bsh;
    hep.nbase = n0;
    for (int c = tid; c < COB * 9 * CPP; c += 256) {  // this block's weight rows
        const int n = c / (9 * CPP), q = c - n * (9 * CPP);
        *reinterpret_cast<uint4*>(&Bs[n * KP + q * 8]) =
            *reinterpret_cast<const uint4*>(wp + (int64_t)(n0 + n) * 9 * CI + q * 8);
    }
    for (int c = tid; c < (DB ? 2 : 1) * HR * CPP; c += 256) {  // the pad column (input column -1) stays zero
        const int bufr = c / CPP, q = c - bufr * CPP;
        *reinterpret_cast<uint4*>(&Hs[(bufr / HR) * HS + ((bufr % HR) * HC) * PS + q * 8]) = make_uint4(0, 0, 0, 0);
    }
    uint4 hr[HR];  // HR rows x 256 chunks / 256 threads
    auto row_off = [&](int b, int ih) { return (((int64_t)b * Hi + ih) * WI + tid / CPP) * CI + (tid % CPP) * 8; };
    // unconditional loads (row -1 clamped to row 0; zeroed when staged): a branch per row made the compiler wait
    // for the loads right after issuing them
    auto load_rows = [&](uint4* h, int t) {
        const int b = t / tpi, oh0 = (t - b * tpi) * ROWS;
#pragma unroll
        for (int u = 0; u < HR; ++u) {
            const int ih = 2 * oh0 - 1 + u;
            h[u] = *reinterpret_cast<const uint4*>(x + row_off(b, ih < 0 ? 0 : ih));
        }
    };
    float pr[XIN ? 4 : 1][8];  // XIN: this thread's 8 channels' BatchNorm parameters
    // XIN: the rows of tile t become activations (in range: all but row -1); rows 2 oh0 .. are this tile's to write
    auto xform_rows = [&](uint4* h, int t) {
        if constexpr (XIN) {
            const int b = t / tpi, oh0 = (t - b * tpi) * ROWS;
#pragma unroll
            for (int u = 0; u < HR; ++u) {
                const int ih = 2 * oh0 - 1 + u;
                if (ih < 0) continue;
                h[u] = bn_in_apply(h[u], pr);
                if (u > 0 && nh == 0) *reinterpret_cast<uint4*>(xin.a_out + row_off(b, ih)) = h[u];
            }
        }
    };
    auto store_rows = [&](const uint4* h, int buf, int t) {
        const bool top = (t % tpi) == 0;  // the tile's row -1 is the zero padding above the image
#pragma unroll
        for (int u = 0; u < HR; ++u)
            *reinterpret_cast<uint4*>(&Hs[buf * HS + (u * HC + tid / CPP + 1) * PS + (tid % CPP) * 8]) =
                (u == 0 && top) ? make_uint4(0, 0, 0, 0) : h[u];
    };
    int t = blockIdx.x / NSPL, buf = 0;
    if (t < ntiles) load_rows(hr, t);  // in flight during the statistics prologue
    if constexpr (XIN) {
        __shared__ BnInLds<CI> bl;
        bn_in_prologue<CI>(xin, bl);
        const int c0 = (tid % CPP) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            pr[0][k] = bl.prm[c0 + k];
            pr[1][k] = bl.prm[CI + c0 + k];
            pr[2][k] = bl.prm[2 * CI + c0 + k];
            pr[3][k] = bl.prm[3 * CI + c0 + k];
        }
    }
    if (t < ntiles) {
        xform_rows(hr, t);
        store_rows(hr, 0, t);
    }
    __syncthreads();
    const int g8 = (lane >> 4) * 8;
    // statistics (kStatMode 1): each lane's column sums over all its tiles in registers, reduced across the block
    // once at the end (a per-tile LDS reduction cost two barriers per tile)
    constexpr int NS = TR ? TN * 4 : TN;
    double run_s[NS], run_q[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) run_s[j] = run_q[j] = 0.0;
    constexpr int WAVES_M = 4 / WAVES_N;
    __shared__ double sred[EP::kStatMode == 1 ? WAVES_M : 1][2][COB];
    for (; t < ntiles; t += bstep) {
        const int tn = t + bstep;
        // in flight during this tile's MFMAs and stores; unconditional (clamped tile index, the last tile re-reads
        // its own rows): with a conditional load the compiler cannot count the loads younger than the ones it must
        // wait for and waits for all of them (measured with the bias / accumulate loads moved out of the loop:
        // 36.6 -> 27.1 us for the 64 x 64 x 32 -> 64 conv; a second register set two tiles ahead: slower)
        uint4* cur = hr;
        load_rows(cur, min(tn, ntiles - 1));
        f32x4_t acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const bf16* H = Hs + buf * HS;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int kh = tap / 3, kw = tap % 3;
#pragma unroll
            for (int kc = 0; kc < CI / 32; ++kc) {
                bf16x8_t af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int m = wm0 + i * 16 + (lane & 15);
                    const int hrow = 2 * (m / WO) + kh, hcol = 2 * (m % WO) + kw;  // (2oh-1+kh, 2ow-1+kw), col +1
                    af[i] = *reinterpret_cast<const bf16x8_t*>(&H[(hrow * HC + hcol) * PS + kc * 32 + g8]);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = wn0 + j * 16 + (lane & 15);
                    bfr[j] = *reinterpret_cast<const bf16x8_t*>(&Bs[n * KP + tap * CI + kc * 32 + g8]);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)  // TR: operands swapped, channels x pixels (epilogue_tile_t)
                        acc[i][j] = mfma_bf16<TR>(af[i], bfr[j], acc[i][j]);
            }
        }
        double cs[TR ? TN * 4 : TN], cq[TR ? TN * 4 : TN];
        if constexpr (TR)
            epilogue_tile_t<TM, TN, HaloEp<EP>, true>(hep, acc, t * TP + wm0, n0 + wn0, lane, M, CO,
                                              *reinterpret_cast<double(*)[TN][4]>(cs),
                                              *reinterpret_cast<double(*)[TN][4]>(cq));
        else
            epilogue_tile<TM, TN>(hep, acc, t * TP + wm0, n0 + wn0, lane, M, CO, cs, cq);
        if constexpr (EP::kStatMode == 1) {
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                run_s[j] += cs[j];
                run_q[j] += cq[j];
            }
        }
        if constexpr (DB) {
            if (tn < ntiles) {
                xform_rows(cur, tn);
                store_rows(cur, buf ^ 1, tn);
            }
            __syncthreads();
            buf ^= 1;
        } else {
            if (tn < ntiles) xform_rows(cur, tn);
            __syncthreads();  // every wave is done with this tile's halo (and the statistics scratch)
            if (tn < ntiles) store_rows(cur, 0, tn);
            __syncthreads();
        }
    }
    if constexpr (EP::kStatMode == 1) {
        stats_to_lds<TR, TN, COB>(run_s, run_q, &sred[0][0][0], wave / WAVES_N, wn0, lane);
        __syncthreads();
        if (tid < COB) {
            double a = 0.0, q = 0.0;
#pragma unroll
            for (int w = 0; w < WAVES_M; ++w) {
                a += sred[w][0][tid];
                q += sred[w][1][tid];
            }
            const int shard = (int)(blockIdx.x % (unsigned)ep.acc.shards);
            xacc_add_shard(ep.acc, shard, n0 + tid, a);
            xacc_add_shard(ep.acc, shard, CO + n0 + tid, q);
        }
    }
}

// ---- sub-pixel (stride-2 transposed 3x3) conv over LDS halo tiles: Ci = 64,
// Co = 32, low-res width 32, bf16 (the decoder's last sub-pixel layer and the encoder layer-2 data gradient).
// A persistent block keeps the packed weights [32][9 x 64] in LDS and walks 128-pixel low-res tiles (4 rows);
// each tile's 5 input rows (the 4 plus the next, and a zero column right of the image) are staged once, and all
// 4 phases' taps (1 + 2 + 2 + 4) read their fragments from there.
// Template: CI input channels, COB output channels per block (NSPL blocks per tile), WI low-res width, ROWS
// low-res rows per tile (TP = ROWS * WI = 128 pixels), DB: double-buffered halo.  WI * CI / 8 == 256.
// WPE: waves per SIMD the register allocation targets (2: two blocks per CU, with DB = false to fit the LDS)
template <int CI, int COB, int NSPL, int WI, int ROWS, bool DB, class EP, bool TR = true, bool XIN = false, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void subpixel_halo_kernel(const bf16* __restrict__ x, int Hi, int ntiles,
                                                            const bf16* __restrict__ wp, EP ep, int M, BnIn xin) {
    constexpr int HR = ROWS + 1, HC = WI + 1, PS = CI + 8, CPP = CI / 8, TP = ROWS * WI;
    static_assert(WI * CPP == 256 && TP == 128 && (COB == 32 || COB == 16), "halo chunk map / wave tiling");
    constexpr int KP = 9 * CI + 8;                        // weight row: fragment rows on distinct 16-byte slots
    constexpr int HS = HR * HC * PS;
    constexpr int TM = 2, TN = COB / 16, CO = NSPL * COB;  // 4 waves x (32 pixels x COB channels)
    __shared__ __attribute__((aligned(16))) bf16 Bs[COB * KP];
    __shared__ __attribute__((aligned(16))) bf16 Hs[(DB ? 2 : 1) * HS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = wave * 32;
    const int tpi = Hi / ROWS;                            // tiles per image
    const int nh = blockIdx.x % NSPL, n0 = nh * COB;
    const int bstep = gridDim.x / NSPL;
    __shared__ float bsh[COB];  // this block's bias columns
    if (tid < COB) bsh[tid] = n0 + tid < CO ? ep.colbias(n0 + tid) : 0.f;
    for (int c = tid; c < COB * 9 * CPP; c += 256) {      // this block's weight rows
        const int n = c / (9 * CPP), q = c - n * (9 * CPP);
        *reinterpret_cast<uint4*>(&Bs[n * KP + q * 8]) =
            *reinterpret_cast<const uint4*>(wp + (int64_t)(n0 + n) * 9 * CI + q * 8);
    }
    for (int c = tid; c < (DB ? 2 : 1) * HR * CPP; c += 256) {  // the pad column (c = WI) stays zero
        const int bufr = c / CPP, q = c - bufr * CPP;
        *reinterpret_cast<uint4*>(&Hs[(bufr / HR) * HS + ((bufr % HR) * HC + WI) * PS + q * 8]) = make_uint4(0, 0, 0, 0);
    }
    uint4 hr[HR];  // HR rows x 256 chunks / 256 threads
    auto row_off = [&](int b, int ih) { return (((int64_t)b * Hi + ih) * WI + tid / CPP) * CI + (tid % CPP) * 8; };
    auto load_rows = [&](uint4* h, int t) {
        const int b = t / tpi, r0 = (t - b * tpi) * ROWS;
#pragma unroll
        for (int u = 0; u < HR; ++u) {
            const int ih = r0 + u;
            h[u] = *reinterpret_cast<const uint4*>(x + row_off(b, ih < Hi ? ih : Hi - 1));  // zeroed when staged
        }
    };
    float pr[XIN ? 4 : 1][8];  // XIN: this thread's 8 channels' BatchNorm parameters
    // XIN: the rows of tile t inside the image become activations; rows r0 .. r0 + ROWS - 1 are this tile's to write
    auto xform_rows = [&](uint4* h, int t) {
        if constexpr (XIN) {
            const int b = t / tpi, r0 = (t - b * tpi) * ROWS;
#pragma unroll
            for (int u = 0; u < HR; ++u) {
                const int ih = r0 + u;
                if (ih >= Hi) continue;
                h[u] = bn_in_apply(h[u], pr);
                if (u < ROWS && nh == 0) *reinterpret_cast<uint4*>(xin.a_out + row_off(b, ih)) = h[u];
            }
        }
    };
    auto store_rows = [&](const uint4* h, int buf, int t) {
        const bool bottom = (t % tpi) == tpi - 1;  // the tile's last row is the zero padding below the image
#pragma unroll
        for (int u = 0; u < HR; ++u)
            *reinterpret_cast<uint4*>(&Hs[buf * HS + (u * HC + tid / CPP) * PS + (tid % CPP) * 8]) =
                (u == HR - 1 && bottom) ? make_uint4(0, 0, 0, 0) : h[u];
    };
    int t = blockIdx.x / NSPL, buf = 0;
    if (t < ntiles) load_rows(hr, t);  // in flight during the statistics prologue
    if constexpr (XIN) {
        __shared__ BnInLds<CI> bl;
        bn_in_prologue<CI>(xin, bl);
        const int c0 = (tid % CPP) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            pr[0][k] = bl.prm[c0 + k];
            pr[1][k] = bl.prm[CI + c0 + k];
            pr[2][k] = bl.prm[2 * CI + c0 + k];
            pr[3][k] = bl.prm[3 * CI + c0 + k];
        }
    }
    if (t < ntiles) {
        xform_rows(hr, t);
        store_rows(hr, 0, t);
    }
    __syncthreads();
    const int g8 = (lane >> 4) * 8;
    // statistics (kStatMode 1): per-lane column sums over all tiles and phases in registers, one block reduction
    // at the end (conv_s2_halo_kernel; per phase it cost two barriers, eight per tile)
    constexpr int NS = TR ? TN * 4 : TN;
    double run_s[NS], run_q[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) run_s[j] = run_q[j] = 0.0;
    __shared__ double sred[EP::kStatMode == 1 ? 4 : 1][2][COB];
    for (; t < ntiles; t += bstep) {
        const int tn = t + bstep;
        uint4* cur = hr;
        load_rows(cur, min(tn, ntiles - 1));  // unconditional: conv_s2_halo_kernel
        const bf16* H = Hs + buf * HS;
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
            const int py = ph >> 1, px = ph & 1;
            f32x4_t acc[TM][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ty = 0; ty < 2; ++ty) {
                if (ty == 1 && !py) continue;
                const int kh = py ? (ty ? 2 : 0) : 1, dr = (py && ty == 0) ? 1 : 0;
#pragma unroll
                for (int tx = 0; tx < 2; ++tx) {
                    if (tx == 1 && !px) continue;
                    const int kw = px ? (tx ? 2 : 0) : 1, dc = (px && tx == 0) ? 1 : 0;
#pragma unroll
                    for (int kc = 0; kc < CI / 32; ++kc) {
                        bf16x8_t af[TM], bfr[TN];
#pragma unroll
                        for (int i = 0; i < TM; ++i) {
                            const int m = wm0 + i * 16 + (lane & 15);
                            af[i] = *reinterpret_cast<const bf16x8_t*>(
                                &H[((m / WI + dr) * HC + m % WI + dc) * PS + kc * 32 + g8]);
                        }
#pragma unroll
                        for (int j = 0; j < TN; ++j) {
                            const int n = j * 16 + (lane & 15);
                            bfr[j] = *reinterpret_cast<const bf16x8_t*>(&Bs[n * KP + (kh * 3 + kw) * CI + kc * 32 + g8]);
                        }
#pragma unroll
                        for (int i = 0; i < TM; ++i)
#pragma unroll
                            for (int j = 0; j < TN; ++j)  // TR: operands swapped (epilogue_tile_t)
                                acc[i][j] = mfma_bf16<TR>(af[i], bfr[j], acc[i][j]);
                    }
                }
            }
            HaloEp<EP> e;
            static_cast<EP&>(e) = ep;
            e.lb = bsh;
            e.nbase = n0;
            e.set_phase(ph);
            double cs[TR ? TN * 4 : TN], cq[TR ? TN * 4 : TN];
            if constexpr (TR)
                epilogue_tile_t<TM, TN, HaloEp<EP>, true>(e, acc, t * TP + wm0, n0, lane, M, CO,
                                                  *reinterpret_cast<double(*)[TN][4]>(cs),
                                                  *reinterpret_cast<double(*)[TN][4]>(cq));
            else
                epilogue_tile<TM, TN>(e, acc, t * TP + wm0, n0, lane, M, CO, cs, cq);
            if constexpr (EP::kStatMode == 1) {
#pragma unroll
                for (int j = 0; j < NS; ++j) {
                    run_s[j] += cs[j];
                    run_q[j] += cq[j];
                }
            }
        }
        if constexpr (DB) {
            if (tn < ntiles) {
                xform_rows(cur, tn);
                store_rows(cur, buf ^ 1, tn);
            }
            __syncthreads();
            buf ^= 1;
        } else {
            if (tn < ntiles) xform_rows(cur, tn);
            __syncthreads();  // every wave is done with this tile's halo
            if (tn < ntiles) store_rows(cur, 0, tn);
            __syncthreads();
        }
    }
    if constexpr (EP::kStatMode == 1) {
        stats_to_lds<TR, TN, COB>(run_s, run_q, &sred[0][0][0], wave, 0, lane);
        __syncthreads();
        if (tid < COB) {
            const double a = (sred[0][0][tid] + sred[1][0][tid]) + (sred[2][0][tid] + sred[3][0][tid]);
            const double q = (sred[0][1][tid] + sred[1][1][tid]) + (sred[2][1][tid] + sred[3][1][tid]);
            const int shard = (int)(blockIdx.x % (unsigned)ep.acc.shards);
            xacc_add_shard(ep.acc, shard, n0 + tid, a);
            xacc_add_shard(ep.acc, shard, CO + n0 + tid, q);
        }
    }
}


}  // namespace

namespace ops {

static BnIn bn_in_of(const BnInput* xi) {
    BnIn b{};
    if (!xi) return b;
    b.acc = xi->acc; b.R = xi->R; b.mean = xi->mean; b.invstd = xi->invstd; b.rmean = xi->rmean; b.rvar = xi->rvar;
    b.nbt = xi->nbt; b.momentum = xi->momentum; b.eps = xi->eps; b.gamma = xi->gamma; b.beta = xi->beta;
    b.a_out = static_cast<bf16*>(xi->a_out);
    return b;
}
static bool conv_halo_shape(int Ci, int Co, int Wi, int Hi, int& which) {
    which = (Ci == 32 && Co == 64 && Wi == 64 && Hi % 8 == 0) ? 1 : (Ci == 64 && Co == 128 && Wi == 32 && Hi % 8 == 0) ? 2 : 0;
    return which != 0;
}
static bool subpixel_halo_shape(int Ci, int Co, int Wi, int Hi, int& which) {
    which = (Ci == 64 && Co == 32 && Wi == 32 && Hi % 4 == 0) ? 1 : (Ci == 128 && Co == 64 && Wi == 16 && Hi % 8 == 0) ? 2 : 0;
    return which != 0;
}
template <typename T>
bool conv_s2_takes_input_bn(int B, int Hi, int Wi, int Ci, int Co) {
    (void)B;
    int w;
    return std::is_same<T, bf16>::value && conv_halo_shape(Ci, Co, Wi, Hi, w);
}
template <typename T>
bool subpixel_takes_input_bn(int B, int Hi, int Wi, int Ci, int Co) {
    (void)B;
    int w;
    return std::is_same<T, bf16>::value && subpixel_halo_shape(Ci, Co, Wi, Hi, w);
}

template <typename T>
int conv_s2(hipStream_t s, const T* x, int B, int Hi, int Wi, int Ci, const T* wp, const float* bias, int Co, T* y, Ws ws,
            ColStats* st, const BnInput* xin) {
    HLMC_CHECK_ARG(!xin || conv_s2_takes_input_bn<T>(B, Hi, Wi, Ci, Co), "conv_s2: input BatchNorm needs a halo shape");
    if (xin) HLMC_CHECK_ARG(xin->acc.p && xin->acc.ncols == 2 * Ci && xin->a_out && st && st->acc.on(),
                            "conv_s2: input BatchNorm arguments");
    constexpr int V = Vec16<T>::N;
    HLMC_CHECK_ARG(Hi % 2 == 0 && Wi % 2 == 0 && Ci % V == 0, "conv_s2: need even H/W and Ci % 8 (bf16) / 4 (f32)");
    HLMC_CHECK_ARG(aligned16(x) && aligned16(wp), "conv_s2: 16-byte alignment");
    const int Ho = Hi / 2, Wo = Wi / 2, M = B * Ho * Wo, K = 9 * Ci;
    ConvS2Loader<T> al{x, Hi, Wi, Ci, Ho, Wo, M, log2_exact(Ci), FastDiv((uint32_t)Wo), FastDiv((uint32_t)Ho)};
    DenseLoader<T> bl{wp, K, Co, K, true};
    StoreRM<T> ep{y, bias, Co, 0, 0};
    probe::site(probe::kConvS2, 2.0 * M * Co * K,
                (double)sizeof(T) * ((double)B * Hi * Wi * Ci + (double)Co * K + (double)M * Co));
    if constexpr (std::is_same<T, bf16>::value) {
        int which;
        conv_halo_shape(Ci, Co, Wi, Hi, which);
        // (CI, Co, Wi): (32, 64, 64) below; (64, 128, 32) two 64-channel halves per 64-pixel tile, one halo buffer
        // (the weights take half the LDS)
        auto run = [&](auto kern_plain, auto kern_stats, auto kern_xin, int tp, int nspl, int cap = 256) -> int {
            const int ntiles = M / tp;  // whole output rows: tiles stay inside an image
            const int grid = std::min(ntiles * nspl, cap);
            HLMC_PROBE_BEGIN(s);
            if (st && st->acc.on()) {
                WithStats<StoreRM<T>> eps;
                static_cast<StoreRM<T>&>(eps) = ep;
                eps.acc = st->acc;
                if (xin) kern_xin<<<grid, 256, 0, s>>>(x, Hi, ntiles, wp, eps, M, bn_in_of(xin));
                else kern_stats<<<grid, 256, 0, s>>>(x, Hi, ntiles, wp, eps, M, BnIn{});
                st->done = true;
            } else {
                if (st) st->done = false;
                kern_plain<<<grid, 256, 0, s>>>(x, Hi, ntiles, wp, ep, M, BnIn{});
            }
            HLMC_PROBE_END(s);
            HLMC_LAUNCHED();
            return (int)HLMC_OK;
        };
        using StRM = WithStats<StoreRM<T>>;  // per-element epilogue (TR = false), see dispatch_nt
        // (32, 64, 64): 2-row (64-pixel) tiles and one halo buffer: 64 KB (73 KB with the input BatchNorm) and 176
        // VGPRs, two blocks per CU on a 512-block grid.  Measured in the step: forward with the input BatchNorm +
        // statistics 49.6 -> 42.7 us, the decoder data gradient 32.2 -> 31.5 us (4-row tiles, double-buffered, one
        // block per CU before); the same with 4-row tiles and two 32-channel blocks per tile (the halo read twice)
        // lost (50 -> 55 us)
        if (which == 1)
            return run(conv_s2_halo_kernel<32, 64, 1, 32, 2, false, StoreRM<T>, false, false, 2>,
                       conv_s2_halo_kernel<32, 64, 1, 32, 2, false, StRM, false, false, 2>,
                       conv_s2_halo_kernel<32, 64, 1, 32, 2, false, StRM, false, true, 2>, 64, 1, 512);
        if (which == 2)
            return run(conv_s2_halo_kernel<64, 64, 2, 16, 4, false, StoreRM<T>, false>,
                       conv_s2_halo_kernel<64, 64, 2, 16, 4, false, StRM, false>,
                       conv_s2_halo_kernel<64, 64, 2, 16, 4, false, StRM, false, true>, 64, 2);
    }
    return dispatch_nt<T>(s, al, bl, ep, M, Co, K, 1, ws, st);
}

template <typename T>
size_t conv_s2_ws(int B, int Hi, int Wi, int Ci, int Co) {
    return dispatch_nt_ws<T>(B * (Hi / 2) * (Wi / 2), Co, 9 * Ci, 1);
}

template <typename T>
int subpixel(hipStream_t s, const T* x, int B, int Hi, int Wi, int Ci, const T* wp, const float* bias, int Co, T* y, Ws ws,
             ColStats* st, const BnInput* xin) {
    HLMC_CHECK_ARG(!xin || subpixel_takes_input_bn<T>(B, Hi, Wi, Ci, Co), "subpixel: input BatchNorm needs a halo shape");
    if (xin) HLMC_CHECK_ARG(xin->acc.p && xin->acc.ncols == 2 * Ci && xin->a_out && st && st->acc.on(),
                            "subpixel: input BatchNorm arguments");
    constexpr int V = Vec16<T>::N;
    HLMC_CHECK_ARG(Ci % V == 0, "subpixel: Ci % 8 (bf16) / 4 (f32)");
    HLMC_CHECK_ARG(aligned16(x) && aligned16(wp), "subpixel: 16-byte alignment");
    const int M = B * Hi * Wi;
    SubpixelLoader<T> al{x, Hi, Wi, Ci, M, log2_exact(Ci), 0, 0, 0, 0, FastDiv((uint32_t)Wi), FastDiv((uint32_t)Hi)};
    SubpixelWeight<T> bl{wp, Ci, Co, log2_exact(Ci), 0, 0, 0, 0};
    StoreSubpixel<T> ep{y, bias, Hi, Wi, Co, 0, 0, FastDiv((uint32_t)Wi), FastDiv((uint32_t)Hi)};
    // the 4 phases hold 1 + 2 + 2 + 4 = 9 taps: 9 Ci MACs per (low-res pixel, output channel)
    probe::site(probe::kSubpixel, 2.0 * M * Co * 9.0 * Ci,
                (double)sizeof(T) * ((double)M * Ci + 9.0 * Ci * Co + 4.0 * M * Co));
    if constexpr (std::is_same<T, bf16>::value) {
        int which;
        subpixel_halo_shape(Ci, Co, Wi, Hi, which);
        // (nspl, cap): channel splits and grid cap of the statistics / input-BN launches; (nspl_p, cap_p): of the
        // plain launch
        auto run = [&](auto kern_plain, auto kern_stats, auto kern_xin, int nspl, int cap, int nspl_p, int cap_p) -> int {
            const int ntiles = M / 128;  // 128 low-res pixels (whole rows) per tile, inside one image
            HLMC_PROBE_BEGIN(s);
            if (st && st->acc.on()) {
                const int grid = std::min(ntiles * nspl, cap);
                WithStats<StoreSubpixel<T>> eps;
                static_cast<StoreSubpixel<T>&>(eps) = ep;
                eps.acc = st->acc;
                if (xin) kern_xin<<<grid, 256, 0, s>>>(x, Hi, ntiles, wp, eps, M, bn_in_of(xin));
                else kern_stats<<<grid, 256, 0, s>>>(x, Hi, ntiles, wp, eps, M, BnIn{});
                st->done = true;
            } else {
                if (st) st->done = false;
                kern_plain<<<std::min(ntiles * nspl_p, cap_p), 256, 0, s>>>(x, Hi, ntiles, wp, ep, M, BnIn{});
            }
            HLMC_PROBE_END(s);
            HLMC_LAUNCHED();
            return (int)HLMC_OK;
        };
        using StSP = WithStats<StoreSubpixel<T>>;  // per-element epilogue (TR = false), see dispatch_nt
        // Two blocks per CU where a block fits in half the LDS (<= 80 KB) and 256 VGPRs: one halo buffer (no
        // double buffering: the co-resident block covers the extra barrier) and a 512-block grid.  Measured
        // (3 alternating rounds): the 32 x 32 / Ci 64 -> Co 32 shape, all three launches, 129.3k vs 128.0k clips/s
        // (forward 53 -> 46 us, data gradient 72 -> 56 us in the step); the 16 x 16 / Ci 128 -> Co 64 data
        // gradient with 16 channels per block (four blocks per tile, 79 KB) 38 -> 33 us, while its statistics /
        // input-BN forms need 90 KB (one block per CU) and lost 48 -> 68 us; the Ci 32 -> Co 64 conv with two
        // 32-channel blocks per tile (the halo read twice) lost 50 -> 55 / 32 -> 36 us
        if (which == 1)
            return run(subpixel_halo_kernel<64, 32, 1, 32, 4, false, StoreSubpixel<T>, false, false, 2>,
                       subpixel_halo_kernel<64, 32, 1, 32, 4, false, StSP, false, false, 2>,
                       subpixel_halo_kernel<64, 32, 1, 32, 4, false, StSP, false, true, 2>, 1, 512, 1, 512);
        if (which == 2)
            return run(subpixel_halo_kernel<128, 16, 4, 16, 8, false, StoreSubpixel<T>, false, false, 2>,
                       subpixel_halo_kernel<128, 32, 2, 16, 8, false, StSP, false>,
                       subpixel_halo_kernel<128, 32, 2, 16, 8, false, StSP, false, true>, 2, 256, 4, 512);
    }
    return dispatch_nt<T>(s, al, bl, ep, M, Co, 4 * Ci, 4, ws, st);
}
template <typename T>
size_t subpixel_ws(int B, int Hi, int Wi, int Ci, int Co) {
    return dispatch_nt_ws<T>(B * Hi * Wi, Co, 4 * Ci, 4);
}

template <typename T>
int wgrad_s2(hipStream_t s, const T* L, int B, int Hl, int Wl, int M, const T* Xh, int C, float* dW, Ws ws,
             XAcc bias_acc, float* dbias) {
    constexpr int V = Vec16<T>::N;
    HLMC_CHECK_ARG(!dbias || bias_acc.on(), "wgrad_s2: a bias gradient needs its accumulator");
    HLMC_CHECK_ARG(M % V == 0 && C % V == 0, "wgrad_s2: channel counts must be multiples of the vector width");
    const int K = B * Hl * Wl, N = 9 * C;
    StoreWgradConv ep{dW, C, bias_acc, dbias};
    probe::site(probe::kWgradS2, 2.0 * M * N * K,
                (double)sizeof(T) * ((double)K * M + 4.0 * K * C) + 4.0 * M * N);
    // power-of-two sides / channels and operands under 2 GB (every layer of the model): the buffer-descriptor loaders
    const double lbytes = (double)K * M * sizeof(T), xbytes = 4.0 * K * C * sizeof(T);
    const int lh = log2_exact(Hl), lw = log2_exact(Wl), lc = log2_exact(C), lm = log2_exact(M);
    if (lh >= 0 && lw >= 0 && lc >= 0 && lm >= 0 && lbytes < 2147483000.0 && xbytes < 2147483000.0 && aligned16(L) &&
        aligned16(Xh)) {
        KRowDenseP2<T> ll{L, lm, K, M, (uint32_t)lbytes};
        KRowConvS2P2<T> hl{Xh, lh, lw, lc, K, (uint32_t)xbytes};
        return dispatch_tn<T>(s, ll, hl, ep, M, N, K, ws);
    }
    KRowDense<T> ll{L, M, K, M, aligned16(L)};
    KRowConvS2<T> hl{Xh, Hl, Wl, C, K, FastDiv((uint32_t)Wl), FastDiv((uint32_t)Hl)};
    return dispatch_tn<T>(s, ll, hl, ep, M, N, K, ws);
}
template <typename T>
size_t wgrad_s2_ws(int B, int Hl, int Wl, int M, int C) {
    return dispatch_tn_ws<T>(M, 9 * C, B * Hl * Wl);
}

template <typename T, typename OutT>
int linear(hipStream_t s, const T* x, int ldx, int M, int K, const T* w, int ldw, const float* bias, int N, OutT* y,
           int ldy, int act, int accumulate, Ws ws, const OutT* relu_ref) {
    constexpr int V = Vec16<T>::N;
    bool vx = (ldx % V == 0) && aligned16(x);
    bool vw = (ldw % V == 0) && aligned16(w);
    DenseLoader<T> al{x, ldx, M, K, vx};
    DenseLoader<T> bl{w, ldw, N, K, vw};
    StoreRM<OutT> ep{y, bias, ldy, act, accumulate};
    probe::site(probe::kLinear, 2.0 * M * N * K, (double)sizeof(T) * ((double)M * K + (double)N * K) + (double)sizeof(OutT) * M * N);
    if (relu_ref) {
        HLMC_CHECK_ARG(act == 0, "linear: a ReLU-backward mask and a forward activation together");
        StoreReluBwd<OutT> em;
        static_cast<StoreRM<OutT>&>(em) = ep;
        em.relu_ref = relu_ref;
        return dispatch_linear<T>(s, al, bl, em, M, N, K, ws);
    }
    return dispatch_linear<T>(s, al, bl, ep, M, N, K, ws);
}
template <typename T>
size_t linear_ws(int M, int K, int N) {
    return dispatch_linear_ws<T>(M, N, K);
}

// Final epilogue of a dense weight gradient whose H operand carries the ones column: C[n][k < K] -> dW[n][k],
// C[n][K] -> db[n] (the bias gradient, a column sum of dy, from the same GEMM and split-K reduction).
struct StoreWgradBias {
    static constexpr bool kDirectTn = true;  // gemm_tn_kernel may store through it directly (TnDirect)
    float* dW;
    float* db;
    int K;
    struct Row {
        float* r;
        int m;
    };
    __device__ void set_phase(int) {}
    __device__ Row row(int m) const { return Row{dW + (int64_t)m * K, m}; }
    __device__ void store(const Row& rw, int n, float v) const {
        if (n < K) rw.r[n] = v;
        else db[rw.m] = v;
    }
};

template <typename T>
int linear_wgrad(hipStream_t s, const T* dy, int lddy, const T* x, int ldx, int Mb, int N, int K, float* dW, float* db,
                 Ws ws) {
    constexpr int V = Vec16<T>::N;
    KRowDense<T> ll{dy, lddy, Mb, N, (lddy % V == 0) && aligned16(dy), false};
    KRowDense<T> hl{x, ldx, Mb, K, (ldx % V == 0) && aligned16(x), db != nullptr};
    probe::site(probe::kLinearWgrad, 2.0 * N * K * Mb, (double)sizeof(T) * ((double)Mb * N + (double)Mb * K) + 4.0 * N * K);
    if (db) return dispatch_tn<T>(s, ll, hl, StoreWgradBias{dW, db, K}, N, K + 1, Mb, ws);
    StoreRM<float> ep{dW, nullptr, K, 0, 0};
    return dispatch_tn<T>(s, ll, hl, ep, N, K, Mb, ws);
}
template <typename T>
size_t linear_wgrad_ws(int Mb, int N, int K) {  // with or without the bias column
    return std::max(dispatch_tn_ws<T>(N, K, Mb), dispatch_tn_ws<T>(N, K + 1, Mb));
}

#define INST(T)                                                                                                     \
    template int conv_s2<T>(hipStream_t, const T*, int, int, int, int, const T*, const float*, int, T*, Ws,         \
                            ColStats*, const BnInput*);                                                  \
    template bool conv_s2_takes_input_bn<T>(int, int, int, int, int);                                              \
    template bool subpixel_takes_input_bn<T>(int, int, int, int, int);                                             \
    template size_t conv_s2_ws<T>(int, int, int, int, int);                                                        \
    template int subpixel<T>(hipStream_t, const T*, int, int, int, int, const T*, const float*, int, T*, Ws,        \
                             ColStats*, const BnInput*);                                                                             \
    template size_t subpixel_ws<T>(int, int, int, int, int);                                                       \
    template int wgrad_s2<T>(hipStream_t, const T*, int, int, int, int, const T*, int, float*, Ws, XAcc, float*);  \
    template size_t wgrad_s2_ws<T>(int, int, int, int, int);                                                       \
    template int linear<T, T>(hipStream_t, const T*, int, int, int, const T*, int, const float*, int, T*, int, int, \
                              int, Ws, const T*);                                                                  \
    template size_t linear_ws<T>(int, int, int);                                                                   \
    template int linear_wgrad<T>(hipStream_t, const T*, int, const T*, int, int, int, int, float*, float*, Ws);    \
    template size_t linear_wgrad_ws<T>(int, int, int);

INST(float)
INST(bf16)
#undef INST
template int linear<bf16, float>(hipStream_t, const bf16*, int, int, int, const bf16*, int, const float*, int, float*,
                                 int, int, int, Ws, const float*);

}  // namespace ops
}  // namespace hlmc
#ifdef HLMC_TN_TS
extern "C" int hlmc_debug_tn_ts(void* host, int nblocks) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(hlmc::g_tn_ts), (size_t)nblocks * 32, 0, hipMemcpyDeviceToHost);
}
#endif
