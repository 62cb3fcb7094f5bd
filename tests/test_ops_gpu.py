"""Op-level parity of the HIP GEMM families vs torch CPU float64 references (NHWC <-> NCHW).

fp32 path (exact-fp32 MFMA): relative L2 error <= 1e-5.  bf16 path: operands rounded to bf16 on
both sides, fp32 accumulation; relative L2 error <= 1e-2 (bf16 output rounding ~4e-3)."""
import ctypes as C
import os

import pytest
import torch
import torch.nn.functional as F

import hlmc_amd
from hlmc_amd import _lib as L

pytestmark = pytest.mark.gpu
DT = {"fp32": (L.HLMC_F32, torch.float32, 1e-5), "bf16": (L.HLMC_BF16, torch.bfloat16, 1e-2)}
WS_BYTES = 512 << 20


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def q(t, dt):  # round to the device dtype and back (reference sees the same operands)
    return t.to(dt).to(torch.float64)


@pytest.fixture(scope="module")
def ws(cuda):
    return torch.empty(WS_BYTES, dtype=torch.uint8, device=cuda)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("B,Hi,Wi,Ci,Co", [(2, 16, 16, 32, 64), (2, 8, 8, 64, 128), (3, 4, 4, 128, 256),
                                          (2, 4, 4, 256, 512), (2, 2, 2, 512, 512), (1, 8, 32, 32, 32),
                                          (5, 4, 8, 64, 64), (3, 16, 64, 32, 64), (2, 64, 64, 32, 64),
                                          (2, 32, 32, 64, 128), (3, 8, 32, 64, 128), (2, 16, 16, 128, 256),
                                          (3, 32, 16, 128, 256)])
def test_conv_s2(cuda, ws, dt, B, Hi, Wi, Ci, Co):
    """(bf16 also covers the shapes of the LDS halo-tile kernels: Ci 32 -> Co 64 at Wi 64 and Ci 64 -> Co 128 at Wi 32;
    fp32 runs the gather GEMM at every shape)"""
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(B * 1000 + Ci)
    x = torch.randn(B, Hi, Wi, Ci, generator=g)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / (3 * Ci ** 0.5)
    b = torch.randn(Co, generator=g)
    ref = F.conv2d(q(x, tdt).permute(0, 3, 1, 2), q(w, tdt), b.double(), stride=2, padding=1).permute(0, 2, 3, 1)
    xd = x.to(cuda, tdt).contiguous()
    wp = w.permute(0, 2, 3, 1).contiguous().to(cuda, tdt)
    y = torch.empty(B, Hi // 2, Wi // 2, Co, dtype=tdt, device=cuda)
    bd = b.to(cuda)
    L.check(L.lib().hlmc_op_conv_s2(L.stream(), code, xd.data_ptr(), B, Hi, Wi, Ci, wp.data_ptr(), bd.data_ptr(), Co,
                                    y.data_ptr(), ws.data_ptr(), WS_BYTES))
    assert rel(y, ref) < tol


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("B,Hi,Wi,Ci,Co", [(2, 2, 2, 512, 512), (2, 4, 4, 512, 256), (2, 8, 8, 256, 128),
                                          (3, 16, 16, 128, 64), (2, 32, 32, 64, 32), (1, 2, 16, 512, 512),
                                          (2, 4, 4, 32, 64), (3, 8, 32, 64, 32), (2, 16, 16, 128, 64),
                                          (3, 8, 16, 128, 64), (2, 16, 8, 256, 128)])
def test_subpixel_convT(cuda, ws, dt, B, Hi, Wi, Ci, Co):
    """(the Ci 64 -> Co 32, 32-wide and Ci 128 -> Co 64, 16-wide shapes run the LDS halo-tile kernels in bf16; fp32
    runs the gather GEMM)"""
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(B * 7 + Ci + Co)
    x = torch.randn(B, Hi, Wi, Ci, generator=g)
    w = torch.randn(Ci, Co, 3, 3, generator=g) / (3 * Ci ** 0.5)   # ConvTranspose2d weight layout
    b = torch.randn(Co, generator=g)
    ref = F.conv_transpose2d(q(x, tdt).permute(0, 3, 1, 2), q(w, tdt), b.double(), stride=2, padding=1,
                             output_padding=1).permute(0, 2, 3, 1)
    xd = x.to(cuda, tdt).contiguous()
    wp = w.permute(1, 2, 3, 0).contiguous().to(cuda, tdt)           # [Co][kh][kw][Ci]
    y = torch.empty(B, 2 * Hi, 2 * Wi, Co, dtype=tdt, device=cuda)
    bd = b.to(cuda)
    L.check(L.lib().hlmc_op_subpixel(L.stream(), code, xd.data_ptr(), B, Hi, Wi, Ci, wp.data_ptr(), bd.data_ptr(), Co,
                                     y.data_ptr(), ws.data_ptr(), WS_BYTES))
    assert rel(y, ref) < tol


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("B,Hl,Wl,M,C", [(2, 8, 8, 64, 32), (2, 4, 4, 128, 64), (2, 2, 2, 512, 256),
                                        (3, 1, 1, 512, 512), (2, 16, 16, 32, 64), (4, 2, 8, 256, 128),
                                        (3, 8, 32, 64, 32), (1, 32, 32, 64, 32)])
def test_wgrad_s2_conv(cuda, ws, dt, B, Hl, Wl, M, C):
    """Conv2d weight gradient: L = dY (low-res, M=Co), Xh = X (high-res, C=Ci), through the weight-gradient TN GEMM
    (the B = 256 bench shapes are test_wgrad_s2_bench_shapes_bf16)."""
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(M + C + B)
    dy = torch.randn(B, Hl, Wl, M, generator=g)
    x = torch.randn(B, 2 * Hl, 2 * Wl, C, generator=g)
    ref = torch.nn.grad.conv2d_weight(q(x, tdt).permute(0, 3, 1, 2), (M, C, 3, 3), q(dy, tdt).permute(0, 3, 1, 2),
                                      stride=2, padding=1)
    dW = torch.empty(M, C, 3, 3, device=cuda)
    dyd, xd = dy.to(cuda, tdt).contiguous(), x.to(cuda, tdt).contiguous()
    L.check(L.lib().hlmc_op_wgrad_s2(L.stream(), code, dyd.data_ptr(), B, Hl, Wl, M, xd.data_ptr(), C, dW.data_ptr(),
                                     ws.data_ptr(), WS_BYTES))
    assert rel(dW, ref) < (1e-5 if dt == "fp32" else 5e-3)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_wgrad_s2_convT(cuda, ws, dt):
    """ConvTranspose2d weight gradient: L = X (low-res input, M=Ci), Xh = dY (high-res, C=Co)."""
    code, tdt, tol = DT[dt]
    B, Hl, Wl, Ci, Co = 2, 4, 4, 128, 64
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, Hl, Wl, Ci, generator=g)
    dy = torch.randn(B, 2 * Hl, 2 * Wl, Co, generator=g)
    w = torch.zeros(Ci, Co, 3, 3, dtype=torch.float64, requires_grad=True)
    out = F.conv_transpose2d(q(x, tdt).permute(0, 3, 1, 2), w, stride=2, padding=1, output_padding=1)
    out.backward(q(dy, tdt).permute(0, 3, 1, 2))
    dW = torch.empty(Ci, Co, 3, 3, device=cuda)
    xd, dyd = x.to(cuda, tdt).contiguous(), dy.to(cuda, tdt).contiguous()
    L.check(L.lib().hlmc_op_wgrad_s2(L.stream(), code, xd.data_ptr(), B, Hl, Wl, Ci, dyd.data_ptr(), Co,
                                     dW.data_ptr(), ws.data_ptr(), WS_BYTES))
    assert rel(dW, w.grad) < (1e-5 if dt == "fp32" else 5e-3)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("M,K,N,ldx,act,acc", [(4, 768, 256, 768, 0, 0), (256, 2048, 1024, 2048, 0, 0),
                                              (5, 370, 128, 376, 1, 0), (256, 2314, 64, 2320, 0, 1),
                                              (33, 128, 1152, 136, 1, 0), (256, 74, 2304, 80, 0, 0),
                                              (2, 1024, 16384, 1152, 0, 0), (2, 1024, 16384, 1152, 0, 1)])
def test_linear(cuda, ws, dt, M, K, N, ldx, act, acc):
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, ldx, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    y0 = torch.randn(M, N, generator=g)
    ref = q(x[:, :K], tdt) @ q(w, tdt).T + b.double()
    if act:
        ref = ref.clamp_min(0)
    if acc:
        ref = ref + q(y0, tdt)
    ldw = ((K + 7) // 8) * 8
    wpad = torch.zeros(N, ldw)
    wpad[:, :K] = w
    y = y0.to(cuda, tdt).contiguous()
    xd, wd, bd = x.to(cuda, tdt).contiguous(), wpad.to(cuda, tdt), b.to(cuda)
    L.check(L.lib().hlmc_op_linear(L.stream(), code, xd.data_ptr(), ldx, M, K, wd.data_ptr(), ldw, bd.data_ptr(), N,
                                   y.data_ptr(), N, act, acc, 0, ws.data_ptr(), WS_BYTES, None))
    assert rel(y, ref) < tol


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("M,K,N,acc", [(256, 2048, 1024, 0), (256, 512, 512, 1), (4, 16384, 1024, 0), (3, 64, 40, 1)])
def test_linear_relu_mask(cuda, ws, dt, M, K, N, acc):
    """Dense data gradient with the ReLU backward of the layer below in the epilogue (engine.cpp lin_bwd)."""
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(M * 7 + K + N)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    y0 = torch.randn(M, N, generator=g)
    act = torch.randn(M, N, generator=g).clamp_min(0)  # post-ReLU activation: ~half the entries exactly 0
    ref = q(x, tdt) @ q(w, tdt).T
    if acc:
        ref = ref + q(y0, tdt)
    ref = torch.where(q(act, tdt) > 0, ref, torch.zeros_like(ref))
    y = y0.to(cuda, tdt).contiguous()
    xd, wd, ad = x.to(cuda, tdt).contiguous(), w.to(cuda, tdt).contiguous(), act.to(cuda, tdt).contiguous()
    L.check(L.lib().hlmc_op_linear(L.stream(), code, xd.data_ptr(), K, M, K, wd.data_ptr(), K, None, N,
                                   y.data_ptr(), N, 0, acc, 0, ws.data_ptr(), WS_BYTES, ad.data_ptr()))
    torch.cuda.synchronize()
    assert rel(y, ref) < tol
    assert bool((y.float().cpu()[act.to(tdt) <= 0] == 0).all())


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("Mb,N,K", [(4, 256, 768), (256, 1024, 2048), (32, 128, 370), (256, 64, 2314),
                                    (7, 2048, 1024)])
def test_linear_wgrad(cuda, ws, dt, Mb, N, K):
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(Mb + N + K)
    ldd, ldx = ((N + 7) // 8) * 8, ((K + 7) // 8) * 8
    dy = torch.randn(Mb, ldd, generator=g)
    x = torch.randn(Mb, ldx, generator=g)
    ref = q(dy[:, :N], tdt).T @ q(x[:, :K], tdt)
    ref_b = q(dy[:, :N], tdt).sum(0)
    dyd, xd = dy.to(cuda, tdt).contiguous(), x.to(cuda, tdt).contiguous()
    for with_bias in (False, True):  # the bias gradient through the GEMM's ones column, and without it
        dW = torch.full((N, K), float("nan"), device=cuda)
        db = torch.full((N,), float("nan"), device=cuda)
        L.check(L.lib().hlmc_op_linear_wgrad(L.stream(), code, dyd.data_ptr(), ldd, xd.data_ptr(), ldx, Mb, N, K,
                                             dW.data_ptr(), db.data_ptr() if with_bias else None, ws.data_ptr(),
                                             WS_BYTES))
        torch.cuda.synchronize()
        assert rel(dW, ref) < (1e-5 if dt == "fp32" else 5e-3)
        if with_bias:
            assert rel(db, ref_b) < 1e-5  # dy x 1 is exact in either dtype; f32 accumulation
        else:
            assert bool(db.isnan().all())


# the bench's 128 x 128 clip and a 128 x 1024 mel row band besides the small case; (16, 128, 128) gives the row-staged
# weight gradient (64-wide layers) two rows per block
@pytest.mark.parametrize("shape", [(3, 16, 32), (2, 128, 128), (2, 32, 64), (1, 16, 1024), (16, 128, 128)])
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_edge_convs(cuda, ws, dt, shape):
    code, tdt, tol = DT[dt]
    g = torch.Generator().manual_seed(9)
    B, H, W = shape
    img = torch.randn(B, H, W, generator=g)
    w1 = torch.randn(32, 1, 3, 3, generator=g) / 3
    b1 = torch.randn(32, generator=g)
    # conv1 forward
    ref = F.conv2d(img.double()[:, None], w1.double(), b1.double(), stride=2, padding=1).permute(0, 2, 3, 1)
    y = torch.empty(B, H // 2, W // 2, 32, dtype=tdt, device=cuda)
    imgd, w1d, b1d = img.to(cuda), w1.to(cuda), b1.to(cuda)
    L.check(L.lib().hlmc_op_conv_c1_s2(L.stream(), code, imgd.data_ptr(), B, H, W, w1d.data_ptr(), b1d.data_ptr(), 32,
                                       y.data_ptr()))
    assert rel(y, ref) < (1e-6 if dt == "fp32" else 1e-2)
    # last convT (32 -> 1)
    a = torch.randn(B, H // 2, W // 2, 32, generator=g)
    wT = torch.randn(32, 1, 3, 3, generator=g) / 10
    bT = torch.randn(1, generator=g)
    refT = F.conv_transpose2d(q(a, tdt).permute(0, 3, 1, 2), wT.double(), bT.double(), stride=2, padding=1,
                              output_padding=1)[:, 0]
    out = torch.empty(B, H, W, device=cuda)
    ad, wTd, bTd = a.to(cuda, tdt).contiguous(), wT.to(cuda), bT.to(cuda)
    L.check(L.lib().hlmc_op_convT_c1(L.stream(), code, ad.data_ptr(), B, H // 2, W // 2, 32, wTd.data_ptr(),
                                     bTd.data_ptr(), out.data_ptr()))
    assert rel(out, refT) < 1e-6
    # weight gradients of both (one-channel high-res side)
    dy = torch.randn(B, H // 2, W // 2, 32, generator=g)
    refw = torch.nn.grad.conv2d_weight(img.double()[:, None], (32, 1, 3, 3), q(dy, tdt).permute(0, 3, 1, 2),
                                       stride=2, padding=1)
    dW = torch.empty(32, 1, 3, 3, device=cuda)
    dyd = dy.to(cuda, tdt).contiguous()
    L.check(L.lib().hlmc_op_wgrad_c1(L.stream(), code, dyd.data_ptr(), B, H // 2, W // 2, 32, imgd.data_ptr(),
                                     dW.data_ptr(), ws.data_ptr(), WS_BYTES))
    assert rel(dW, refw) < 1e-5


@pytest.mark.parametrize("shape", [(1, 7, 64), (3, 11, 64), (1, 5, 64), (2, 9, 24)])
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_wgrad_c1_odd_heights(cuda, ws, dt, shape):
    """hlmc_op_wgrad_c1 at odd low-res heights and B = 1 (Xh is [B][2 Hl][2 Wl] f32, include/hlmc.h): the row-streamed
    kernel of the 64-wide layers (wgrad_c1_rows_kernel: high-res width 2 Wl = 128 and height 2 Hl) and the generic one
    (Wl = 24) against the float64 formula."""
    code, tdt, _ = DT[dt]
    B, Hl, Wl = shape
    g = torch.Generator().manual_seed(Hl * 31 + B)
    img = torch.randn(B, 2 * Hl, 2 * Wl, generator=g)
    dy = torch.randn(B, Hl, Wl, 32, generator=g)
    refw = torch.nn.grad.conv2d_weight(img.double()[:, None], (32, 1, 3, 3), q(dy, tdt).permute(0, 3, 1, 2),
                                       stride=2, padding=1)
    dW = torch.empty(32, 1, 3, 3, device=cuda)
    imgd, dyd = img.to(cuda), dy.to(cuda, tdt).contiguous()
    L.check(L.lib().hlmc_op_wgrad_c1(L.stream(), code, dyd.data_ptr(), B, Hl, Wl, 32, imgd.data_ptr(), dW.data_ptr(),
                                     ws.data_ptr(), WS_BYTES))
    torch.cuda.synchronize()
    assert rel(dW, refw) < 1e-5


@pytest.mark.parametrize("nt", [0, 4 * 384])
def test_loss_sums_backward_fused_equals_separate(cuda, nt):
    """hlmc_loss_sums_backward (one pass) == hlmc_loss_sums + hlmc_loss_backward, bit for bit (same grid, same
    per-element arithmetic and partial order)."""
    g = torch.Generator(device=cuda).manual_seed(11)
    na, nl = 4 * 128 * 128, 4 * 128
    ra, a = torch.randn(na, device=cuda, generator=g), torch.randn(na, device=cuda, generator=g)
    rt, t = torch.randn(max(nt, 1), device=cuda, generator=g), torch.randn(max(nt, 1), device=cuda, generator=g)
    mu, lv = torch.randn(nl, device=cuda, generator=g), torch.randn(nl, device=cuda, generator=g) * 0.3
    coef = torch.tensor([2.0, 0.7, 4.0], device=cuda)
    lib = L.lib()
    ws = torch.empty(int(lib.hlmc_loss_workspace(na, nt, nl)), dtype=torch.uint8, device=cuda)
    outs = []
    for fused in (False, True):
        sums = torch.zeros(3, dtype=torch.float64, device=cuda)
        dra, drt = torch.empty_like(ra), torch.empty_like(rt)
        dmu, dlv = torch.empty_like(mu), torch.empty_like(lv)
        ptr_t = (rt.data_ptr(), t.data_ptr(), drt.data_ptr()) if nt else (None, None, None)
        if fused:
            L.check(lib.hlmc_loss_sums_backward(L.stream(), ra.data_ptr(), a.data_ptr(), na, dra.data_ptr(), ptr_t[0],
                                                ptr_t[1], nt, ptr_t[2], mu.data_ptr(), lv.data_ptr(), nl,
                                                coef.data_ptr(), dmu.data_ptr(), dlv.data_ptr(), sums.data_ptr(),
                                                ws.data_ptr()))
        else:
            L.check(lib.hlmc_loss_sums(L.stream(), ra.data_ptr(), a.data_ptr(), na, ptr_t[0], ptr_t[1], nt,
                                       mu.data_ptr(), lv.data_ptr(), nl, sums.data_ptr(), ws.data_ptr()))
            L.check(lib.hlmc_loss_backward(L.stream(), ra.data_ptr(), a.data_ptr(), na, dra.data_ptr(), ptr_t[0],
                                           ptr_t[1], nt, ptr_t[2], mu.data_ptr(), lv.data_ptr(), nl, coef.data_ptr(),
                                           dmu.data_ptr(), dlv.data_ptr()))
        outs.append((sums.cpu(), dra.cpu(), drt.cpu() if nt else None, dmu.cpu(), dlv.cpu()))
    for x, y in zip(*outs):
        if x is not None:
            assert torch.equal(x, y)
    ref = float(((ra - a).double() ** 2).sum())
    assert abs(float(outs[1][0][0]) - ref) <= 1e-9 * ref


# ---- the EXACT B = 256 layer shapes of the benchmarked step (bench.py: audio-only HybridVAE 128 x 128, bf16), each
# through the dispatch the bench takes: the 32/64-channel layers on the LDS halo-tile kernels, the split-K deep
# layers on the <= 512-block LDS-DMA ring, the rest on the register-staged GEMM; the weight gradients' split-K
# slabs (up to 342 splits) and their grouped reduction.  Encoder forward conv shapes = the decoder's data-gradient
# convs, decoder sub-pixel shapes = the encoder's data gradients, and the ten weight gradients reduce to five
# (M, C, Hl, Wl) shapes.  Reference: CPU float32 on the same bf16-rounded operands (its own error ~1e-6).
#   NT (bf16 output): rel L2 <= 3e-3 (output rounding alone is ~1.1e-3; a dropped K-split of S <= 16 costs >= 6%)
#   weight gradients (fp32 output, fp32 accumulation of bf16 products): rel L2 <= 1e-4 (one dropped slab of the
#   deepest 342-way split costs ~3e-3)
BENCH_CONV = [(64, 64, 32, 64), (32, 32, 64, 128), (16, 16, 128, 256), (8, 8, 256, 512), (4, 4, 512, 512)]
BENCH_SUBPIXEL = [(2, 2, 512, 512), (4, 4, 512, 256), (8, 8, 256, 128), (16, 16, 128, 64), (32, 32, 64, 32)]
BENCH_WGRAD = [(32, 32, 64, 32), (16, 16, 128, 64), (8, 8, 256, 128), (4, 4, 512, 256), (2, 2, 512, 512)]
BB = 256


@pytest.mark.parametrize("Hi,Wi,Ci,Co", BENCH_CONV)
def test_conv_s2_bench_shapes_bf16(cuda, ws, Hi, Wi, Ci, Co):
    g = torch.Generator().manual_seed(Hi * 7 + Ci)
    x = torch.randn(BB, Hi, Wi, Ci, generator=g).to(torch.bfloat16)
    w = (torch.randn(Co, Ci, 3, 3, generator=g) / (3 * Ci ** 0.5)).to(torch.bfloat16)
    b = torch.randn(Co, generator=g)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b, stride=2, padding=1).permute(0, 2, 3, 1)
    xd = x.to(cuda).contiguous()
    wp = w.permute(0, 2, 3, 1).contiguous().to(cuda)
    y = torch.empty(BB, Hi // 2, Wi // 2, Co, dtype=torch.bfloat16, device=cuda)
    bd = b.to(cuda)
    L.check(L.lib().hlmc_op_conv_s2(L.stream(), L.HLMC_BF16, xd.data_ptr(), BB, Hi, Wi, Ci, wp.data_ptr(),
                                    bd.data_ptr(), Co, y.data_ptr(), ws.data_ptr(), WS_BYTES))
    e = rel(y, ref)
    print(f"conv_s2 B={BB} {Hi}x{Wi} {Ci}->{Co}: rel L2 {e:.2e}")
    assert e < 3e-3


@pytest.mark.parametrize("Hi,Wi,Ci,Co", BENCH_SUBPIXEL)
def test_subpixel_bench_shapes_bf16(cuda, ws, Hi, Wi, Ci, Co):
    g = torch.Generator().manual_seed(Hi * 11 + Ci + Co)
    x = torch.randn(BB, Hi, Wi, Ci, generator=g).to(torch.bfloat16)
    w = (torch.randn(Ci, Co, 3, 3, generator=g) / (3 * Ci ** 0.5)).to(torch.bfloat16)
    b = torch.randn(Co, generator=g)
    ref = F.conv_transpose2d(x.float().permute(0, 3, 1, 2), w.float(), b, stride=2, padding=1,
                             output_padding=1).permute(0, 2, 3, 1)
    xd = x.to(cuda).contiguous()
    wp = w.permute(1, 2, 3, 0).contiguous().to(cuda)
    y = torch.empty(BB, 2 * Hi, 2 * Wi, Co, dtype=torch.bfloat16, device=cuda)
    bd = b.to(cuda)
    L.check(L.lib().hlmc_op_subpixel(L.stream(), L.HLMC_BF16, xd.data_ptr(), BB, Hi, Wi, Ci, wp.data_ptr(),
                                     bd.data_ptr(), Co, y.data_ptr(), ws.data_ptr(), WS_BYTES))
    e = rel(y, ref)
    print(f"subpixel B={BB} {Hi}x{Wi} {Ci}->{Co}: rel L2 {e:.2e}")
    assert e < 3e-3


@pytest.mark.parametrize("Hl,Wl,M,C", BENCH_WGRAD)
def test_wgrad_s2_bench_shapes_bf16(cuda, ws, Hl, Wl, M, C):
    g = torch.Generator().manual_seed(Hl * 13 + M + C)
    dy = torch.randn(BB, Hl, Wl, M, generator=g).to(torch.bfloat16)
    x = torch.randn(BB, 2 * Hl, 2 * Wl, C, generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (M, C, 3, 3), dy.double().permute(0, 3, 1, 2),
                                      stride=2, padding=1)
    dW = torch.empty(M, C, 3, 3, device=cuda)
    dyd, xd = dy.to(cuda).contiguous(), x.to(cuda).contiguous()   # held: a freed temporary's block gets reused
    L.check(L.lib().hlmc_op_wgrad_s2(L.stream(), L.HLMC_BF16, dyd.data_ptr(), BB, Hl, Wl, M, xd.data_ptr(), C,
                                     dW.data_ptr(), ws.data_ptr(), WS_BYTES))
    e = rel(dW, ref)
    print(f"wgrad_s2 B={BB} {Hl}x{Wl} M={M} C={C}: rel L2 {e:.2e}")
    assert e < 1e-4


def test_device_randn_matches_philox_restatement(cuda):
    """hlmc_randn (the engine's reparameterisation noise) = oracle/rng_oracle.py's Philox4x32-10 + Box-Muller
    restatement element for element (float32 libm rounding of log / cos / sin: <= 2e-6), any offset, and N(0, 1)."""
    from oracle import rng_oracle
    out = torch.empty(1001, device=cuda)
    for seed, off in [(0, 0), (42, 0), (2 ** 40 + 7, 4096), (123456789, 1 << 33)]:
        L.check(L.lib().hlmc_randn(L.stream(), out.data_ptr(), out.numel(), seed, off))
        ref = torch.from_numpy(rng_oracle.normals(out.numel(), seed, off))
        err = float((out.cpu() - ref).abs().max())
        assert err <= 2e-6 * max(1.0, float(ref.abs().max())), (seed, off, err)
    big = torch.empty(1 << 22, device=cuda)
    L.check(L.lib().hlmc_randn(L.stream(), big.data_ptr(), big.numel(), 7, 0))
    m, sd = float(big.mean()), float(big.std())
    assert abs(m) < 2e-3 and abs(sd - 1) < 2e-3, (m, sd)
    # the engine draws its forward's eps from the net's stream: simple VAE z = mu + eps * exp(lv / 2)
    torch.manual_seed(3)
    vae = hlmc_amd.VAE(370, [128, 64, 32], 32).cuda().eval()
    seed, off = C.c_uint64(), C.c_uint64()
    net = vae._native_net()
    L.check(L.lib().hlmc_net_get_rng(net.h, C.byref(seed), C.byref(off)))
    assert seed.value == torch.initial_seed() and off.value == 0
    x = torch.randn(6, 370, device=cuda)
    with torch.no_grad():
        _, mu, lv, z = vae(x)
    eps = torch.from_numpy(rng_oracle.normals(6 * 32, seed.value, 0)).view(6, 32)
    torch.testing.assert_close(z.cpu(), mu.cpu() + eps * torch.exp(0.5 * lv.cpu()), rtol=1e-5, atol=1e-5)
    L.check(L.lib().hlmc_net_get_rng(net.h, C.byref(seed), C.byref(off)))
    assert off.value == 6 * 32


# The four LDS halo-tile shapes of the B = 256 bench step, through hlmc_op_halo_fwd: the train-mode forward as the
# engine launches it — epilogue statistics accumulated per lane over all of a persistent block's tiles (8 tiles per
# block at these shapes) and, with bn_in, the layer below's BatchNorm + LeakyReLU applied while the input is staged
# (BnInput; src/Convolutional_VAE.py:80-100 encoder, :124-139 decoder).  Checked:
#   * output vs CPU float32 conv of the bf16 operands (the kernel's own activation a_out as input): rel L2 <= 3e-3;
#   * out_sums vs the float64 sums of the kernel's own bf16 output: rel <= 1e-9 (exact accumulator, f64 order only);
#   * bn_in: batch mean / invstd vs float64 statistics of the input <= 1e-6 rel; running statistics as torch's
#     BatchNorm2d(momentum 0.1) updates them; num_batches_tracked 1; a_out = bf16(LeakyReLU((x - mean) * invstd *
#     gamma + beta)) within one bf16 ulp, <= 0.1 % of elements off by that ulp (fp32 contraction order).
HALO = [(0, 64, 64, 32, 64), (0, 32, 32, 64, 128), (1, 32, 32, 64, 32), (1, 16, 16, 128, 64)]


@pytest.mark.parametrize("bn_in", [False, True], ids=["stats", "bn_in+stats"])
@pytest.mark.parametrize("kind,Hi,Wi,Ci,Co", HALO)
def test_halo_fwd_bn_stats_bench_shapes(cuda, kind, Hi, Wi, Ci, Co, bn_in):
    g = torch.Generator().manual_seed(kind * 100 + Hi + Ci + int(bn_in))
    shift, scale = torch.randn(Ci, generator=g) * 0.5, torch.rand(Ci, generator=g) + 0.5
    yin = (torch.randn(BB, Hi, Wi, Ci, generator=g) * scale + shift).to(torch.bfloat16)
    if kind == 0:
        w = (torch.randn(Co, Ci, 3, 3, generator=g) / (3 * Ci ** 0.5)).to(torch.bfloat16)
        wp = w.permute(0, 2, 3, 1).contiguous()
        oshape = (BB, Hi // 2, Wi // 2, Co)
    else:
        w = (torch.randn(Ci, Co, 3, 3, generator=g) / (3 * Ci ** 0.5)).to(torch.bfloat16)
        wp = w.permute(1, 2, 3, 0).contiguous()
        oshape = (BB, 2 * Hi, 2 * Wi, Co)
    b = torch.randn(Co, generator=g) * 0.1
    gamma, beta = 1 + 0.1 * torch.randn(Ci, generator=g), 0.1 * torch.randn(Ci, generator=g)
    rm0, rv0 = 0.1 * torch.randn(Ci, generator=g), 1 + 0.1 * torch.rand(Ci, generator=g)
    d = {k: v.to(cuda).contiguous() for k, v in dict(yin=yin, wp=wp, b=b, gamma=gamma, beta=beta, rm=rm0.clone(),
                                                     rv=rv0.clone()).items()}
    nbt = torch.zeros(1, dtype=torch.int64, device=cuda)
    mean_o, inv_o = torch.empty(Ci, device=cuda), torch.empty(Ci, device=cuda)
    a_out = torch.empty(BB, Hi, Wi, Ci, dtype=torch.bfloat16, device=cuda)
    y = torch.empty(*oshape, dtype=torch.bfloat16, device=cuda)
    sums = torch.empty(2 * Co, dtype=torch.float64, device=cuda)
    wsb = int(L.lib().hlmc_op_halo_workspace(Ci, Co))
    hws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    P = L.ptr
    L.check(L.lib().hlmc_op_halo_fwd(L.stream(), kind, P(d["yin"]), BB, Hi, Wi, Ci, P(d["wp"]), P(d["b"]), Co, P(y),
                                     P(sums), P(d["gamma"]) if bn_in else None, P(d["beta"]) if bn_in else None,
                                     P(d["rm"]), P(d["rv"]), P(nbt), 0.1, 1e-5, P(mean_o), P(inv_o), P(a_out),
                                     P(hws), wsb), "hlmc_op_halo_fwd")
    torch.cuda.synchronize()
    inp = yin
    if bn_in:
        y64 = yin.double().reshape(-1, Ci)
        m64, v64 = y64.mean(0), y64.var(0, unbiased=False)
        e_mean = float(((mean_o.cpu().double() - m64).abs() / (v64.sqrt())).max())
        e_inv = float(((inv_o.cpu().double() - 1 / (v64 + 1e-5).sqrt()).abs() * (v64 + 1e-5).sqrt()).max())
        assert e_mean < 1e-6 and e_inv < 1e-6, (e_mean, e_inv)
        n = y64.shape[0]
        torch.testing.assert_close(d["rm"].cpu().double(), 0.9 * rm0.double() + 0.1 * m64, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(d["rv"].cpu().double(), 0.9 * rv0.double() + 0.1 * v64 * n / (n - 1), rtol=1e-6,
                                   atol=1e-7)
        assert int(nbt.item()) == 1
        z = (yin.float() - mean_o.cpu()) * inv_o.cpu() * gamma + beta
        a_ref = torch.nn.functional.leaky_relu(z, 0.01).to(torch.bfloat16)
        got = a_out.cpu()
        diff = (got.float() - a_ref.float()).abs()
        ulp = a_ref.float().abs().clamp_min(1e-30) * 2.0 ** -7
        frac_off = float((diff > 0).float().mean())
        print(f"halo bn_in {Hi}x{Wi} {Ci}->{Co}: mean {e_mean:.1e} invstd {e_inv:.1e}, a_out off-by-ulp {frac_off:.1e}")
        assert bool((diff <= ulp).all()) and frac_off <= 1e-3
        inp = got
    else:
        assert torch.equal(d["rm"].cpu(), rm0) and int(nbt.item()) == 0   # untouched without gamma
    x = inp.float().permute(0, 3, 1, 2)
    if kind == 0:
        ref = F.conv2d(x, w.float(), b, stride=2, padding=1)
    else:
        ref = F.conv_transpose2d(x, w.float(), b, stride=2, padding=1, output_padding=1)
    ref = ref.permute(0, 2, 3, 1)
    e = rel(y, ref)
    yo = y.cpu().double().reshape(-1, Co)
    s_ref = torch.cat([yo.sum(0), (yo * yo).sum(0)])
    e_s = float(((sums.cpu() - s_ref).abs() / s_ref.abs().clamp_min(1e-300)).max())
    # the first moment can cancel: bound it by the sum of |y| instead
    e_s1 = float(((sums.cpu()[:Co] - s_ref[:Co]).abs() / yo.abs().sum(0)).max())
    e_s2 = float(((sums.cpu()[Co:] - s_ref[Co:]).abs() / s_ref[Co:]).max())
    print(f"halo kind {kind} {Hi}x{Wi} {Ci}->{Co} bn_in={bn_in}: rel L2 {e:.2e}, stats {e_s1:.1e} / {e_s2:.1e}")
    assert e < 3e-3 and e_s1 < 1e-9 and e_s2 < 1e-9


def test_halo_fwd_rejects_other_shapes(cuda):
    ws_ = torch.empty(1 << 20, dtype=torch.uint8, device=cuda)
    st = L.lib().hlmc_op_halo_fwd(L.stream(), 0, ws_.data_ptr(), 4, 8, 8, 256, ws_.data_ptr(), None, 512,
                                  ws_.data_ptr(), ws_.data_ptr(), None, None, None, None, None, 0.1, 1e-5, None, None,
                                  None, ws_.data_ptr(), 1 << 20)
    assert st != 0 and b"halo" in L.lib().hlmc_last_error()


def test_halo_fwd_nan_propagates(cuda):
    """A non-finite value reaching the exact statistics accumulators comes out as NaN (torch's BatchNorm of a diverged
    run), not as finite garbage: one NaN in channel 3 of the pre-BN input -> that channel's batch mean / invstd /
    running statistics NaN, every other input channel finite; the conv outputs next to it are NaN in every channel,
    so every output column sum is NaN."""
    B, Hi, Wi, Ci, Co = 2, 64, 64, 32, 64
    g = torch.Generator().manual_seed(11)
    yin = torch.randn(B, Hi, Wi, Ci, generator=g)
    yin[1, 10, 20, 3] = float("nan")
    yin = yin.to(torch.bfloat16).to(cuda)
    wp = (torch.randn(Co, 3, 3, Ci, generator=g) / 30).to(torch.bfloat16).to(cuda)
    gamma, beta = torch.ones(Ci, device=cuda), torch.zeros(Ci, device=cuda)
    rm, rv = torch.zeros(Ci, device=cuda), torch.ones(Ci, device=cuda)
    nbt = torch.zeros(1, dtype=torch.int64, device=cuda)
    mean_o, inv_o = torch.empty(Ci, device=cuda), torch.empty(Ci, device=cuda)
    a_out = torch.empty(B, Hi, Wi, Ci, dtype=torch.bfloat16, device=cuda)
    y = torch.empty(B, Hi // 2, Wi // 2, Co, dtype=torch.bfloat16, device=cuda)
    sums = torch.empty(2 * Co, dtype=torch.float64, device=cuda)
    wsb = int(L.lib().hlmc_op_halo_workspace(Ci, Co))
    hws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    P = L.ptr
    L.check(L.lib().hlmc_op_halo_fwd(L.stream(), 0, P(yin), B, Hi, Wi, Ci, P(wp), None, Co, P(y), P(sums), P(gamma),
                                     P(beta), P(rm), P(rv), P(nbt), 0.1, 1e-5, P(mean_o), P(inv_o), P(a_out), P(hws), wsb))
    torch.cuda.synchronize()
    m = mean_o.cpu()
    assert torch.isnan(m[3]) and torch.isnan(inv_o.cpu()[3]) and torch.isnan(rm.cpu()[3]) and torch.isnan(rv.cpu()[3])
    others = torch.arange(Ci) != 3
    assert torch.isfinite(m[others]).all() and torch.isfinite(rm.cpu()[others]).all()
    assert torch.isnan(sums.cpu()).all()


# every BatchNorm layer shape of the bench step (B = 256, 128 x 128) plus a small one
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("R,C", [(4 * 8 * 8, 64), (256 * 64 * 64, 32), (256 * 32 * 32, 64), (256 * 16 * 16, 128),
                                 (256 * 8 * 8, 256), (256 * 4 * 4, 512), (256 * 2 * 2, 512), (1500, 64),
                                 (3001, 128), (5000, 256), (2049, 512)])
def test_bn_bwd_op_matches_reference(cuda, dt, R, C):
    """hlmc_op_bn_bwd (the engine's moments + apply passes of train-mode BatchNorm2d + LeakyReLU(0.01) backward,
    src/Convolutional_VAE.py:80-100 backward) vs the float64 formula on the same (quantised) inputs:
    dz = da * lrelu'(xhat gamma + beta), dy = gamma invstd (dz - sum dz / R - xhat sum(dz xhat) / R),
    dgamma = sum dz xhat, dbeta = sum dz, dbias = column sums of the stored dy.  bf16: dy within 1e-2 relative L2
    (its own rounding is 2^-9), the sums within 1e-4; fp32: 1e-5 / 1e-5."""
    code, tdt, _ = DT[dt]
    g = torch.Generator().manual_seed(R % 9973 + C)
    y = torch.randn(R, C, generator=g) * 1.7 + 0.3
    da = torch.randn(R, C, generator=g)
    gamma = 1 + 0.2 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    yq, daq = q(y, tdt), q(da, tdt)
    mean = yq.mean(0).float()
    invstd = (1.0 / torch.sqrt(yq.var(0, unbiased=False) + 1e-5)).float()
    xh = (yq - mean.double()) * invstd.double()
    z = xh * gamma.double() + beta.double()
    dz = daq * torch.where(z > 0, 1.0, 0.01).double()
    s0, sx = dz.sum(0), (dz * xh).sum(0)
    ref = gamma.double() * invstd.double() * (dz - s0 / R - xh * sx / R)
    yd, dad = y.to(cuda, tdt).contiguous(), da.to(cuda, tdt).contiguous()
    dy = torch.empty(R, C, dtype=tdt, device=cuda)
    dg, db, dbias = (torch.empty(C, device=cuda) for _ in range(3))
    wsb = int(L.lib().hlmc_op_bn_bwd_workspace(C))
    bws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    P = L.ptr
    md, ivd, gd, bd = (t.to(cuda) for t in (mean, invstd, gamma, beta))   # kept alive across the async launch
    L.check(L.lib().hlmc_op_bn_bwd(L.stream(), code, P(dad), P(yd), R, C, P(md), P(ivd), P(gd), P(bd), P(dy), P(dg),
                                   P(db), P(dbias), P(bws), wsb))
    torch.cuda.synchronize()
    tol_dy, tol_s = (1e-2, 1e-4) if dt == "bf16" else (1e-5, 1e-5)
    assert rel(dy, ref) < tol_dy
    assert rel(dg, sx) < tol_s and rel(db, s0) < tol_s
    # dbias: the stored dy's column sums (mathematically ~0 here: a bias feeding BatchNorm), checked absolutely
    # against the stored values' float64 sums, at the per-thread float32 accumulation's scale
    dyh = dy.double().cpu()
    err = (dbias.cpu().double() - dyh.sum(0)).abs()
    assert bool((err <= 1e-5 * dyh.abs().sum(0) + 1e-6).all()), float(err.max())


@pytest.mark.parametrize("R,C", [(256 * 8 * 8, 256), (256 * 4 * 4, 512), (5000, 256), (2049, 512)])
def test_bn_bwd_fused_repeatable(cuda, R, C):
    """The one-launch BatchNorm backward of the mid-size layers (kernels.hip bn_bwd_fused_kernel: moments, a grid-wide
    arrival count, then the apply on the rows held in registers).  Its statistics are exact integer sums, so every
    block that folds them after the count must see every block's adds: 24 repeats give bit-identical dgamma / dbeta /
    dy / dbias (a fold that ran ahead of an add would change them), and they agree with the two-pass form
    (hlmc_test_bn_fused(0, -1); its per-thread float32 partials cover other rows, so the totals differ in the last
    bits)."""
    g = torch.Generator().manual_seed(R + C)
    y = (torch.randn(R, C, generator=g) * 1.3 - 0.2).to(cuda, torch.bfloat16)
    da = torch.randn(R, C, generator=g).to(cuda, torch.bfloat16)
    mean = y.float().mean(0)
    invstd = 1.0 / torch.sqrt(y.float().var(0, unbiased=False) + 1e-5)
    gamma = (1 + 0.2 * torch.randn(C, generator=g)).to(cuda)
    beta = (0.1 * torch.randn(C, generator=g)).to(cuda)
    wsb = int(L.lib().hlmc_op_bn_bwd_workspace(C))
    ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    P = L.ptr

    def run():
        dy = torch.empty(R, C, dtype=torch.bfloat16, device=cuda)
        dg, db, dbias = (torch.empty(C, device=cuda) for _ in range(3))
        L.check(L.lib().hlmc_op_bn_bwd(L.stream(), L.HLMC_BF16, P(da), P(y), R, C, P(mean), P(invstd), P(gamma),
                                       P(beta), P(dy), P(dg), P(db), P(dbias), P(ws), wsb))
        return dy, dg, db, dbias

    first = run()
    outs = [run() for _ in range(24)]
    torch.cuda.synchronize()
    for o in outs:
        for a, b in zip(first, o):
            assert torch.equal(a, b)
    L.check(L.lib().hlmc_test_bn_fused(0, -1))
    try:
        two = run()
        torch.cuda.synchronize()
    finally:
        L.check(L.lib().hlmc_test_bn_fused(-1, -1))
    assert rel(first[1], two[1]) < 1e-5 and rel(first[2], two[2]) < 1e-5
    assert rel(first[0], two[0]) < 1e-2
    assert L.lib().hlmc_device_status(0) == 0


@pytest.mark.parametrize("R,C", [(256 * 8 * 8, 256), (256 * 4 * 4, 512)])
def test_bn_bwd_fused_timeout_is_loud(cuda, R, C):
    """bn_bwd_fused_kernel's grid-wide arrival spin is bounded; a block whose spin runs out must not fold partial
    totals into finite values.  With the test hook's spin bound 0 every block but the last to arrive gives up at once:
    those blocks' dgamma / dbeta / dy come out NaN, the device status word's bit 0 is raised, the next C-ABI backward
    call returns HLMC_EDEVICE (checked through Trainer-free hlmc_op_bn_bwd), and clearing the word restores service
    with the default bound (bit-identical to a fresh run)."""
    g = torch.Generator().manual_seed(R - C)
    y = torch.randn(R, C, generator=g).to(cuda, torch.bfloat16)
    da = torch.randn(R, C, generator=g).to(cuda, torch.bfloat16)
    mean = y.float().mean(0)
    invstd = 1.0 / torch.sqrt(y.float().var(0, unbiased=False) + 1e-5)
    gamma, beta = torch.ones(C, device=cuda), torch.zeros(C, device=cuda)
    wsb = int(L.lib().hlmc_op_bn_bwd_workspace(C))
    ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    P = L.ptr

    def launch():
        dy = torch.empty(R, C, dtype=torch.bfloat16, device=cuda)
        dg, db, dbias = (torch.empty(C, device=cuda) for _ in range(3))
        st = L.lib().hlmc_op_bn_bwd(L.stream(), L.HLMC_BF16, P(da), P(y), R, C, P(mean), P(invstd), P(gamma), P(beta),
                                    P(dy), P(dg), P(db), P(dbias), P(ws), wsb)
        return st, dy, dg, db

    assert L.lib().hlmc_device_status(1) == 0
    ok = launch()
    torch.cuda.synchronize()
    L.check(L.lib().hlmc_test_bn_fused(-1, 0))
    try:
        st, dy, dg, db = launch()
        torch.cuda.synchronize()
    finally:
        L.check(L.lib().hlmc_test_bn_fused(-1, -1))
    assert st == 0
    assert L.lib().hlmc_device_status(0) & 1
    nan_rows = (~torch.isfinite(dy.float())).any(1)
    print(f"spin bound 0: {int(nan_rows.sum())} of {R} dy rows NaN, dgamma finite {bool(torch.isfinite(dg).all())}")
    assert int(nan_rows.sum()) > 0
    # every row is either exact (its block saw the full count) or NaN: no finite partial totals
    fin = ~nan_rows
    assert torch.equal(dy[fin], ok[1][fin])
    assert bool(torch.isfinite(dg).all()) == torch.equal(dg, ok[2])
    # the next backward call reports the fault instead of computing
    st2, _, _, _ = launch()
    assert st2 == -4, st2
    assert "BatchNorm backward" in L.lib().hlmc_last_error().decode()
    with pytest.raises(L.HLMCError):
        L.check_device("test")
    assert L.lib().hlmc_device_status(1) & 1 and L.lib().hlmc_device_status(0) == 0
    again = launch()
    torch.cuda.synchronize()
    assert again[0] == 0
    for a, b in zip(ok[1:], again[1:]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("R,C", [(256 * 8 * 8, 256), (256 * 4 * 4, 512)])
def test_bn_bwd_fused_nan_propagates(cuda, R, C):
    """A non-finite gradient in one channel of a one-launch BatchNorm backward layer reaches the exact accumulator as
    its sticky flag (common.hpp kXAccBad) and comes out NaN in that channel's dgamma / dbeta / dy only, as torch's
    backward of a diverged run would; every other channel stays finite."""
    g = torch.Generator().manual_seed(7 + C)
    y = torch.randn(R, C, generator=g).to(cuda, torch.bfloat16)
    da = torch.randn(R, C, generator=g)
    da[R // 3, 5] = float("inf")
    da = da.to(cuda, torch.bfloat16)
    mean = y.float().mean(0)
    invstd = 1.0 / torch.sqrt(y.float().var(0, unbiased=False) + 1e-5)
    gamma, beta = torch.ones(C, device=cuda), torch.zeros(C, device=cuda)
    wsb = int(L.lib().hlmc_op_bn_bwd_workspace(C))
    ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    dy = torch.empty(R, C, dtype=torch.bfloat16, device=cuda)
    dg, db, dbias = (torch.empty(C, device=cuda) for _ in range(3))
    P = L.ptr
    L.check(L.lib().hlmc_op_bn_bwd(L.stream(), L.HLMC_BF16, P(da), P(y), R, C, P(mean), P(invstd), P(gamma), P(beta),
                                   P(dy), P(dg), P(db), P(dbias), P(ws), wsb))
    torch.cuda.synchronize()
    dg, db, dy = dg.cpu(), db.cpu(), dy.float().cpu()
    assert not torch.isfinite(dg[5]) and not torch.isfinite(db[5])
    others = torch.arange(C) != 5
    assert torch.isfinite(dg[others]).all() and torch.isfinite(db[others]).all()
    assert torch.isfinite(dy[:, others]).all() and not torch.isfinite(dy[:, 5]).all()
