"""Per-layer timing of every conv implicit-GEMM launch family of one audio-only train step (bf16, B=256,
128x128): forward, data gradient and weight gradient, via the op-level C-ABI, HIP events on the launch
stream.  Prints us/launch, TF/s and the ideal time max(flops / 2.5 PF, compulsory bytes / 6 TB/s)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402,F401
from hlmc_amd import _lib as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda")
WS = 768 << 20
ws = torch.empty(WS, dtype=torch.uint8, device=dev)
ENC = (1, 32, 64, 128, 256, 512, 512)
DEC = (512, 512, 256, 128, 64, 32, 1)
bf = torch.bfloat16
lib = L.lib()


def timeit(fn, reps=20):
    for _ in range(3):
        L.check(fn())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


rows = []


def report(name, us, flops, nbytes):
    ideal = max(flops / 2.5e15, nbytes / 6e12) * 1e6
    rows.append((name, us, ideal))
    print(f"{name:28s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  ideal {ideal:6.1f} us  ({us / ideal:4.1f}x)", flush=True)


def conv_case(tag, Bn, Hi, Wi, Ci, Co):
    x = torch.randn(Bn, Hi, Wi, Ci, device=dev).to(bf)
    wp = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(bf)
    y = torch.empty(Bn, Hi // 2, Wi // 2, Co, device=dev, dtype=bf)
    fl = 2.0 * Bn * (Hi // 2) * (Wi // 2) * Co * 9 * Ci
    by = 2.0 * (x.numel() + y.numel() + wp.numel())
    us = timeit(lambda: lib.hlmc_op_conv_s2(L.stream(), L.HLMC_BF16, x.data_ptr(), Bn, Hi, Wi, Ci, wp.data_ptr(), None, Co,
                                            y.data_ptr(), ws.data_ptr(), WS))
    report(f"{tag} conv_s2 {Hi}x{Ci}->{Co}", us, fl, by)


def subpixel_case(tag, Bn, Hi, Wi, Ci, Co):
    x = torch.randn(Bn, Hi, Wi, Ci, device=dev).to(bf)
    wp = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(bf)
    y = torch.empty(Bn, 2 * Hi, 2 * Wi, Co, device=dev, dtype=bf)
    fl = 2.0 * Bn * Hi * Wi * Co * 9 * Ci
    by = 2.0 * (x.numel() + y.numel() + wp.numel())
    us = timeit(lambda: lib.hlmc_op_subpixel(L.stream(), L.HLMC_BF16, x.data_ptr(), Bn, Hi, Wi, Ci, wp.data_ptr(), None, Co,
                                             y.data_ptr(), ws.data_ptr(), WS))
    report(f"{tag} subpixel {Hi}x{Ci}->{Co}", us, fl, by)


def wgrad_case(tag, Bn, Hl, Wl, M, C):
    lo = torch.randn(Bn, Hl, Wl, M, device=dev).to(bf)
    xh = torch.randn(Bn, 2 * Hl, 2 * Wl, C, device=dev).to(bf)
    dw = torch.empty(M, C, 3, 3, device=dev)
    fl = 2.0 * M * 9 * C * Bn * Hl * Wl
    by = 2.0 * (lo.numel() + xh.numel()) + 4.0 * dw.numel()
    us = timeit(lambda: lib.hlmc_op_wgrad_s2(L.stream(), L.HLMC_BF16, lo.data_ptr(), Bn, Hl, Wl, M, xh.data_ptr(), C,
                                             dw.data_ptr(), ws.data_ptr(), WS))
    report(f"{tag} wgrad {Hl}x{M}x{C}", us, fl, by)


ONLY = os.environ.get("HLMC_BENCH_ONLY", "")  # e.g. "wgrad": time only that family
if ONLY:
    _keep = {"conv": conv_case, "subpixel": subpixel_case, "wgrad": wgrad_case}
    conv_case, subpixel_case, wgrad_case = [(f if ONLY == k else (lambda *a, **kw: None))
                                            for k, f in (("conv", conv_case), ("subpixel", subpixel_case),
                                                         ("wgrad", wgrad_case))]
h = 128
for l in range(1, 6):
    h //= 2  # input spatial of enc layer l: 128 / 2^l
    ci, co = ENC[l], ENC[l + 1]
    conv_case(f"enc{l + 1} fwd", B, h, h, ci, co)
    wgrad_case(f"enc{l + 1} wgrad", B, h // 2, h // 2, co, ci)
    subpixel_case(f"enc{l + 1} dgrad", B, h // 2, h // 2, co, ci)
h = 2
for l in range(5):
    ci, co = DEC[l], DEC[l + 1]
    subpixel_case(f"dec{l} fwd", B, h, h, ci, co)
    wgrad_case(f"dec{l} wgrad", B, h, h, ci, co)
    conv_case(f"dec{l} dgrad", B, 2 * h, 2 * h, co, ci)
    h *= 2
tot = sum(r[1] for r in rows)
ideal = sum(r[2] for r in rows)
print(f"TOTAL {tot:.1f} us  ideal {ideal:.1f} us")

# single-channel edge convolutions (VALU / HBM kernels): ideal = bytes / 6 TB/s
audio = torch.randn(B, 128, 128, device=dev)
w9 = torch.randn(32, 9, device=dev) * 0.1
bias = torch.zeros(32, device=dev)
y0 = torch.empty(B, 64, 64, 32, device=dev, dtype=bf)
us = timeit(lambda: lib.hlmc_op_conv_c1_s2(L.stream(), L.HLMC_BF16, audio.data_ptr(), B, 128, 128, w9.data_ptr(),
                                           bias.data_ptr(), 32, y0.data_ptr()))
report("enc1 fwd conv_c1_s2 1->32", us, 2.0 * y0.numel() * 9, 4.0 * audio.numel() + 2.0 * y0.numel())
rec = torch.empty(B, 128, 128, device=dev)
us = timeit(lambda: lib.hlmc_op_convT_c1(L.stream(), L.HLMC_BF16, y0.data_ptr(), B, 64, 64, 32, w9.data_ptr(),
                                         bias[:1].data_ptr(), rec.data_ptr()))
report("dec5 fwd convT_c1 32->1", us, 2.0 * y0.numel() * 9, 2.0 * y0.numel() + 4.0 * rec.numel())
dw = torch.empty(32, 9, device=dev)
us = timeit(lambda: lib.hlmc_op_wgrad_c1(L.stream(), L.HLMC_BF16, y0.data_ptr(), B, 64, 64, 32, audio.data_ptr(),
                                         dw.data_ptr(), ws.data_ptr(), WS))
report("enc1 wgrad wgrad_c1 32x9", us, 2.0 * y0.numel() * 9, 2.0 * y0.numel() + 4.0 * audio.numel())
