"""Deep-layer GEMM yardsticks (bf16, B=256 bench step): our conv_s2 launch vs the same implicit GEMM as a dense
hipBLASLt matmul (torch.matmul on the im2col operand) and MIOpen's channels-last conv2d, so the per-layer target
is a measured vendor number rather than the 2.5 PF peak.  HIP events on the current stream."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402,F401
from hlmc_amd import _lib as L  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
WS = 512 << 20
ws = torch.empty(WS, dtype=torch.uint8, device=dev)
lib = L.lib()


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


B = 256
for (hi, ci, co) in [(16, 128, 256), (8, 256, 512), (4, 512, 512)]:
    ho = hi // 2
    M, N, K = B * ho * ho, co, 9 * ci
    x = torch.randn(B, hi, hi, ci, device=dev).to(bf)
    wp = (torch.randn(co, 3, 3, ci, device=dev) * 0.05).to(bf)
    y = torch.empty(B, ho, ho, co, device=dev, dtype=bf)
    ours = timeit(lambda: lib.hlmc_op_conv_s2(L.stream(), L.HLMC_BF16, x.data_ptr(), B, hi, hi, ci, wp.data_ptr(), None,
                                              co, y.data_ptr(), ws.data_ptr(), WS))
    a = torch.randn(M, K, device=dev).to(bf)
    bt = torch.randn(K, N, device=dev).to(bf)
    mm = timeit(lambda: torch.matmul(a, bt))
    ww = wp.permute(0, 3, 1, 2).contiguous()  # [co][ci][3][3]
    xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wc = ww.contiguous(memory_format=torch.channels_last)
    try:
        cv = timeit(lambda: F.conv2d(xc, wc, stride=2, padding=1))
    except Exception as ex:  # noqa: BLE001
        cv = float("nan")
        print("conv2d failed:", ex)
    fl = 2.0 * M * N * K
    print(f"conv {hi}x{ci}->{co}  M={M} N={N} K={K}: ours {ours:6.1f} us ({fl / ours / 1e6:6.1f} TF/s)  "
          f"hipBLASLt dense {mm:6.1f} us ({fl / mm / 1e6:6.1f} TF/s)  MIOpen conv2d {cv:6.1f} us", flush=True)
    # the weight gradient of the same layer: dW[co][9ci] = dy^T x_im2col over M rows
    g = torch.randn(M, N, device=dev).to(bf)
    mw = timeit(lambda: torch.matmul(g.t(), a))
    ow = torch.empty(co, 9 * ci, device=dev)
    yw = timeit(lambda: lib.hlmc_op_wgrad_s2(L.stream(), L.HLMC_BF16, g.data_ptr(), B, ho, ho, co, x.data_ptr(), ci,
                                             ow.data_ptr(), ws.data_ptr(), WS))
    print(f"   wgrad: ours {yw:6.1f} us ({fl / yw / 1e6:6.1f} TF/s)  hipBLASLt dense {mw:6.1f} us ({fl / mw / 1e6:6.1f} TF/s)",
          flush=True)
