"""Run one conv GEMM op repeatedly (for rocprofv3 counter passes):
   python scripts/op_probe.py conv|subpixel|wgrad B Hi Wi Ci Co [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402,F401
from hlmc_amd import _lib as L  # noqa: E402

kind = sys.argv[1]
B, Hi, Wi, Ci, Co = (int(v) for v in sys.argv[2:7])
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 20
dev = torch.device("cuda")
WS = 512 << 20
ws = torch.empty(WS, dtype=torch.uint8, device=dev)
bf = torch.bfloat16
lib = L.lib()
if kind == "conv":
    x = torch.randn(B, Hi, Wi, Ci, device=dev).to(bf)
    wp = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(bf)
    y = torch.empty(B, Hi // 2, Wi // 2, Co, device=dev, dtype=bf)
    fn = lambda: lib.hlmc_op_conv_s2(L.stream(), L.HLMC_BF16, x.data_ptr(), B, Hi, Wi, Ci, wp.data_ptr(), None, Co,  # noqa
                                     y.data_ptr(), ws.data_ptr(), WS)
elif kind == "subpixel":
    x = torch.randn(B, Hi, Wi, Ci, device=dev).to(bf)
    wp = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(bf)
    y = torch.empty(B, 2 * Hi, 2 * Wi, Co, device=dev, dtype=bf)
    fn = lambda: lib.hlmc_op_subpixel(L.stream(), L.HLMC_BF16, x.data_ptr(), B, Hi, Wi, Ci, wp.data_ptr(), None, Co,  # noqa
                                      y.data_ptr(), ws.data_ptr(), WS)
else:  # wgrad: L low-res [B,Hi,Wi,Ci(=M)], Xh [B,2Hi,2Wi,Co(=C)]
    lo = torch.randn(B, Hi, Wi, Ci, device=dev).to(bf)
    xh = torch.randn(B, 2 * Hi, 2 * Wi, Co, device=dev).to(bf)
    dw = torch.empty(Ci, Co, 3, 3, device=dev)
    fn = lambda: lib.hlmc_op_wgrad_s2(L.stream(), L.HLMC_BF16, lo.data_ptr(), B, Hi, Wi, Ci, xh.data_ptr(), Co,  # noqa
                                      dw.data_ptr(), ws.data_ptr(), WS)
for _ in range(reps):
    L.check(fn())
torch.cuda.synchronize()
print("ok")
