"""Phase timestamps of the weight-gradient TN kernel (diagnostic build with -DHLMC_TN_TS, hlmc_debug_tn_ts):
   HLMC_LIB=abl/ts/libhlmc.so python scripts/tn_ts.py.  Per layer shape: kernel span, block start spread,
   prologue / K-loop / epilogue durations per block (100 MHz wall clock, 10 ns ticks)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402,F401
from hlmc_amd import _lib as L  # noqa: E402

dev = torch.device("cuda")
WS = 512 << 20
ws = torch.empty(WS, dtype=torch.uint8, device=dev)
lib = L.lib()
bf = torch.bfloat16
buf = np.zeros((8192, 4), dtype=np.uint64)
for tag, (B, Hi, Wi, Ci, Co) in {"enc2": (256, 32, 32, 64, 32), "enc3": (256, 16, 16, 128, 64),
                                 "enc4": (256, 8, 8, 256, 128), "enc5": (256, 4, 4, 512, 256),
                                 "enc6": (256, 2, 2, 512, 512)}.items():
    lo = torch.randn(B, Hi, Wi, Ci, device=dev).to(bf)
    xh = torch.randn(B, 2 * Hi, 2 * Wi, Co, device=dev).to(bf)
    dw = torch.empty(Ci, Co, 3, 3, device=dev)
    fn = lambda: lib.hlmc_op_wgrad_s2(L.stream(), L.HLMC_BF16, lo.data_ptr(), B, Hi, Wi, Ci, xh.data_ptr(), Co,  # noqa
                                      dw.data_ptr(), ws.data_ptr(), WS)
    for _ in range(5):
        L.check(fn())
    torch.cuda.synchronize()
    L.check(fn())
    torch.cuda.synchronize()
    lib.hlmc_debug_tn_ts(buf.ctypes.data_as(ctypes.c_void_p), 8192)
    t = buf.astype(np.int64)
    last = t[:, 0].max()
    sel = t[(t[:, 0] > last - 100000) & (t[:, 3] >= t[:, 0])]
    t0 = sel[:, 0] - sel[:, 0].min()
    pro, loop, epi = sel[:, 1] - sel[:, 0], sel[:, 2] - sel[:, 1], sel[:, 3] - sel[:, 2]
    span = (sel[:, 3].max() - sel[:, 0].min()) / 100
    q = lambda a: "p50 %.2f p90 %.2f max %.2f" % (np.percentile(a, 50) / 100, np.percentile(a, 90) / 100, a.max() / 100)
    print(f"{tag}: blocks {len(sel)} span {span:.2f} us | start {q(t0)} | prologue {q(pro)} | loop {q(loop)} | "
          f"epilogue {q(epi)} (us)", flush=True)
