"""Standalone timing of the BatchNorm backward pair (hlmc_op_bn_bwd: moments + apply) at every BatchNorm shape of
the bench step (bf16, B = 256, 128 x 128), HIP events on the launch stream, against the HBM floor of its
algorithmic bytes (moments: read y, da; apply: read y, da, write dy: 10 bytes per element in all)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402,F401
from hlmc_amd import _lib as L  # noqa: E402

dev = torch.device("cuda")
lib = L.lib()
P = L.ptr


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
    return s.elapsed_time(e) / reps * 1e3


tot = 0.0
for (h, C) in [(64, 32), (32, 64), (16, 128), (8, 256), (4, 512), (2, 512)]:
    R = 256 * h * h
    y = torch.randn(R, C, device=dev).to(torch.bfloat16)
    da = torch.randn(R, C, device=dev).to(torch.bfloat16)
    dy = torch.empty_like(y)
    mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    dg, db, dbias = (torch.empty(C, device=dev) for _ in range(3))
    wsb = int(lib.hlmc_op_bn_bwd_workspace(C))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    us = timeit(lambda: lib.hlmc_op_bn_bwd(L.stream(), L.HLMC_BF16, P(da), P(y), R, C, P(mean), P(inv), P(gam), P(bet),
                                           P(dy), P(dg), P(db), P(dbias), P(ws), wsb))
    by = 10.0 * R * C
    tot += us
    print(f"bn_bwd {h:3d}x{h:<3d} C {C:3d}  {us:7.1f} us  {by / us / 1e3:7.1f} GB/s  floor {by / 6.0e12 * 1e6:6.1f} us",
          flush=True)
print(f"TOTAL {tot:.1f} us (x2: encoder + decoder layers of one step)")
