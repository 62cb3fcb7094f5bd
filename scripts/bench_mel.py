"""Micro-benchmark of the mel stage alone: hlmc_mel_db over PCM [B, 65024] (128 frames), HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402
from hlmc_amd import _lib as L  # noqa: E402

B, N = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 127 * 512
dev = torch.device("cuda")
pcm = (torch.rand(B, N, device=dev) * 2 - 1) * 0.1
plan = hlmc_amd.features._plan(22050, 2048, 512, 128)
out = torch.empty(B, 128, 128, device=dev)
ws = torch.empty(int(L.lib().hlmc_mel_workspace(plan, B, N)), dtype=torch.uint8, device=dev)
fn = lambda: L.check(L.lib().hlmc_mel_db(plan, L.stream(), pcm.data_ptr(), B, N, 128, 1e-10, 80.0, out.data_ptr(),  # noqa
                                         ws.data_ptr()))
for _ in range(3):
    fn()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
for _ in range(50):
    fn()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 50
print(f"mel_db B={B}: {ms * 1e3:.1f} us/call  {B / ms * 1e3:.0f} clips/s  {B * (N * 4 + 128 * 128 * 4) / ms / 1e6:.1f} GB/s")
