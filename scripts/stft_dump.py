"""Dump the power mel spectrogram (hlmc_melspectrogram) of a fixed synthetic batch: used to check that two builds of
libhlmc.so (HLMC_LIB) produce bit-identical STFT / mel output.  usage: python scripts/stft_dump.py OUT.npy"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import hlmc_amd  # noqa: E402
from hlmc_amd import _lib as L  # noqa: E402

dev = torch.device("cuda")
outs = []
for B, n in ((64, bench.N_SAMPLES), (8, 30 * 22050), (3, 50001)):
    pcm = bench.synthetic_pcm(B, n, seed=77 + B, device=dev)
    plan = hlmc_amd.features._plan(22050, 2048, 512, 128)
    T = int(L.lib().hlmc_mel_frames(plan, n))
    out = torch.empty(B, 128, T, device=dev)
    ws = torch.empty(int(L.lib().hlmc_mel_workspace(plan, B, n)), dtype=torch.uint8, device=dev)
    L.check(L.lib().hlmc_melspectrogram(plan, L.stream(), pcm.data_ptr(), B, n, out.data_ptr(), ws.data_ptr()))
    torch.cuda.synchronize()
    outs.append(out.cpu().numpy().ravel())
np.save(sys.argv[1], np.concatenate(outs))
print("dumped", sum(o.size for o in outs))
