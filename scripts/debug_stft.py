"""Power bins of the STFT kernel (chroma pass A writes them to its workspace) against numpy, with the bin
permutation that explains any mismatch: a diagnostic for the cross-lane FFT's exchange patterns."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402
from hlmc_amd import _lib as L  # noqa: E402
from oracle import mel_oracle as mo  # noqa: E402

N = 127 * 512
rng = np.random.default_rng(1)
y = (rng.standard_normal(N) * 0.1).astype(np.float32)
pcm = torch.from_numpy(y[None]).cuda()
plan = hlmc_amd.features._plan(22050, 2048, 512, 128)
T = 1 + N // 512
ws = torch.zeros(int(L.lib().hlmc_chroma_workspace(plan, 1, N)), dtype=torch.uint8, device="cuda")
out = torch.empty(1, 12, T, device="cuda")
L.check(L.lib().hlmc_chroma_stft(plan, L.stream(), pcm.data_ptr(), 1, N, out.data_ptr(), None, ws.data_ptr()))
torch.cuda.synchronize()
S = ws[: T * 1028 * 4].view(torch.float32).view(T, 1028)[:, :1025].cpu().numpy()
ref = mo.power_spectrogram(y).T  # [T, 1025]
t = T // 2
g, r = S[t], ref[t]
rel = np.abs(g - r) / r.max()
print("frame", t, "max rel err", rel.max(), "bad bins", int((rel > 1e-4).sum()))
order = np.argsort(r)
bad = np.nonzero(rel > 1e-4)[0]
for f in bad[:48]:
    j = order[np.clip(np.searchsorted(r[order], g[f]), 0, 1024)]
    cands = [k for k in range(1025) if abs(r[k] - g[f]) <= 1e-4 * r.max()]
    print(f"bin {f:4d} (lane-part {f % 64:2d} m {f // 64:2d}) gpu {g[f]:.5g} ref {r[f]:.5g} matches ref bins {cands[:4]}")
print("first frame max rel err", (np.abs(S[0] - ref[0]) / ref[0].max()).max(), "last", (np.abs(S[-1] - ref[-1]) / ref[-1].max()).max())
