"""Where does the GPU mel power differ from the oracle? (relative error per mel band / frame)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402
from oracle import mel_oracle as MO  # noqa: E402

y = MO.synthetic_pcm(2, 65024, seed=7)
got = hlmc_amd.melspectrogram(y)
ref = MO.melspectrogram(y)
rel = np.abs(got - ref) / np.maximum(ref, 1e-12)
print("shape", got.shape, "max rel", rel.max(), "at", np.unravel_index(rel.argmax(), rel.shape))
print("per-band max rel (first 8 / last 8):", rel.max(axis=(0, 2))[:8], rel.max(axis=(0, 2))[-8:])
print("per-frame max rel (first 4 / last 4):", rel.max(axis=(0, 1))[:4], rel.max(axis=(0, 1))[-4:])
bad = np.argwhere(rel > 1e-3)
print("n bad", len(bad), bad[:10])
fx = np.load("tests/golden/features.npz")
db = hlmc_amd.extract_mel_spectrogram(y)
e = np.abs(db - fx["mel_db"])
print("db max err", e.max(), np.unravel_index(e.argmax(), e.shape), "ref db there", fx["mel_db"][np.unravel_index(e.argmax(), e.shape)])
