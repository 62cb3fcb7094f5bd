"""Throughput of the handcrafted frame features (§8f row 2) on the GPU vs the numpy restatement on the host.

Workload: B clips of 30 s at 22050 Hz (src/1_preprocessing.py CONFIG duration=30), the features
extract_spectral_features computes per file (src/1_preprocessing.py:73-91).  Prints one JSON line per kernel
plus the end-to-end batch rate.  Algorithmic bytes: PCM read once (4 n B) + outputs."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import hlmc_amd  # noqa: E402
from hlmc_amd import _lib as L  # noqa: E402
from hlmc_amd.features import _plan  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    B, n = 256, 22050 * 30
    y = torch.randn(B, n, device="cuda") * 0.1
    p = _plan(22050, 2048, 512, 128)
    T = int(L.lib().hlmc_mel_frames(p, n))
    shape = torch.empty(B, 3, T, dtype=torch.float64, device="cuda")
    zcr = torch.empty(B, T, dtype=torch.float64, device="cuda")
    rms = torch.empty(B, T, dtype=torch.float32, device="cuda")
    ms_shape = timed(lambda: L.check(L.lib().hlmc_spectral_shape(p, L.stream(), y.data_ptr(), B, n, 0.85,
                                                                 shape.data_ptr())))
    ms_zr = timed(lambda: L.check(L.lib().hlmc_zcr_rms(p, L.stream(), y.data_ptr(), B, n, zcr.data_ptr(),
                                                       rms.data_ptr())))
    pcm = 4.0 * B * n
    print(json.dumps({"kernel": "spectral_shape (stft_mel_kernel<1>)", "clips": B, "ms": round(ms_shape, 3),
                      "clips_per_s": round(B / ms_shape * 1e3, 1),
                      "pcm_GBps": round(pcm / ms_shape / 1e6, 1)}))
    print(json.dumps({"kernel": "zcr_rms_kernel", "clips": B, "ms": round(ms_zr, 3),
                      "clips_per_s": round(B / ms_zr * 1e3, 1), "pcm_GBps": round(pcm / ms_zr / 1e6, 1),
                      "hbm_frac": round(pcm / ms_zr / 1e6 / 8000.0, 3)}))
    ws = torch.empty(int(L.lib().hlmc_chroma_workspace(p, B, n)), dtype=torch.uint8, device="cuda")
    ch = torch.empty(B, 12, T, device="cuda")
    ms_ch = timed(lambda: L.check(L.lib().hlmc_chroma_stft(p, L.stream(), y.data_ptr(), B, n, ch.data_ptr(), None,
                                                           ws.data_ptr())), reps=5)
    print(json.dumps({"kernel": "chroma_stft (piptrack STFT + tuning + chroma passes)", "clips": B,
                      "ms": round(ms_ch, 3), "clips_per_s": round(B / ms_ch * 1e3, 1)}))
    del ws
    from hlmc_amd import preprocess as P

    def advanced():
        P.handcrafted_features(y, kind="advanced")
        hlmc_amd.extract_mel_spectrogram(y, fixed_time_steps=1024)
    ms_adv = timed(advanced, reps=3)
    print(json.dumps({"path": "processed_data2 per-clip work (mel-dB 128x1024 + 290-d vector)", "clips": B,
                      "ms": round(ms_adv, 3), "clips_per_s": round(B / ms_adv * 1e3, 1)}))
    ms_all = timed(lambda: hlmc_amd.spectral_stats(y), reps=5)
    from oracle import spectral_oracle as SO
    yh = y[:2].cpu().numpy()
    t0 = time.perf_counter()
    for c in yh:
        SO.spectral_stats(c)
    cpu = (time.perf_counter() - t0) / 2
    from oracle import mel_oracle as MO
    t0 = time.perf_counter()
    c = yh[0]
    mel = MO.extract_mel_spectrogram(c)
    SO.spectral_stats(c)
    SO.chroma_stft(c)
    MO.extract_mel_spectrogram(c, fixed_time_steps=1024)
    cpu_adv = time.perf_counter() - t0
    print(json.dumps({"path": "processed_data2 per-clip work, numpy restatement", "cpu_clips_per_s": round(1 / cpu_adv, 2),
                      "cpu_cores": 1, "gpu_speedup": round(B / ms_adv * 1e3 * cpu_adv, 1)}))
    print(json.dumps({"path": "spectral_stats (10 pooled values per clip)", "clips": B, "ms": round(ms_all, 3),
                      "clips_per_s": round(B / ms_all * 1e3, 1),
                      "cpu_oracle_clips_per_s": round(1.0 / cpu, 2), "cpu_cores": 1}))


if __name__ == "__main__":
    main()
