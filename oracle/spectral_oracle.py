"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy restatement of librosa's handcrafted frame features.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker.  The reference calls (src/1_preprocessing.py:73-91,
src/1_preprocessing_advanced.py:133-137), all with sr=22050, n_fft=2048, hop_length=512:
  * librosa.feature.spectral_centroid  = sum_k freq_k * normalize(S, norm=1, axis=-2)_k,  S = |stft|
  * librosa.feature.spectral_bandwidth = (sum_k S_norm_k |freq_k - centroid|^2) ** 0.5   (p=2, norm=True)
  * librosa.feature.spectral_rolloff   = freq of the first bin with cumsum(S) >= 0.85 * cumsum(S)[-1]
  * librosa.feature.zero_crossing_rate = mean over the frame of signbit changes (edge padding,
                                         |y| <= 1e-10 -> 0, pad=False)
  * librosa.feature.rms                = sqrt(mean(frame**2)) (zero padding)
librosa (>= 0.10, version unpinned by the reference) is NOT installed and the reference ships no values of
these features, so parity against librosa itself is UNPINNED; the restatement is pinned by property tests
(pure tones, silence, known-answer zcr/rms) in tests/test_oracle_cpu.py.
"""
from __future__ import annotations

import numpy as np

from .mel_oracle import HOP, N_FFT, SR, hann_window, n_frames


def magnitude_spectrogram(y: np.ndarray, n_fft: int = N_FFT, hop: int = HOP) -> np.ndarray:
    """np.abs(librosa.stft(y)) for float32 y: float32 [1 + n_fft//2, T] (center=True, zero padding)."""
    y = np.asarray(y, dtype=np.float32)
    yp = np.pad(y, (n_fft // 2, n_fft // 2), mode="constant")
    T = n_frames(y.shape[-1], hop)
    idx = np.arange(n_fft)[None, :] + hop * np.arange(T)[:, None]
    spec = np.fft.rfft(yp[idx].astype(np.float64) * hann_window(n_fft), axis=-1).astype(np.complex64)
    return np.abs(spec).T                                                   # float32 [F, T]


def fft_frequencies(sr: int = SR, n_fft: int = N_FFT) -> np.ndarray:
    return np.fft.rfftfreq(n=n_fft, d=1.0 / sr)


def _normalize_l1(S: np.ndarray) -> np.ndarray:
    """librosa.util.normalize(S, norm=1, axis=-2): columns with sum < float32 tiny stay unnormalised."""
    length = np.sum(np.abs(S), axis=-2, keepdims=True)
    length[length < np.finfo(S.dtype).tiny] = 1.0
    return S / length


def spectral_centroid(y: np.ndarray, sr: int = SR, n_fft: int = N_FFT, hop: int = HOP) -> np.ndarray:
    S = magnitude_spectrogram(y, n_fft, hop)
    freq = fft_frequencies(sr, n_fft)[:, None]
    return np.sum(freq * _normalize_l1(S), axis=-2, keepdims=True)         # float64 [1, T]


def spectral_bandwidth(y: np.ndarray, sr: int = SR, n_fft: int = N_FFT, hop: int = HOP) -> np.ndarray:
    S = magnitude_spectrogram(y, n_fft, hop)
    freq = fft_frequencies(sr, n_fft)[:, None]
    Sn = _normalize_l1(S)
    centroid = np.sum(freq * Sn, axis=-2, keepdims=True)
    dev = np.abs(freq - centroid)
    return np.sum(Sn * dev ** 2, axis=-2, keepdims=True) ** 0.5


def spectral_rolloff(y: np.ndarray, sr: int = SR, n_fft: int = N_FFT, hop: int = HOP,
                     roll_percent: float = 0.85) -> np.ndarray:
    S = magnitude_spectrogram(y, n_fft, hop)
    freq = fft_frequencies(sr, n_fft)[:, None]
    total = np.cumsum(S, axis=-2)
    thr = roll_percent * total[-1:, :]
    ind = np.where(total < thr, np.nan, 1.0)
    return np.nanmin(ind * freq, axis=-2, keepdims=True)


def _frames(yp: np.ndarray, frame_length: int, hop: int, T: int) -> np.ndarray:
    idx = np.arange(frame_length)[:, None] + hop * np.arange(T)[None, :]
    return yp[idx]                                                           # [frame_length, T]


def zero_crossing_rate(y: np.ndarray, frame_length: int = N_FFT, hop: int = HOP) -> np.ndarray:
    y = np.asarray(y, dtype=np.float32)
    T = n_frames(y.shape[-1], hop)
    fr = _frames(np.pad(y, (frame_length // 2, frame_length // 2), mode="edge"), frame_length, hop, T).copy()
    fr[np.abs(fr) <= 1e-10] = 0
    sb = np.signbit(fr)
    cross = np.concatenate([np.zeros((1, T), dtype=bool), sb[1:] != sb[:-1]], axis=0)
    return np.mean(cross, axis=0, keepdims=True)                             # float64 [1, T]


def rms(y: np.ndarray, frame_length: int = N_FFT, hop: int = HOP) -> np.ndarray:
    y = np.asarray(y, dtype=np.float32)
    T = n_frames(y.shape[-1], hop)
    fr = _frames(np.pad(y, (frame_length // 2, frame_length // 2), mode="constant"), frame_length, hop, T)
    return np.sqrt(np.mean(fr ** 2, axis=0, keepdims=True))                  # float32 [1, T]


def extract_spectral_features(y: np.ndarray, sr: int = SR, hop: int = HOP) -> dict:
    """src/1_preprocessing.py:73-91 restated."""
    return {
        "spectral_centroid": spectral_centroid(y, sr, N_FFT, hop),
        "spectral_bandwidth": spectral_bandwidth(y, sr, N_FFT, hop),
        "spectral_rolloff": spectral_rolloff(y, sr, N_FFT, hop),
        "zcr": zero_crossing_rate(y, N_FFT, hop),
        "rms": rms(y, N_FFT, hop),
    }


def spectral_stats(y: np.ndarray, sr: int = SR, hop: int = HOP) -> np.ndarray:
    """src/1_preprocessing.py:123-125: [mean, std] per feature, in dict order -> float64 [10]."""
    out = []
    for feat in extract_spectral_features(y, sr, hop).values():
        out += [np.mean(feat), np.std(feat)]
    return np.asarray(out, dtype=np.float64)
