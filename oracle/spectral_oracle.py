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


# ----------------------------------------------------------------------------- chroma_stft
# librosa >= 0.10 (src/1_preprocessing.py:94-102, src/1_preprocessing_advanced.py:139-141):
#   S = |stft|**2; tuning = estimate_tuning(S=S) (piptrack -> median magnitude -> pitch_tuning);
#   chroma = normalize(filters.chroma(tuning) @ S, norm=inf).
def chroma_filterbank(sr: int = SR, n_fft: int = N_FFT, tuning: float = 0.0, n_chroma: int = 12) -> np.ndarray:
    """librosa.filters.chroma(ctroct=5, octwidth=2, norm=2, base_c=True): float32 [12, 1 + n_fft//2]."""
    frequencies = np.linspace(0, sr, n_fft, endpoint=False)[1:]
    a440 = 440.0 * 2.0 ** (tuning / n_chroma)
    frqbins = n_chroma * np.log2(frequencies / (a440 / 16))
    frqbins = np.concatenate(([frqbins[0] - 1.5 * n_chroma], frqbins))
    binwidthbins = np.concatenate((np.maximum(frqbins[1:] - frqbins[:-1], 1.0), [1]))
    D = np.subtract.outer(frqbins, np.arange(0, n_chroma, dtype="d")).T
    n_chroma2 = np.round(float(n_chroma) / 2)
    D = np.remainder(D + n_chroma2 + 10 * n_chroma, n_chroma) - n_chroma2
    wts = np.exp(-0.5 * (2 * D / np.tile(binwidthbins, (n_chroma, 1))) ** 2)
    length = np.sqrt(np.sum(wts ** 2, axis=0, keepdims=True))
    length[length < np.finfo(np.float64).tiny] = 1.0
    wts = wts / length
    wts *= np.tile(np.exp(-0.5 * (((frqbins / n_chroma - 5.0) / 2) ** 2)), (n_chroma, 1))
    wts = np.roll(wts, -3 * (n_chroma // 12), axis=0)
    return np.ascontiguousarray(wts[:, : int(1 + n_fft / 2)], dtype=np.float32)


def piptrack(S: np.ndarray, sr: int = SR, n_fft: int = N_FFT, fmin: float = 150.0, fmax: float = 4000.0,
             threshold: float = 0.1):
    """librosa.piptrack(S=S) on a float32 power spectrogram [F, T] -> (pitches, mags) float32 [F, T]."""
    S = np.abs(S)
    fmax = min(fmax, float(sr) / 2)
    fft_freqs = fft_frequencies(sr, n_fft)
    F, T = S.shape
    # numba stencils: a = x[1] + x[-1] - 2 * x[0] and b = (x[1] - x[-1]) / 2 promote to float64
    a = (S[2:] + S[:-2]).astype(np.float64) - 2 * S[1:-1].astype(np.float64)
    b = (S[2:] - S[:-2]).astype(np.float64) / 2
    with np.errstate(divide="ignore", invalid="ignore"):
        sh = np.where(np.abs(b) >= np.abs(a), 0.0, -b / a)
    shift = np.zeros_like(S)
    shift[1:-1] = sh.astype(np.float32)
    avg = np.gradient(S, axis=-2)
    dskew = 0.5 * avg * shift
    pitches = np.zeros_like(S)
    mags = np.zeros_like(S)
    freq_mask = ((fmin <= fft_freqs) & (fft_freqs < fmax))[:, None]
    ref_value = threshold * np.max(S, axis=-2, keepdims=True)
    x = S * (S > ref_value)
    lm = np.zeros_like(x, dtype=bool)
    lm[1:-1] = (x[1:-1] > x[:-2]) & (x[1:-1] >= x[2:])
    idx = np.nonzero(freq_mask & lm)
    pitches[idx] = (idx[-2] + shift[idx]) * float(sr) / n_fft
    mags[idx] = S[idx] + dskew[idx]
    return pitches, mags


def estimate_tuning(S: np.ndarray, sr: int = SR, n_fft: int = N_FFT, resolution: float = 0.01,
                    bins_per_octave: int = 12) -> float:
    pitch, mag = piptrack(S, sr, n_fft)
    pitch_mask = pitch > 0
    threshold = np.median(mag[pitch_mask]) if pitch_mask.any() else 0.0
    freqs = pitch[(mag >= threshold) & pitch_mask]
    freqs = freqs[freqs > 0]
    if not np.any(freqs):
        return 0.0
    residual = np.mod(bins_per_octave * np.log2(freqs / (440.0 / 16)), 1.0)
    residual[residual >= 0.5] -= 1.0
    bins = np.linspace(-0.5, 0.5, int(np.ceil(1.0 / resolution)), endpoint=False)
    counts, tuning = np.histogram(residual, bins)
    return float(tuning[np.argmax(counts)])


def chroma_stft(y: np.ndarray, sr: int = SR, n_fft: int = N_FFT, hop: int = HOP):
    """-> (chroma float32 [12, T], tuning)"""
    from .mel_oracle import power_spectrogram
    S = power_spectrogram(y, n_fft, hop)
    tuning = estimate_tuning(S, sr, n_fft)
    raw = np.einsum("cf,ft->ct", chroma_filterbank(sr, n_fft, tuning), S, optimize=True)
    length = np.max(np.abs(raw), axis=0, keepdims=True)
    length[length < np.finfo(np.float32).tiny] = 1.0
    return (raw / length).astype(np.float32), tuning
