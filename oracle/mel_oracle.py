"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy restatement of the librosa feature path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU baseline. The product path never routes through it.

The reference calls librosa at:
  * ``src/1_preprocessing_advanced.py:97-114``  extract_mel_spectrogram (melspectrogram + power_to_db(ref=np.max), crop/pad to 1024)
  * ``src/1_preprocessing.py:48-58``           extract_mel_spectrogram (no crop)
  * ``src/1_preprocessing.py:61-70``           extract_mfcc (librosa.feature.mfcc, n_mfcc=40)
  * ``src/1_preprocessing.py:115-121``         mean/std pooling
librosa is NOT installed here (no network) and its version is unpinned by the reference, so this
restates librosa >= 0.10's published algorithm:
  stft(center=True, pad_mode='constant', window='hann' periodic) -> rfft in float64 of
  (float64 window * float32 frame), stored complex64 -> |X|**2 (float32) -> Slaney mel filterbank
  (float32 [n_mels, 1+n_fft//2]) -> power_to_db(amin=1e-10, top_db=80) -> (mfcc) DCT-II ortho.
Pins: librosa's documented example ``filters.mel(sr=22050, n_fft=2048)[0, 1] ~= 0.016`` (see
tests/test_oracle_cpu.py) plus property tests.  Against librosa itself parity is UNPINNED
(librosa absent; the reference ships no mel values).
"""
from __future__ import annotations

import numpy as np

SR = 22050
N_FFT = 2048
HOP = 512
N_MELS = 128
N_MFCC = 40


# ----------------------------------------------------------------------------- mel filterbank
def hz_to_mel(f):
    """Slaney mel scale (librosa.core.convert.hz_to_mel, htk=False)."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        log_t = f >= min_log_hz
        mels = np.array(mels, dtype=np.float64)
        mels[log_t] = min_log_mel + np.log(f[log_t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(mels):
    mels = np.asanyarray(mels, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if mels.ndim:
        log_t = mels >= min_log_mel
        freqs = np.array(freqs, dtype=np.float64)
        freqs[log_t] = min_log_hz * np.exp(logstep * (mels[log_t] - min_log_mel))
    elif mels >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (mels - min_log_mel))
    return freqs


def mel_filterbank(sr: int = SR, n_fft: int = N_FFT, n_mels: int = N_MELS, fmin: float = 0.0,
                   fmax: float | None = None) -> np.ndarray:
    """librosa.filters.mel(norm='slaney', htk=False, dtype=float32) restated."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def hann_window(n_fft: int = N_FFT) -> np.ndarray:
    """scipy.signal.get_window('hann', n_fft, fftbins=True) (what librosa.filters.get_window calls), restated
    operation for operation so it is bit-identical (tests/test_oracle_cpu.py): scipy 1.15's
    windows.general_cosine(M, [0.5, 0.5], sym=False) extends the window to M + 1 points, evaluates
    w = 0 + 0.5 cos(0 fac) + 0.5 cos(fac) on fac = linspace(-pi, pi, M + 1) and drops the last point."""
    fac = np.linspace(-np.pi, np.pi, n_fft + 1)
    w = np.zeros(n_fft + 1)
    for k, a in enumerate((0.5, 0.5)):
        w += a * np.cos(k * fac)
    return w[:-1]


def n_frames(n_samples: int, hop: int = HOP) -> int:
    """Frames of a center=True STFT (librosa pads n_fft//2 zeros on both sides)."""
    return 1 + n_samples // hop


# ----------------------------------------------------------------------------- spectrogram
def power_spectrogram(y: np.ndarray, n_fft: int = N_FFT, hop: int = HOP) -> np.ndarray:
    """|stft(y)|**2 as librosa computes it for float32 y: float32 [..., 1+n_fft//2, T]."""
    y = np.asarray(y, dtype=np.float32)
    pad = [(0, 0)] * (y.ndim - 1) + [(n_fft // 2, n_fft // 2)]
    yp = np.pad(y, pad, mode="constant")
    T = n_frames(y.shape[-1], hop)
    idx = np.arange(n_fft)[None, :] + hop * np.arange(T)[:, None]          # [T, n_fft]
    frames = yp[..., idx]                                                   # [..., T, n_fft] f32
    win = hann_window(n_fft)
    spec = np.fft.rfft(frames.astype(np.float64) * win, axis=-1).astype(np.complex64)
    mag = np.abs(spec) ** 2                                                 # float32
    return np.swapaxes(mag, -1, -2)                                         # [..., F, T]


def melspectrogram(y: np.ndarray, sr: int = SR, n_fft: int = N_FFT, hop_length: int = HOP,
                   n_mels: int = N_MELS) -> np.ndarray:
    """librosa.feature.melspectrogram(power=2) restated: float32 [..., n_mels, T]."""
    S = power_spectrogram(y, n_fft, hop_length)
    mel = mel_filterbank(sr, n_fft, n_mels)
    return np.einsum("...ft,mf->...mt", S, mel, optimize=True).astype(np.float32)


def power_to_db(S: np.ndarray, ref=np.max, amin: float = 1e-10, top_db: float | None = 80.0) -> np.ndarray:
    """librosa.power_to_db restated (float32 arithmetic, ref over the whole array it is given)."""
    S = np.asarray(S, dtype=np.float32)
    ref_value = ref(S) if callable(ref) else np.abs(ref)
    log_spec = np.float32(10.0) * np.log10(np.maximum(np.float32(amin), S))
    log_spec -= np.float32(10.0) * np.log10(np.maximum(np.float32(amin), np.float32(ref_value)))
    if top_db is not None:
        log_spec = np.maximum(log_spec, log_spec.max() - np.float32(top_db))
    return log_spec.astype(np.float32)


def power_to_db_batched(S: np.ndarray, ref_max: bool = True, top_db: float | None = 80.0) -> np.ndarray:
    """power_to_db applied per clip ([B, M, T]), as the reference calls it once per file."""
    return np.stack([power_to_db(s, ref=np.max if ref_max else 1.0, top_db=top_db) for s in S])


def extract_mel_spectrogram(y: np.ndarray, fixed_time_steps: int | None = None) -> np.ndarray:
    """src/1_preprocessing_advanced.py:97-114 (fixed_time_steps=1024) / src/1_preprocessing.py:48-58 (None).

    The dB reference max is taken over ALL frames before the crop (advanced.py:106-109).  The pad
    branch (advanced.py:111-112) pads with the per-clip minimum.
    """
    mel_db = power_to_db(melspectrogram(y), ref=np.max)
    if fixed_time_steps is not None:
        if mel_db.shape[1] > fixed_time_steps:
            mel_db = mel_db[:, :fixed_time_steps]
        else:
            pad = fixed_time_steps - mel_db.shape[1]
            mel_db = np.pad(mel_db, ((0, 0), (0, pad)), mode="constant", constant_values=mel_db.min())
    return mel_db


def dct_ortho_matrix(n_in: int = N_MELS, n_out: int = N_MFCC) -> np.ndarray:
    """DCT-II, norm='ortho' (scipy.fftpack.dct type 2, what librosa.feature.mfcc calls) as a [n_out, n_in] float64
    matrix: D[k, n] = s_k cos(pi k (2n + 1) / (2 N)), s_0 = sqrt(1/N), s_k = sqrt(2/N).  The phase k (2n + 1) is
    reduced modulo 4N in integers first, so the cosine's argument is below 2 pi and carries one rounding (scipy's
    pocketfft result agrees to 1e-15, tests/test_oracle_cpu.py)."""
    k = np.arange(n_out)[:, None]
    n = np.arange(n_in)[None, :]
    m = (k * (2 * n + 1)) % (4 * n_in)
    D = np.cos(np.pi * m / (2.0 * n_in)) * np.sqrt(2.0 / n_in)
    D[0] = np.sqrt(1.0 / n_in)
    return D


def mfcc(y: np.ndarray, n_mfcc: int = N_MFCC) -> np.ndarray:
    """librosa.feature.mfcc (src/1_preprocessing.py:61-70): power_to_db(ref=1.0) then DCT-II ortho."""
    S = power_to_db(melspectrogram(y), ref=1.0)
    D = dct_ortho_matrix(S.shape[-2], n_mfcc)
    return np.einsum("km,mt->kt", D, S.astype(np.float64)).astype(np.float32)


def mean_std_pool(feat: np.ndarray) -> np.ndarray:
    """np.mean / np.std(ddof=0) over time (src/1_preprocessing.py:117-121): returns [2*rows]."""
    feat = np.asarray(feat, dtype=np.float32)
    return np.concatenate([feat.mean(axis=1), feat.std(axis=1)]).astype(np.float32)


def synthetic_pcm(batch: int, n_samples: int, seed: int = 0) -> np.ndarray:
    """SURVEY §8d synthetic PCM: 8 random sinusoids (50-8000 Hz, amp U(0.02,0.1)) + N(0,0.01^2)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples, dtype=np.float64) / SR
    out = np.empty((batch, n_samples), dtype=np.float32)
    for b in range(batch):
        f = rng.uniform(50.0, 8000.0, size=8)
        a = rng.uniform(0.02, 0.1, size=8)
        ph = rng.uniform(0.0, 2 * np.pi, size=8)
        sig = (a[:, None] * np.sin(2 * np.pi * f[:, None] * t[None, :] + ph[:, None])).sum(0)
        sig += rng.normal(0.0, 0.01, size=n_samples)
        out[b] = np.clip(sig, -1.0, 1.0)
    return out
