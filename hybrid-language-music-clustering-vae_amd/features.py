"""Audio features on the GPU with librosa's call signatures (batched over clips).

Replaces (reference call sites):
  * ``librosa.feature.melspectrogram`` + ``librosa.power_to_db(ref=np.max)`` —
    src/1_preprocessing.py:48-58, src/1_preprocessing_advanced.py:97-114 (``extract_mel_spectrogram``)
  * ``librosa.feature.mfcc(n_mfcc=40)`` — src/1_preprocessing.py:61-70
  * mean/std pooling — src/1_preprocessing.py:115-121, src/1_preprocessing_advanced.py:144-146
  * ``librosa.feature.spectral_centroid / spectral_bandwidth / spectral_rolloff / zero_crossing_rate /
    rms`` and their mean/std pooling — src/1_preprocessing.py:73-91,123-125,
    src/1_preprocessing_advanced.py:133-137,149-151 (``extract_spectral_features``)
  * ``StandardScaler`` — src/1_preprocessing.py:305-311, src/1_preprocessing_advanced.py:376-391
    (per-pixel z-score over [N, 128*T]; the fit can be distributed across ranks)
Inputs may be numpy arrays (results come back as numpy, like librosa) or CUDA tensors (results stay
on the device).  STFT: center=True with zero padding, periodic Hann, n_fft=2048, Slaney mel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L

_PLANS = {}


def _plan(sr, n_fft, hop, n_mels, fmin=0.0, fmax=None):
    key = (int(sr), int(n_fft), int(hop), int(n_mels), float(fmin), float(fmax or 0.0))
    if key not in _PLANS:
        h = C.c_void_p()
        L.check(L.lib().hlmc_mel_plan_create(key[0], key[1], key[2], key[3], key[4], key[5], C.byref(h)),
                "hlmc_mel_plan_create")
        _PLANS[key] = h
    return _PLANS[key]


def _to_dev(y):
    """(2-D float32 CUDA tensor, was_numpy, squeeze)"""
    was_np = not torch.is_tensor(y)
    t = torch.as_tensor(np.asarray(y, dtype=np.float32)) if was_np else y
    squeeze = t.dim() == 1
    t = t.reshape(1, -1) if squeeze else t
    if was_np or not t.is_cuda:
        t = t.to("cuda")
    return t.to(torch.float32).contiguous(), was_np, squeeze


def _ret(t, was_np, squeeze):
    if squeeze:
        t = t[0]
    return t.cpu().numpy() if was_np else t


def mel_filterbank(sr=22050, n_fft=2048, n_mels=128, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels) as built by the library (float32 [n_mels, 1 + n_fft//2])."""
    p = _plan(sr, n_fft, 512, n_mels, fmin, fmax)
    out = np.empty((n_mels, 1 + n_fft // 2), dtype=np.float32)
    L.check(L.lib().hlmc_mel_filterbank(p, out.ctypes.data), "hlmc_mel_filterbank")
    return out


def melspectrogram(y, sr=22050, n_fft=2048, hop_length=512, n_mels=128, fmin=0.0, fmax=None):
    """Power mel spectrogram [..., n_mels, T] of y [..., n_samples]."""
    x, was_np, sq = _to_dev(y)
    p = _plan(sr, n_fft, hop_length, n_mels, fmin, fmax)
    B, n = x.shape
    T = int(L.lib().hlmc_mel_frames(p, n))
    out = torch.empty(B, n_mels, T, device=x.device)
    ws = torch.empty(max(16, 8 * B), dtype=torch.uint8, device=x.device)
    L.check(L.lib().hlmc_melspectrogram(p, L.stream(), x.data_ptr(), B, n, out.data_ptr(), ws.data_ptr()),
            "hlmc_melspectrogram")
    return _ret(out, was_np, sq)


def power_to_db(S, ref=1.0, amin=1e-10, top_db=80.0):
    """librosa.power_to_db for one clip [F, T] or a batch [B, F, T] (ref=np.max -> per-clip maximum)."""
    x = S if torch.is_tensor(S) else torch.as_tensor(np.asarray(S, dtype=np.float32))
    was_np = not torch.is_tensor(S)
    single = x.dim() <= 2
    xb = x.reshape(1, -1) if single else x.reshape(x.shape[0], -1)
    xb = xb.to("cuda").to(torch.float32).contiguous()
    ref_max = callable(ref)
    if ref_max and ref not in (np.max, np.amax, max):
        raise ValueError("callable ref other than np.max is not supported")
    out = torch.empty_like(xb)
    ws = torch.empty(max(16, 8 * xb.shape[0]), dtype=torch.uint8, device=xb.device)
    L.check(L.lib().hlmc_power_to_db(L.stream(), xb.data_ptr(), xb.shape[0], xb.shape[1], int(ref_max),
                                     0.0 if ref_max else float(ref), float(amin),
                                     -1.0 if top_db is None else float(top_db), out.data_ptr(), ws.data_ptr()),
            "hlmc_power_to_db")
    out = out.reshape(x.shape)
    return out.cpu().numpy() if was_np else out


def extract_mel_spectrogram(audio, sr=22050, n_mels=128, n_fft=2048, hop_length=512, fixed_time_steps=None,
                            amin=1e-10, top_db=80.0, scaler=None, out_dtype=torch.float32):
    """src/1_preprocessing_advanced.py:97-114 (fixed_time_steps=1024) / src/1_preprocessing.py:48-58 (None).

    dB reference = maximum over ALL frames of the clip, then crop (or pad with the clip minimum) to
    fixed_time_steps frames.  Batched: audio [B, n] -> [B, n_mels, T'].
    scaler: a fitted StandardScaler over the flattened [n_mels * T'] mel (src/1_preprocessing_advanced.py:376-379);
    its transform is applied inside the dB pass (hlmc_mel_db_zscore, T' % 4 == 0), output in out_dtype."""
    x, was_np, sq = _to_dev(audio)
    p = _plan(sr, n_fft, hop_length, n_mels)
    B, n = x.shape
    T = int(L.lib().hlmc_mel_frames(p, n))
    keep = T if fixed_time_steps is None else int(fixed_time_steps)
    ws = torch.empty(int(L.lib().hlmc_mel_workspace(p, B, n)), dtype=torch.uint8, device=x.device)
    if scaler is not None:
        if scaler.mean_d.numel() != n_mels * keep:
            raise ValueError(f"scaler fitted on {scaler.mean_d.numel()} columns, mel has {n_mels * keep}")
        out = torch.empty(B, n_mels, keep, device=x.device, dtype=out_dtype)
        L.check(L.lib().hlmc_mel_db_zscore(p, L.stream(), x.data_ptr(), B, n, keep, float(amin), float(top_db),
                                           scaler.mean_d.data_ptr(), scaler.scale_d.data_ptr(),
                                           L.HLMC_BF16 if out_dtype == torch.bfloat16 else L.HLMC_F32,
                                           out.data_ptr(), ws.data_ptr()), "hlmc_mel_db_zscore")
        return _ret(out, was_np, sq)
    out = torch.empty(B, n_mels, keep, device=x.device)
    L.check(L.lib().hlmc_mel_db(p, L.stream(), x.data_ptr(), B, n, keep, float(amin), float(top_db),
                                out.data_ptr(), ws.data_ptr()), "hlmc_mel_db")
    return _ret(out, was_np, sq)


def mfcc(y, sr=22050, n_mfcc=20, n_fft=2048, hop_length=512, n_mels=128):
    """librosa.feature.mfcc: power_to_db(melspectrogram, ref=1.0) -> DCT-II ortho -> first n_mfcc rows."""
    x, was_np, sq = _to_dev(y)
    p = _plan(sr, n_fft, hop_length, n_mels)
    B, n = x.shape
    T = int(L.lib().hlmc_mel_frames(p, n))
    out = torch.empty(B, n_mfcc, T, device=x.device)
    ws = torch.empty(int(L.lib().hlmc_mel_workspace(p, B, n)), dtype=torch.uint8, device=x.device)
    L.check(L.lib().hlmc_mfcc(p, L.stream(), x.data_ptr(), B, n, n_mfcc, out.data_ptr(), ws.data_ptr()), "hlmc_mfcc")
    return _ret(out, was_np, sq)


def _spectral_shape(y, sr, n_fft, hop_length, roll_percent):
    x, was_np, sq = _to_dev(y)
    p = _plan(sr, n_fft, hop_length, 128)
    B, n = x.shape
    T = int(L.lib().hlmc_mel_frames(p, n))
    out = torch.empty(B, 3, T, dtype=torch.float64, device=x.device)
    L.check(L.lib().hlmc_spectral_shape(p, L.stream(), x.data_ptr(), B, n, float(roll_percent), out.data_ptr()),
            "hlmc_spectral_shape")
    return out, was_np, sq


def _zcr_rms(y, frame_length, hop_length):
    x, was_np, sq = _to_dev(y)
    p = _plan(22050, frame_length, hop_length, 128)
    B, n = x.shape
    T = int(L.lib().hlmc_mel_frames(p, n))
    zcr = torch.empty(B, 1, T, dtype=torch.float64, device=x.device)
    rms_ = torch.empty(B, 1, T, dtype=torch.float32, device=x.device)
    L.check(L.lib().hlmc_zcr_rms(p, L.stream(), x.data_ptr(), B, n, zcr.data_ptr(), rms_.data_ptr()), "hlmc_zcr_rms")
    return zcr, rms_, was_np, sq


def spectral_centroid(y, sr=22050, n_fft=2048, hop_length=512):
    """librosa.feature.spectral_centroid(y, sr, hop_length) -> float64 [..., 1, T] (Hz)."""
    out, was_np, sq = _spectral_shape(y, sr, n_fft, hop_length, 0.85)
    return _ret(out[:, 0:1], was_np, sq)


def spectral_bandwidth(y, sr=22050, n_fft=2048, hop_length=512):
    """librosa.feature.spectral_bandwidth(y, sr, hop_length) (p=2, norm=True) -> float64 [..., 1, T] (Hz)."""
    out, was_np, sq = _spectral_shape(y, sr, n_fft, hop_length, 0.85)
    return _ret(out[:, 1:2], was_np, sq)


def spectral_rolloff(y, sr=22050, n_fft=2048, hop_length=512, roll_percent=0.85):
    """librosa.feature.spectral_rolloff(y, sr, hop_length, roll_percent) -> float64 [..., 1, T] (Hz)."""
    out, was_np, sq = _spectral_shape(y, sr, n_fft, hop_length, roll_percent)
    return _ret(out[:, 2:3], was_np, sq)


def zero_crossing_rate(y, frame_length=2048, hop_length=512):
    """librosa.feature.zero_crossing_rate(y, frame_length, hop_length) -> float64 [..., 1, T]."""
    zcr, _, was_np, sq = _zcr_rms(y, frame_length, hop_length)
    return _ret(zcr, was_np, sq)


def rms(y=None, frame_length=2048, hop_length=512):
    """librosa.feature.rms(y=y, frame_length, hop_length) -> float32 [..., 1, T]."""
    _, r, was_np, sq = _zcr_rms(y, frame_length, hop_length)
    return _ret(r, was_np, sq)


def chroma_stft(y, sr=22050, n_fft=2048, hop_length=512, return_tuning=False):
    """librosa.feature.chroma_stft(y, sr, n_fft, hop_length) (src/1_preprocessing.py:94-102,
    src/1_preprocessing_advanced.py:139-141): power STFT -> estimate_tuning -> chroma filterbank -> norm=inf.
    float32 [..., 12, T]; with return_tuning also the per-clip tuning estimate (float64 [...])."""
    x, was_np, sq = _to_dev(y)
    p = _plan(sr, n_fft, hop_length, 128)
    B, n = x.shape
    T = int(L.lib().hlmc_mel_frames(p, n))
    out = torch.empty(B, 12, T, dtype=torch.float32, device=x.device)
    tun = torch.empty(B, dtype=torch.float64, device=x.device)
    ws = torch.empty(int(L.lib().hlmc_chroma_workspace(p, B, n)), dtype=torch.uint8, device=x.device)
    L.check(L.lib().hlmc_chroma_stft(p, L.stream(), x.data_ptr(), B, n, out.data_ptr(), tun.data_ptr(),
                                     ws.data_ptr()), "hlmc_chroma_stft")
    del ws
    c = _ret(out, was_np, sq)
    return (c, _ret(tun, was_np, sq)) if return_tuning else c


SPECTRAL_FEATURES = ("spectral_centroid", "spectral_bandwidth", "spectral_rolloff", "zcr", "rms")


def extract_spectral_features(audio, sr=22050, hop_length=512):
    """src/1_preprocessing.py:73-91: dict of the five frame features, two kernel launches for the batch
    (one STFT pass for centroid/bandwidth/rolloff, one time-domain pass for zcr/rms)."""
    shape, was_np, sq = _spectral_shape(audio, sr, 2048, hop_length, 0.85)
    zcr, r, _, _ = _zcr_rms(audio, 2048, hop_length)
    feats = (shape[:, 0:1], shape[:, 1:2], shape[:, 2:3], zcr, r)
    return {k: _ret(v, was_np, sq) for k, v in zip(SPECTRAL_FEATURES, feats)}


def spectral_stats(audio, sr=22050, hop_length=512):
    """The 10 pooled values src/1_preprocessing.py:123-125 appends (per feature: np.mean, np.std over frames),
    float64 [..., 10] in the reference's order."""
    shape, was_np, sq = _spectral_shape(audio, sr, 2048, hop_length, 0.85)
    zcr, r, _, _ = _zcr_rms(audio, 2048, hop_length)
    feats = torch.cat([shape, zcr, r.to(torch.float64)], dim=1)          # [B, 5, T]
    stats = torch.stack([feats.mean(-1), feats.std(-1, unbiased=False)], dim=-1).reshape(feats.shape[0], 10)
    return _ret(stats, was_np, sq)


def mean_std_pool(feat):
    """np.mean / np.std(ddof=0) over the last axis of [..., rows, T] -> [..., 2*rows] (means then stds)."""
    x = feat if torch.is_tensor(feat) else torch.as_tensor(np.asarray(feat, dtype=np.float32))
    was_np = not torch.is_tensor(feat)
    lead = x.shape[:-2]
    rows, cols = x.shape[-2], x.shape[-1]
    xb = x.reshape(-1, cols).to("cuda").to(torch.float32).contiguous()
    mean = torch.empty(xb.shape[0], device=xb.device)
    sd = torch.empty_like(mean)
    L.check(L.lib().hlmc_row_mean_std(L.stream(), xb.data_ptr(), xb.shape[0], cols, mean.data_ptr(), sd.data_ptr()),
            "hlmc_row_mean_std")
    out = torch.cat([mean.reshape(*lead, rows), sd.reshape(*lead, rows)], dim=-1)
    return out.cpu().numpy() if was_np else out


def scaler_finalize(n_total, col_sum, corr, m2):
    """sklearn StandardScaler statistics from the (globally reduced) pass outputs, float64 torch tensors:
    mean = sum / n; var = (M2 - corr^2 / n) / n (the corrected two-pass of _incremental_mean_and_var);
    scale = sqrt(var) with near-constant columns (var <= n eps var + (n mean eps)^2) -> 1."""
    N = float(n_total)
    mean = col_sum / N
    var = (m2 - corr * corr / N) / N
    eps = np.finfo(np.float64).eps
    upper = N * eps * var + (N * mean * eps) ** 2
    scale = torch.sqrt(var)
    scale = torch.where(var <= upper, torch.ones_like(scale), scale)
    return mean, var, scale


class StandardScaler:
    """sklearn.preprocessing.StandardScaler (with_mean, with_std) with float64 accumulators on the GPU.

    ``fit`` = two passes (sum; centred corr + M2), the correction of sklearn's
    _incremental_mean_and_var, ``scale_ = sqrt(var_)`` with near-constant columns -> 1.  With
    ``process_group`` set, each rank passes its shard of rows and the pass outputs are all-reduced
    (SUM) so every rank ends with the global statistics."""

    def __init__(self, process_group=None):
        self.process_group = process_group

    def _allreduce(self, t):
        if self.process_group is not None:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.process_group)
        return t

    def fit(self, X):
        x = X if torch.is_tensor(X) else torch.as_tensor(np.asarray(X, dtype=np.float32))
        x = x.reshape(x.shape[0], -1).to("cuda").to(torch.float32).contiguous()
        n, cols = x.shape
        dev = x.device
        ws = torch.empty(max(16, int(L.lib().hlmc_colstats_workspace(n, cols))), dtype=torch.uint8, device=dev)
        total = self._allreduce(torch.tensor([float(n)], dtype=torch.float64, device=dev))
        s = torch.empty(cols, dtype=torch.float64, device=dev)
        L.check(L.lib().hlmc_colstats_sum(L.stream(), x.data_ptr(), n, cols, s.data_ptr(), ws.data_ptr()))
        self._allreduce(s)
        N = float(total.item())
        mean = s / N
        corr = torch.empty_like(s)
        m2 = torch.empty_like(s)
        L.check(L.lib().hlmc_colstats_centered(L.stream(), x.data_ptr(), n, cols, mean.data_ptr(), corr.data_ptr(),
                                               m2.data_ptr(), ws.data_ptr()))
        self._allreduce(corr)
        self._allreduce(m2)
        mean, var, scale = scaler_finalize(N, s, corr, m2)
        self.mean_d, self.scale_d = mean.contiguous(), scale.contiguous()
        self.mean_ = mean.cpu().numpy()
        self.var_ = var.cpu().numpy()
        self.scale_ = scale.cpu().numpy()
        self.n_samples_seen_ = int(N)
        self.n_features_in_ = cols
        return self

    def transform(self, X, out_dtype=torch.float32):
        was_np = not torch.is_tensor(X)
        x = X if torch.is_tensor(X) else torch.as_tensor(np.asarray(X, dtype=np.float32))
        shape = x.shape
        x = x.reshape(shape[0], -1).to("cuda").to(torch.float32).contiguous()
        out = torch.empty(x.shape, dtype=out_dtype, device=x.device)
        L.check(L.lib().hlmc_zscore_apply(L.stream(), x.data_ptr(), x.shape[0], x.shape[1], self.mean_d.data_ptr(),
                                          self.scale_d.data_ptr(), L.HLMC_BF16 if out_dtype == torch.bfloat16 else L.HLMC_F32,
                                          out.data_ptr()), "hlmc_zscore_apply")
        out = out.reshape(shape)
        return out.cpu().numpy() if was_np else out

    def fit_transform(self, X):
        return self.fit(X).transform(X)
