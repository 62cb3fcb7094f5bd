"""Batched GPU preprocessing and the ``processed_data1`` / ``processed_data2`` writers.

Replaces the per-file librosa loops and the joblib pool of the reference, keeping its output format:
  * ``src/1_preprocessing.py:105-129`` ``extract_all_features``: the 370-d vector (mel-dB mean/std 256, MFCC(40)
    mean/std 80, five spectral features' mean/std 10, chroma mean/std 24);
  * ``src/1_preprocessing_advanced.py:97-114,120-156`` ``extract_mel_spectrogram`` (128 x 1024) and
    ``extract_flattened_features`` (the 290-d vector: mel-dB 256, spectral 10, chroma 24);
  * ``src/1_preprocessing.py:296-343`` and ``src/1_preprocessing_advanced.py:371-421``: SimpleImputer(mean) +
    StandardScaler on the vectors, the per-pixel StandardScaler over [N, 128*1024] (on the GPU, f64
    accumulators, distributable over ranks), and the saved files (``.npy``, ``metadata.csv``, ``.pkl``).

Clips arrive as decoded float PCM already padded to 30 s (``load_audio_file``, WAV decoding stays outside
the boundary).  Everything per clip runs batched on the GPU.  Two small host steps remain: the imputer and
scaler of the [N, 290|370] vectors, and building the pickled scaler objects.  Both use sklearn itself, so the
pickles are the objects the reference writes.
"""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch

from . import features as F

# src/1_preprocessing.py:21-29 and src/1_preprocessing_advanced.py:28-37
CONFIG_BASIC = {"sample_rate": 22050, "duration": 30, "n_mels": 128, "n_fft": 2048, "hop_length": 512,
                "n_mfcc": 40, "max_samples_per_class": 160}
CONFIG_ADVANCED = {"sample_rate": 22050, "duration": 30, "n_mels": 128, "n_fft": 2048, "hop_length": 512,
                   "fixed_time_steps": 1024, "max_samples_per_class": 200, "lyrics_max_features": 768}


def pad_clip(audio, sr=22050, duration=30):
    """load_audio_file's length rule (src/1_preprocessing.py:146-151): zero-pad to sr * duration samples."""
    a = np.asarray(audio, dtype=np.float32)
    need = sr * duration
    return np.pad(a, (0, need - len(a))) if len(a) < need else a


def handcrafted_features(audio, sr=22050, kind="advanced", hop_length=512):
    """The reference's per-file feature vector for a batch [B, n] of clips, float64 [B, 290] ("advanced",
    src/1_preprocessing_advanced.py:120-156) or [B, 370] ("basic", src/1_preprocessing.py:105-129).
    Order: mel-dB means, mel-dB stds, (MFCC means, MFCC stds), per spectral feature (mean, std), chroma means,
    chroma stds."""
    if kind not in ("advanced", "basic"):
        raise ValueError("kind must be 'advanced' or 'basic'")
    x, was_np, _ = F._to_dev(audio)
    mel_db = F.extract_mel_spectrogram(x, sr=sr, hop_length=hop_length)           # all frames, ref = clip max
    parts = [F.mean_std_pool(mel_db).to(torch.float64)]                            # [B, 256]
    if kind == "basic":
        parts.append(F.mean_std_pool(F.mfcc(x, sr=sr, n_mfcc=40, hop_length=hop_length)).to(torch.float64))
    parts.append(F.spectral_stats(x, sr=sr, hop_length=hop_length))                # [B, 10]
    parts.append(F.mean_std_pool(F.chroma_stft(x, sr=sr, hop_length=hop_length)).to(torch.float64))  # [B, 24]
    out = torch.cat(parts, dim=1)
    return out.cpu().numpy() if was_np else out


def extract_batches(clips, kind="advanced", batch=64, sr=22050, fixed_time_steps=1024):
    """Run the per-clip feature extraction over [N, n] clips in batches of ``batch`` on the GPU.
    Returns (mel_raw float32 [N, 128, fixed_time_steps] or None for "basic", features_raw float64 [N, d])."""
    clips = np.asarray(clips, dtype=np.float32)
    mels, feats = [], []
    for i in range(0, len(clips), batch):
        x = torch.from_numpy(clips[i:i + batch]).cuda()
        if kind == "advanced":
            mels.append(F.extract_mel_spectrogram(x, sr=sr, fixed_time_steps=fixed_time_steps).cpu().numpy())
        feats.append(handcrafted_features(x, sr=sr, kind=kind).cpu().numpy())
    mel_raw = np.concatenate(mels) if mels else None
    return mel_raw, np.concatenate(feats)


def _sklearn_scaler(mean, var, scale, n):
    """An sklearn StandardScaler carrying statistics computed on the GPU (what the reference pickles)."""
    from sklearn.preprocessing import StandardScaler as SkScaler
    s = SkScaler()
    s.mean_ = np.asarray(mean, dtype=np.float64)
    s.var_ = np.asarray(var, dtype=np.float64)
    s.scale_ = np.asarray(scale, dtype=np.float64)
    s.n_samples_seen_ = np.int64(n)
    s.n_features_in_ = int(s.mean_.shape[0])
    return s


def normalize_vectors(features_raw):
    """src/1_preprocessing.py:301-311: inf -> nan, SimpleImputer(mean), StandardScaler (host, [N, d] small)."""
    from sklearn.impute import SimpleImputer
    from sklearn.preprocessing import StandardScaler as SkScaler
    clean = np.where(np.isinf(features_raw), np.nan, features_raw)
    imputer = SimpleImputer(strategy="mean")
    imputed = imputer.fit_transform(clean)
    scaler = SkScaler()
    return scaler.fit_transform(imputed), imputer, scaler


def normalize_mel(mel_raw, process_group=None):
    """src/1_preprocessing_advanced.py:376-382: per-pixel StandardScaler over [N, 128*T] on the GPU.
    Returns (mel_normalized float32 [N, 128, T], sklearn StandardScaler with the fitted statistics)."""
    N = mel_raw.shape[0]
    sc = F.StandardScaler(process_group=process_group)
    flat = torch.from_numpy(np.ascontiguousarray(mel_raw.reshape(N, -1), dtype=np.float32)).cuda()
    norm = sc.fit_transform(flat).cpu().numpy().reshape(mel_raw.shape)
    return norm, _sklearn_scaler(sc.mean_, sc.var_, sc.scale_, sc.n_samples_seen_)


def _metadata_csv(path, metadata, labels):
    import pandas as pd
    df = pd.DataFrame(list(metadata))
    df["label"] = list(labels)
    df.to_csv(path, index=False)


def write_processed_data2(out_dir, mel_raw, features_raw, lyrics_embeddings, labels, metadata, config=None,
                          process_group=None):
    """src/1_preprocessing_advanced.py:371-421.  metadata: per clip dicts with language, genre, filename,
    file_id (advanced.py:301-306); labels: genre strings.  Writes mel_spectrograms_{raw,normalized}.npy,
    features_{raw,normalized}.npy, lyrics_embeddings.npy, labels.npy, metadata.csv, mel_scaler.pkl,
    flat_scaler.pkl, imputer.pkl, config.pkl.  Returns the paths written."""
    os.makedirs(out_dir, exist_ok=True)
    if not (len(mel_raw) == len(features_raw) == len(lyrics_embeddings) == len(labels) == len(metadata)):
        raise ValueError("Mismatch between audio and lyrics samples!")
    mel_norm, mel_scaler = normalize_mel(mel_raw, process_group)
    feat_norm, imputer, flat_scaler = normalize_vectors(features_raw)
    files = {
        "mel_spectrograms_raw.npy": np.asarray(mel_raw),
        "mel_spectrograms_normalized.npy": mel_norm,
        "features_raw.npy": np.asarray(features_raw),
        "features_normalized.npy": feat_norm,
        "lyrics_embeddings.npy": np.asarray(lyrics_embeddings),
        "labels.npy": np.asarray(labels),
    }
    written = []
    for name, arr in files.items():
        np.save(os.path.join(out_dir, name), arr)
        written.append(name)
    _metadata_csv(os.path.join(out_dir, "metadata.csv"), metadata, labels)
    for name, obj in (("mel_scaler.pkl", mel_scaler), ("flat_scaler.pkl", flat_scaler), ("imputer.pkl", imputer),
                      ("config.pkl", dict(config or CONFIG_ADVANCED))):
        with open(os.path.join(out_dir, name), "wb") as f:
            pickle.dump(obj, f)
    return written + ["metadata.csv", "mel_scaler.pkl", "flat_scaler.pkl", "imputer.pkl", "config.pkl"]


def write_processed_data1(out_dir, features_raw, labels, metadata, config=None):
    """src/1_preprocessing.py:296-343: features_{raw,normalized}.npy, labels.npy, metadata.csv (language, genre,
    filename, label), scaler.pkl, imputer.pkl, config.pkl."""
    os.makedirs(out_dir, exist_ok=True)
    feat_norm, imputer, scaler = normalize_vectors(features_raw)
    np.save(os.path.join(out_dir, "features_raw.npy"), np.asarray(features_raw))
    np.save(os.path.join(out_dir, "features_normalized.npy"), feat_norm)
    np.save(os.path.join(out_dir, "labels.npy"), np.array(labels))
    _metadata_csv(os.path.join(out_dir, "metadata.csv"), metadata, labels)
    for name, obj in (("scaler.pkl", scaler), ("imputer.pkl", imputer), ("config.pkl", dict(config or CONFIG_BASIC))):
        with open(os.path.join(out_dir, name), "wb") as f:
            pickle.dump(obj, f)
    return ["features_raw.npy", "features_normalized.npy", "labels.npy", "metadata.csv", "scaler.pkl", "imputer.pkl",
            "config.pkl"]
