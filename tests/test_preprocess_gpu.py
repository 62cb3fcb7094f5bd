"""Batched preprocessing + processed_data1/2 writers vs the oracle restatements and sklearn.

The per-clip vectors are checked against the oracle composition of the reference's functions
(src/1_preprocessing.py:105-129, src/1_preprocessing_advanced.py:120-156); parity vs librosa itself is
unpinned (librosa absent).  Tolerances: mel-dB pooled values atol 5e-3 dB (the STFT runs in float32 on the GPU),
spectral / chroma pooled values as in tests/test_spectral_gpu.py."""
import os
import pickle

import numpy as np
import pandas as pd
import pytest
from sklearn.preprocessing import StandardScaler as SkScaler

import hlmc_amd
from hlmc_amd import preprocess as P
from oracle import mel_oracle as MO
from oracle import spectral_oracle as SO

pytestmark = pytest.mark.gpu
DF = 22050 / 2048.0


def _oracle_vector(y, kind):
    mel = MO.extract_mel_spectrogram(y)
    v = [mel.mean(1), mel.std(1)]
    if kind == "basic":
        m = MO.mfcc(y)
        v += [m.mean(1), m.std(1)]
    v.append(SO.spectral_stats(y))
    ch, _ = SO.chroma_stft(y)
    v += [ch.mean(1), ch.std(1)]
    return np.concatenate([np.asarray(a, np.float64) for a in v])


@pytest.mark.parametrize("kind,dim", [("advanced", 290), ("basic", 370)])
def test_handcrafted_vector_vs_oracle(cuda, kind, dim):
    y = MO.synthetic_pcm(2, 22050 * 5, seed=3)
    got = P.handcrafted_features(y, kind=kind)
    assert got.shape == (2, dim) and got.dtype == np.float64
    for b in range(2):
        ref = _oracle_vector(y[b], kind)
        n_mel = 256 + (80 if kind == "basic" else 0)
        np.testing.assert_allclose(got[b, :n_mel], ref[:n_mel], atol=5e-3)
        sp = slice(n_mel, n_mel + 10)
        keep = [0, 1, 2, 3, 6, 7, 8, 9]
        np.testing.assert_allclose(got[b, sp][keep], ref[sp][keep], rtol=2e-4, atol=1e-6)
        np.testing.assert_allclose(got[b, sp][4:6], ref[sp][4:6], atol=0.02 * DF)
        np.testing.assert_allclose(got[b, n_mel + 10:], ref[n_mel + 10:], rtol=1e-4, atol=1e-5)


def test_write_processed_data2(cuda, tmp_path):
    N = 5
    clips = np.stack([P.pad_clip(c) for c in MO.synthetic_pcm(N, 22050 * 4, seed=9)])  # padded to 30 s
    assert clips.shape == (N, 22050 * 30)
    mel_raw, feats = P.extract_batches(clips, kind="advanced", batch=2)
    assert mel_raw.shape == (N, 128, 1024) and feats.shape == (N, 290)
    np.testing.assert_allclose(mel_raw, hlmc_amd.extract_mel_spectrogram(clips, fixed_time_steps=1024))
    rng = np.random.default_rng(0)
    lyrics = rng.normal(size=(N, 768)).astype(np.float32)
    genres = ["rock", "pop", "rock", "folk", "pop"]
    meta = [{"language": "en" if i % 2 else "bn", "genre": g, "filename": f"{i}.wav", "file_id": str(i)}
            for i, g in enumerate(genres)]
    out = str(tmp_path / "processed_data2")
    P.write_processed_data2(out, mel_raw, feats, lyrics, genres, meta)
    for f in ["mel_spectrograms_raw.npy", "mel_spectrograms_normalized.npy", "features_raw.npy",
              "features_normalized.npy", "lyrics_embeddings.npy", "labels.npy", "metadata.csv", "mel_scaler.pkl",
              "flat_scaler.pkl", "imputer.pkl", "config.pkl"]:
        assert os.path.exists(os.path.join(out, f)), f
    # what src/Convolutional_VAE.py:39-46 and src/Conditional_VAE.py:63-66 load
    mel_n = np.load(os.path.join(out, "mel_spectrograms_normalized.npy"))
    ref = SkScaler().fit_transform(mel_raw.reshape(N, -1)).reshape(mel_raw.shape)
    assert mel_n.dtype == np.float32
    np.testing.assert_allclose(mel_n, ref, rtol=1e-5, atol=1e-5)
    assert list(np.load(os.path.join(out, "labels.npy"))) == genres
    md = pd.read_csv(os.path.join(out, "metadata.csv"))
    assert list(md.columns) == ["language", "genre", "filename", "file_id", "label"]
    with open(os.path.join(out, "mel_scaler.pkl"), "rb") as f:  # our own file
        sc = pickle.load(f)
    np.testing.assert_allclose(sc.transform(mel_raw.reshape(N, -1)).reshape(mel_raw.shape), mel_n, rtol=1e-5, atol=1e-5)
    fn = np.load(os.path.join(out, "features_normalized.npy"))
    np.testing.assert_allclose(fn, SkScaler().fit_transform(feats), rtol=1e-10, atol=1e-12)


def test_write_processed_data1(cuda, tmp_path):
    y = MO.synthetic_pcm(4, 22050 * 3, seed=2)
    _, feats = P.extract_batches(y, kind="basic", batch=3)
    assert feats.shape == (4, 370)
    feats[1, 5] = np.inf                                     # imputed with the column mean, as the reference does
    meta = [{"language": "en", "genre": g, "filename": f"{i}.wav"} for i, g in enumerate("abab")]
    out = str(tmp_path / "processed_data1")
    P.write_processed_data1(out, feats, list("abab"), meta)
    fn = np.load(os.path.join(out, "features_normalized.npy"))
    assert np.isfinite(fn).all() and fn.shape == (4, 370)
    assert list(pd.read_csv(os.path.join(out, "metadata.csv")).columns) == ["language", "genre", "filename", "label"]
