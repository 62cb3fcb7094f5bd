"""Handcrafted frame features (§8f row 2) vs the numpy restatement of librosa (oracle/spectral_oracle.py).

librosa is absent and the reference ships no values of these features: parity against librosa itself is
UNPINNED; the oracle is pinned by the property tests in tests/test_oracle_cpu.py.  Tolerances (the GPU
STFT runs in float32, the oracle's in float64 -> complex64, as librosa's):
  * centroid / bandwidth: |d| <= 1e-5 * value + 0.05 Hz
  * rolloff: a frame whose cumulative magnitude sits within rounding of the threshold may pick the
    neighbouring bin: <= 1% of frames differ, each by exactly one bin (10.77 Hz)
  * zcr: bit-exact (same samples, integer counts); rms: rtol 1e-5
"""
import numpy as np
import pytest
import torch

import hlmc_amd
from oracle import mel_oracle as MO
from oracle import spectral_oracle as SO

pytestmark = pytest.mark.gpu
DF = 22050 / 2048.0


def _check_shape_feats(got, y):
    for b in range(y.shape[0]):
        c = SO.spectral_centroid(y[b])[0]
        bw = SO.spectral_bandwidth(y[b])[0]
        ro = SO.spectral_rolloff(y[b])[0]
        np.testing.assert_allclose(got["spectral_centroid"][b, 0], c, rtol=1e-5, atol=0.05)
        np.testing.assert_allclose(got["spectral_bandwidth"][b, 0], bw, rtol=1e-5, atol=0.05)
        d = np.abs(got["spectral_rolloff"][b, 0] - ro)
        assert np.all((d == 0) | (np.abs(d - DF) < 1e-9)), d.max()
        assert (d > 0).mean() <= 0.01


@pytest.mark.parametrize("n_samples", [65024, 22050 * 3 + 17, 661500])
def test_spectral_features_vs_oracle(cuda, n_samples):
    y = MO.synthetic_pcm(2, n_samples, seed=n_samples % 89)
    got = hlmc_amd.extract_spectral_features(y)
    T = MO.n_frames(n_samples)
    for k in hlmc_amd.SPECTRAL_FEATURES:
        assert got[k].shape == (2, 1, T), k
    assert got["rms"].dtype == np.float32 and got["spectral_centroid"].dtype == np.float64
    _check_shape_feats(got, y)
    for b in range(2):
        np.testing.assert_array_equal(got["zcr"][b, 0], SO.zero_crossing_rate(y[b])[0])
        np.testing.assert_allclose(got["rms"][b, 0], SO.rms(y[b])[0], rtol=1e-5, atol=1e-9)


def test_spectral_edge_cases(cuda):
    # silence: librosa leaves all-zero columns unnormalised -> every feature is 0
    z = np.zeros((1, 8192), np.float32)
    got = hlmc_amd.extract_spectral_features(z)
    for k in hlmc_amd.SPECTRAL_FEATURES:
        assert not np.any(got[k]), k
    # clip shorter than one frame (every frame is an edge frame), 1-D input, values at the zcr threshold
    rng = np.random.default_rng(3)
    y = rng.normal(0, 0.1, 1500).astype(np.float32)
    y[::7] = 1e-10
    y[3::11] = -1e-10
    y[5::13] = -0.0
    assert hlmc_amd.spectral_centroid(y).shape == (1, MO.n_frames(1500))
    np.testing.assert_array_equal(hlmc_amd.zero_crossing_rate(y), SO.zero_crossing_rate(y))
    np.testing.assert_allclose(hlmc_amd.rms(y), SO.rms(y), rtol=1e-5)
    got = {k: v[None] for k, v in hlmc_amd.extract_spectral_features(y).items()}
    _check_shape_feats(got, y[None])
    # a pure bin-centred tone: centroid at the tone, rolloff one bin above (Hann main lobe)
    t = np.arange(22050) / 22050
    tone = (0.5 * np.sin(2 * np.pi * 100 * DF * t)).astype(np.float32)
    ro = hlmc_amd.spectral_rolloff(tone)[0, 4:-4]
    assert np.all(ro == 101 * DF)


def test_spectral_stats_and_device_io(cuda):
    y = MO.synthetic_pcm(3, 44100, seed=11)
    st = hlmc_amd.spectral_stats(y)
    assert st.shape == (3, 10)
    for b in range(3):
        ref = SO.spectral_stats(y[b])
        keep = [0, 1, 2, 3, 6, 7, 8, 9]
        np.testing.assert_allclose(st[b, keep], ref[keep], rtol=2e-4, atol=1e-6)
        # rolloff mean / std: the <= 1% one-bin flips above move them by at most ~0.02 bins
        np.testing.assert_allclose(st[b, 4:6], ref[4:6], atol=0.02 * DF)
    yt = torch.from_numpy(y).cuda()
    d = hlmc_amd.extract_spectral_features(yt)
    assert all(v.is_cuda for v in d.values())
    h = hlmc_amd.extract_spectral_features(y)
    for k in hlmc_amd.SPECTRAL_FEATURES:
        np.testing.assert_array_equal(d[k].cpu().numpy(), h[k])   # deterministic across calls


def test_spectral_rejects_bad_arguments(cuda):
    with pytest.raises(Exception):
        hlmc_amd.spectral_rolloff(np.zeros(4096, np.float32), roll_percent=1.5)


def _tones(n, dets, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 22050
    out = []
    for d in dets:
        f = 440 * 2 ** (d / 12)
        y = 0.3 * np.sin(2 * np.pi * f * t) + 0.2 * np.sin(2 * np.pi * f * 1.5 * t) + rng.normal(0, 0.01, n)
        out.append(y)
    return np.asarray(out, dtype=np.float32)


@pytest.mark.parametrize("kind", ["tones", "synthetic"])
def test_chroma_stft_vs_oracle(cuda, kind):
    """Tuning estimates must agree exactly (they select the filterbank); chroma then rtol 1e-4 (float32 sums
    in a different order than numpy's BLAS einsum)."""
    y = _tones(22050 * 3, [0.0, 0.23, -0.31]) if kind == "tones" else MO.synthetic_pcm(3, 22050 * 4 + 5, seed=5)
    got, tun = hlmc_amd.chroma_stft(y, return_tuning=True)
    assert got.shape == (3, 12, MO.n_frames(y.shape[1])) and got.dtype == np.float32
    for b in range(3):
        ref, rt = SO.chroma_stft(y[b])
        assert tun[b] == rt, (b, tun[b], rt)
        np.testing.assert_allclose(got[b], ref, rtol=1e-4, atol=1e-6)


def test_chroma_edge_cases(cuda):
    z = np.zeros((2, 4096), np.float32)                      # silence: no peaks -> tuning 0, chroma 0
    c, tun = hlmc_amd.chroma_stft(z, return_tuning=True)
    assert not c.any() and not tun.any()
    y = _tones(1500, [0.1])[0]                               # shorter than one frame, 1-D input
    c, tun = hlmc_amd.chroma_stft(y, return_tuning=True)
    ref, rt = SO.chroma_stft(y)
    assert c.shape == ref.shape and float(tun) == rt
    np.testing.assert_allclose(c, ref, rtol=1e-4, atol=1e-6)
    # an A tone: the A chroma (index 9, base_c=True) dominates
    a = _tones(22050 * 2, [0.0])
    assert np.argmax(hlmc_amd.chroma_stft(a)[0][:, 8:-8].mean(1)) == 9


def test_other_rate_and_hop(cuda):
    """sr = 16 kHz, hop = 256: the bin frequencies, the piptrack mask and the chroma filterbank follow sr."""
    sr, hop = 16000, 256
    y = MO.synthetic_pcm(2, sr * 2, seed=21)
    c = hlmc_amd.spectral_centroid(y, sr=sr, hop_length=hop)
    assert c.shape == (2, 1, 1 + y.shape[1] // hop)
    for b in range(2):
        np.testing.assert_allclose(c[b, 0], SO.spectral_centroid(y[b], sr, 2048, hop)[0], rtol=1e-5, atol=0.05)
        np.testing.assert_array_equal(hlmc_amd.zero_crossing_rate(y[b:b + 1], hop_length=hop)[0, 0],
                                      SO.zero_crossing_rate(y[b], 2048, hop)[0])
    ch, tun = hlmc_amd.chroma_stft(y, sr=sr, hop_length=hop, return_tuning=True)
    for b in range(2):
        ref, rt = SO.chroma_stft(y[b], sr, 2048, hop)
        assert tun[b] == rt
        np.testing.assert_allclose(ch[b], ref, rtol=1e-4, atol=1e-6)
