"""Feature kernels vs the numpy restatement of librosa (oracle/mel_oracle.py) and sklearn.

librosa itself is absent here and the reference ships no mel values: the mel/MFCC parity is
UNPINNED against librosa (pinned only by librosa's documented filterbank value and properties, see
tests/test_oracle_cpu.py).  Tolerances: the reference computes the STFT in float64 (then complex64);
the GPU kernel computes it in float32, so dB values agree to <= 2e-3 dB for bins above -60 dB and
are compared with atol 0.05 dB overall (bins near the -80 dB floor have ~1e-4 relative power error)."""
import numpy as np
import pytest
import torch
from sklearn.preprocessing import StandardScaler as SkScaler

import hlmc_amd
from oracle import mel_oracle as MO
from oracle import kmeans_oracle as KO

pytestmark = pytest.mark.gpu


def test_filterbank_matches_oracle(cuda):
    fb = hlmc_amd.mel_filterbank()
    ref = MO.mel_filterbank()
    np.testing.assert_allclose(fb, ref, rtol=1e-6, atol=1e-9)
    assert (fb > 0).sum() == 2018


@pytest.mark.parametrize("n_samples,keep", [(65024, None), (65024, 128), (22050 * 3, 256), (661500, 1024),
                                             (22050 * 3 + 17, None), (1500, 8)])
def test_mel_db(cuda, n_samples, keep):
    """Even lengths take the kernel's 8-byte sample-pair loads, odd lengths the 4-byte ones; 1500 samples is
    shorter than one frame (every frame reads the zero padding through the loads' range check)."""
    y = MO.synthetic_pcm(2, n_samples, seed=n_samples % 97)
    got = hlmc_amd.extract_mel_spectrogram(y, fixed_time_steps=keep)
    ref = np.stack([MO.extract_mel_spectrogram(c, fixed_time_steps=keep) for c in y])
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, atol=0.05)
    hi = ref > -60
    assert np.abs(got - ref)[hi].max() < 2e-3


@pytest.mark.parametrize("n_samples,keep", [(65024, 128), (22050 * 3, 256), (661500, 1024)])
def test_mel_db_zscore_fused_bitexact(cuda, n_samples, keep):
    """hlmc_mel_db_zscore (the scaler's transform inside the dB pass, the bench's mel stage) is bit-identical to
    extract_mel_spectrogram followed by StandardScaler.transform; pad (T < keep) and crop (T > keep) cases."""
    y = torch.from_numpy(MO.synthetic_pcm(3, n_samples, seed=5)).cuda()
    mel = hlmc_amd.extract_mel_spectrogram(y, fixed_time_steps=keep)
    sc = hlmc_amd.StandardScaler().fit(mel.reshape(3, -1))
    for dt in (torch.float32, torch.bfloat16):
        fused = hlmc_amd.extract_mel_spectrogram(y, fixed_time_steps=keep, scaler=sc, out_dtype=dt)
        two = sc.transform(mel.reshape(3, -1), out_dtype=dt).reshape(fused.shape)
        assert fused.dtype == dt and torch.equal(fused, two), dt
    with pytest.raises(RuntimeError):
        hlmc_amd.extract_mel_spectrogram(y[:, :65024 - 512], fixed_time_steps=126,
                                         scaler=hlmc_amd.StandardScaler().fit(torch.zeros(2, 128 * 126).cuda()))


def test_mel_db_vector_and_scalar_paths_agree(cuda):
    """The 4-frame vector dB kernel (keep % 4 == 0) and the scalar one (otherwise) give identical frames."""
    y = MO.synthetic_pcm(2, 22050 * 3, seed=9)   # T = 130 frames
    a = hlmc_amd.extract_mel_spectrogram(y, fixed_time_steps=130)
    b = hlmc_amd.extract_mel_spectrogram(y, fixed_time_steps=132)
    assert np.array_equal(a, b[:, :, :130])
    assert np.array_equal(b[:, :, 130], b[:, :, 131])   # padded with the clip minimum


def test_mel_db_golden(cuda):
    fx = np.load("tests/golden/features.npz")
    y = MO.synthetic_pcm(2, 65024, seed=7)
    np.testing.assert_allclose(hlmc_amd.extract_mel_spectrogram(y), fx["mel_db"], atol=0.05)
    np.testing.assert_allclose(hlmc_amd.mfcc(y, n_mfcc=40), fx["mfcc"], atol=0.05, rtol=1e-3)


def test_melspectrogram_power(cuda):
    y = MO.synthetic_pcm(3, 32768, seed=2)
    got = hlmc_amd.melspectrogram(y)
    ref = MO.melspectrogram(y)
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-6 * ref.max())


def test_silence_and_tone(cuda):
    # silence -> all zeros dB (ref = max = 0 < amin); tone at a bin centre peaks in its mel band
    z = np.zeros((1, 65024), np.float32)
    assert np.all(hlmc_amd.extract_mel_spectrogram(z) == 0.0)
    f = 100 * 22050 / 2048
    t = np.arange(65024) / 22050
    tone = (0.5 * np.sin(2 * np.pi * f * t)).astype(np.float32)[None]
    db = hlmc_amd.extract_mel_spectrogram(tone)[0]
    fb = MO.mel_filterbank()
    assert int(np.argmax(db[:, 64])) == int(np.argmax(fb[:, 100]))


def test_power_to_db_and_mfcc(cuda):
    y = MO.synthetic_pcm(2, 40000, seed=4)
    S = MO.melspectrogram(y)
    got = hlmc_amd.power_to_db(S, ref=np.max)
    ref = MO.power_to_db_batched(S)
    np.testing.assert_allclose(got, ref, atol=1e-3)
    np.testing.assert_allclose(hlmc_amd.power_to_db(S[0], ref=1.0), MO.power_to_db(S[0], ref=1.0), atol=1e-3)
    mf = hlmc_amd.mfcc(y, n_mfcc=40)
    mref = np.stack([MO.mfcc(c) for c in y])
    np.testing.assert_allclose(mf, mref, atol=0.05, rtol=1e-3)


def test_mean_std_pool(cuda):
    x = np.random.default_rng(0).normal(-30, 10, (5, 128, 300)).astype(np.float32)
    got = hlmc_amd.mean_std_pool(x)
    ref = np.stack([MO.mean_std_pool(a) for a in x])
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


def test_standard_scaler_bitexact(cuda):
    rng = np.random.default_rng(11)
    X = (rng.standard_normal((300, 513)) * rng.uniform(0.1, 5, 513) + rng.uniform(-3, 3, 513)).astype(np.float32)
    X[:, 7] = 1.25
    sk = SkScaler().fit(X)
    ours = hlmc_amd.StandardScaler().fit(X)
    np.testing.assert_allclose(ours.mean_, sk.mean_, rtol=1e-14)
    np.testing.assert_allclose(ours.var_, sk.var_, rtol=1e-10)
    np.testing.assert_allclose(ours.scale_, sk.scale_, rtol=1e-10)
    out = ours.transform(X)
    ref = sk.transform(X)
    assert np.mean(out == ref) > 0.999
    np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-6)


def test_standard_scaler_golden(cuda):
    fx = np.load("tests/golden/features.npz")
    rng = np.random.default_rng(11)
    cols = (rng.standard_normal((64, 300)) * rng.uniform(0.1, 5, 300) + rng.uniform(-3, 3, 300)).astype(np.float32)
    cols[:, 5] = 2.5
    ours = hlmc_amd.StandardScaler().fit(cols)
    np.testing.assert_allclose(ours.scale_, fx["scaler_scale"], rtol=1e-10)
    np.testing.assert_allclose(ours.transform(cols), fx["scaler_out"], rtol=1e-6, atol=1e-6)


def test_mel_deterministic_repeat(cuda):
    """The STFT-mel path is deterministic: repeated calls are bit-identical and stay within tolerance."""
    fx = np.load("tests/golden/features.npz")
    y = MO.synthetic_pcm(2, 65024, seed=7)
    d0, m0 = hlmc_amd.extract_mel_spectrogram(y), hlmc_amd.mfcc(y, n_mfcc=40)
    bad = []
    for i in range(10):
        d, m = hlmc_amd.extract_mel_spectrogram(y), hlmc_amd.mfcc(y, n_mfcc=40)
        if not (np.array_equal(d, d0) and np.array_equal(m, m0)):
            bad.append((i, float(np.abs(d - d0).max()), float(np.abs(m - m0).max())))
    e_db = float(np.abs(d0 - fx["mel_db"]).max())
    e_mf = np.abs(m0 - fx["mfcc"]) - (0.05 + 1e-3 * np.abs(fx["mfcc"]))
    assert not bad, f"non-deterministic repeats: {bad}"
    assert e_db < 0.05, e_db
    assert float(e_mf.max()) <= 0, (float(e_mf.max()), np.unravel_index(e_mf.argmax(), e_mf.shape))
