"""CPU checks of the oracle itself against the reference's pins and the committed golden fixtures."""
import os

import numpy as np
import pytest
import torch

from oracle import kmeans_oracle as KO
from oracle import mel_oracle as MO
from oracle import models_oracle as OM
from tests.golden import fixtures as FX

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_librosa_documented_filterbank_value():
    # librosa docs: filters.mel(sr=22050, n_fft=2048)[0, 1] ~= 0.016; 2018 non-zeros; band 0 = bins 1..4
    W = MO.mel_filterbank()
    assert abs(W[0, 1] - 0.016) < 5e-4
    assert (W > 0).sum() == 2018
    nz0 = np.nonzero(W[0])[0]
    nz127 = np.nonzero(W[127])[0]
    assert (nz0[0], nz0[-1]) == (1, 4) and (nz127[0], nz127[-1]) == (971, 1023)


def test_window_and_dct_match_scipy():
    """The two scipy primitives librosa's mel / MFCC path calls (src/1_preprocessing_advanced.py:99-106 via
    librosa.stft's get_window; src/1_preprocessing.py:61-70 via librosa.feature.mfcc's scipy.fftpack.dct), pinned
    against scipy itself (importable here and on the GPU box): the periodic Hann window bit for bit, the
    DCT-II ortho matrix to 1e-15."""
    import scipy.fftpack
    import scipy.signal
    for n in (2048, 1024, 400):
        np.testing.assert_array_equal(MO.hann_window(n), scipy.signal.get_window("hann", n, fftbins=True))
    D = scipy.fftpack.dct(np.eye(128), type=2, norm="ortho", axis=0)[:40]
    assert float(np.abs(MO.dct_ortho_matrix() - D).max()) <= 1e-15
    x = np.random.default_rng(3).standard_normal((128, 7))
    np.testing.assert_allclose(MO.dct_ortho_matrix() @ x, scipy.fftpack.dct(x, type=2, norm="ortho", axis=0)[:40],
                               rtol=0, atol=1e-13)


def test_frames_and_shapes():
    assert MO.n_frames(65024) == 128 and MO.n_frames(661500) == 1292
    y = MO.synthetic_pcm(1, 65024, seed=1)[0]
    assert MO.extract_mel_spectrogram(y).shape == (128, 128)
    assert MO.extract_mel_spectrogram(y, fixed_time_steps=1024).shape == (128, 1024)
    assert MO.mfcc(y).shape == (40, 128)


def test_mel_fixture_reproduces():
    fx = np.load("tests/golden/features.npz")
    y = MO.synthetic_pcm(2, 65024, seed=7)
    np.testing.assert_array_equal(np.stack([MO.extract_mel_spectrogram(c) for c in y]), fx["mel_db"])
    np.testing.assert_array_equal(MO.mel_filterbank(), fx["mel_basis"])


def test_db_properties():
    y = MO.synthetic_pcm(1, 65024, seed=3)[0]
    db = MO.extract_mel_spectrogram(y)
    assert db.max() == 0.0 and db.min() >= -80.0
    assert np.all(MO.extract_mel_spectrogram(np.zeros(65024, np.float32)) == 0.0)


@pytest.mark.parametrize("case", FX.KMEANS_CASES[:4], ids=lambda c: f"n{c[0]}_d{c[1]}_k{c[3]}")
def test_kmeans_oracle_matches_sklearn_fixture(case):
    n, d, centers, k, n_init = case
    X = FX.blobs(n, d, centers, seed=n + d + k)
    fx = np.load(f"tests/golden/kmeans_n{n}_d{d}_k{k}_i{n_init}.npz")
    km = KO.KMeans(k, random_state=42, n_init=n_init).fit(X)
    np.testing.assert_array_equal(km.labels_, fx["labels"])
    assert km.n_iter_ == int(fx["n_iter"])


@pytest.mark.parametrize("case", [c for c in FX.KMEANS_OVERLAP_CASES if c[0] * c[4] <= 14000],
                         ids=lambda c: f"n{c[0]}_d{c[1]}_s{c[3]}_k{c[4]}_i{c[5]}")
def test_kmeans_oracle_matches_sklearn_overlap_fixture(case):
    """Overlapping clusters: labels decided by float32 rounding at near-ties; the oracle's bit-level E-step
    restatement reproduces sklearn's labels, n_iter and inertia exactly."""
    n, d, true_k, spread, k, n_init = case
    X = FX.overlap_blobs(n, d, true_k, spread, FX.overlap_seed(case))
    fx = np.load("tests/golden/" + FX.overlap_fixture_name(case))
    km = KO.KMeans(k, random_state=42, n_init=n_init).fit(X)
    np.testing.assert_array_equal(km.labels_, fx["labels"])
    assert km.n_iter_ == int(fx["n_iter"]) and km.inertia_ == float(fx["inertia"])


@pytest.mark.parametrize("k", [2, 7, 14])
def test_kmeans_oracle_matches_sklearn_latent_fixture(k):
    fx = np.load("tests/golden/kmeans_latents_n1336_d128.npz")
    km = KO.KMeans(k, random_state=42, n_init=10).fit(fx["X"])
    np.testing.assert_array_equal(km.labels_, fx[f"labels_k{k}"])
    assert km.n_iter_ == int(fx[f"n_iter_k{k}"]) and km.inertia_ == float(fx[f"inertia_k{k}"])


@pytest.mark.parametrize("n,d,k", [(1336, 128, 2), (1336, 128, 10), (1000, 64, 5), (513, 100, 13), (257, 32, 16),
                                   (300, 130, 3), (77, 40, 1)])
def test_estep_restatement_matches_blas(n, d, k):
    """oracle estep_dist (the arithmetic hlmc_km_assign implements) == the sgemm call sklearn makes
    (scipy's OpenBLAS, column-major TN per 256-row chunk), bit for bit, on near-tie data."""
    from threadpoolctl import threadpool_info, threadpool_limits
    archs = {i.get("architecture") for i in threadpool_info() if i.get("internal_api") == "openblas"}
    if archs != {"SkylakeX"}:
        pytest.skip(f"the restatement is of the SkylakeX OpenBLAS kernels the fixtures were made with, not {archs}")
    rng = np.random.default_rng(n * 31 + d * 7 + k)
    C = rng.standard_normal((k, d)).astype(np.float32)
    X = rng.standard_normal((n, d)).astype(np.float32)
    if k >= 2:
        m, u = (C[0] + C[1]) / 2, C[1] - C[0]
        u = u / np.linalg.norm(u)
        X = (m + 0.3 * (X - np.outer(X @ u, u)) + np.outer(rng.standard_normal(n) * 1e-6, u)).astype(np.float32)
    cn = KO.row_norms_sq_f32(C)
    np.testing.assert_array_equal(cn, np.einsum("ij,ij->i", C, C))
    with threadpool_limits(1, "blas"):
        for s in range(0, n, KO.CHUNK):
            np.testing.assert_array_equal(KO.estep_dist(X[s:s + KO.CHUNK], C, cn),
                                          KO.estep_dist_blas(X[s:s + KO.CHUNK], C, cn))


def test_scaler_oracle_matches_fixture():
    fx = np.load("tests/golden/features.npz")
    rng = np.random.default_rng(11)
    cols = (rng.standard_normal((64, 300)) * rng.uniform(0.1, 5, 300) + rng.uniform(-3, 3, 300)).astype(np.float32)
    cols[:, 5] = 2.5
    m, v, s = KO.standard_scaler_fit(cols)
    np.testing.assert_array_equal(s, fx["scaler_scale"])
    np.testing.assert_array_equal(KO.standard_scaler_transform(cols, m, s), fx["scaler_out"])


@pytest.mark.parametrize("name", ["audio_128x128", "hybrid_128x128_td768", "cvae_128x128", "simple_370"])
def test_model_oracle_reproduces_fixture(name):
    case = FX.case_by_name(name)
    fx = np.load(f"tests/golden/model_{name}.npz")
    torch.manual_seed(42)
    m = {"hybrid": OM.HybridVAE, "cvae": OM.ConditionalVAE, "simple": OM.VAE}[case["kind"]](**FX.oracle_ctor(case))
    assert [n for n, _ in m.named_parameters()] == list(fx["param_names"])
    np.testing.assert_array_equal(FX.param_summary(m), fx["param_checksum_init"])
    ins, eps = FX.inputs_fn(case)(0)
    torch.manual_seed(7)
    m.train()
    out = m(*ins, eps=eps)
    if case["kind"] == "simple":
        loss = OM.vae_loss(out[0], ins[0], out[1], out[2], beta=0.8)
    elif case["kind"] == "hybrid":
        loss = OM.loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3])
    else:
        loss = OM.cvae_loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3], beta=4.0)
    np.testing.assert_allclose([float(t) for t in loss], fx["loss_step0"], rtol=1e-6)
    loss[0].backward()
    np.testing.assert_allclose(FX.grad_summary(m), fx["grad_summary"], rtol=1e-5, atol=1e-7)


def test_native_shapes_match_reference_at_128x1024():
    torch.manual_seed(42)
    m = OM.HybridVAE()  # reference default (128 x 1024)
    assert m.audio_fc.weight.shape == (1024, 16384) and sum(p.numel() for p in m.parameters()) == 43272065


# ---------------------------------------------------------------- cluster-quality metrics (§8f rows 1, 4)
@pytest.mark.parametrize("case", FX.METRICS_CASES)
def test_metrics_oracle_matches_sklearn_fixtures(case):
    """The numpy restatement (the GPU tests' checker) reproduces sklearn's recorded scores; the host label
    metrics of hlmc_amd.metrics (ARI / NMI / purity) reproduce sklearn and the reference's calculate_purity."""
    from oracle import metrics_oracle as MO
    import hlmc_amd
    n, d, centers, k, n_init = case
    fx = np.load(os.path.join(GOLDEN, FX.metrics_fixture_name(case)))
    X = FX.blobs(n, d, centers, seed=n + d + k)
    y_true = FX.blob_labels(n, d, centers, seed=n + d + k)
    y_pred = np.load(os.path.join(GOLDEN, FX.kmeans_fixture_name(case)))["labels"].astype(np.int64)
    np.testing.assert_allclose(MO.silhouette_samples(X, y_pred), fx["silhouette_samples"], rtol=1e-5, atol=1e-6)
    assert abs(MO.silhouette_score(X, y_pred) - float(fx["silhouette"])) <= 1e-6 * abs(float(fx["silhouette"])) + 1e-7
    assert abs(MO.davies_bouldin_score(X, y_pred) - float(fx["davies_bouldin"])) <= 1e-6 * float(fx["davies_bouldin"])  # sklearn: float32 centroids
    assert abs(MO.calinski_harabasz_score(X, y_pred) - float(fx["calinski_harabasz"])) <= 1e-6 * float(fx["calinski_harabasz"])
    M = hlmc_amd.metrics
    assert abs(M.adjusted_rand_score(y_true, y_pred) - float(fx["ari"])) <= 1e-12
    assert abs(M.normalized_mutual_info_score(y_true, y_pred) - float(fx["nmi"])) <= 1e-12
    assert M.calculate_purity(y_true, y_pred) == float(fx["purity"])


def test_spectral_oracle_properties():
    """Pins the restatement of librosa's frame features (parity against librosa itself is unpinned):
    a bin-centred tone has its centroid and rolloff at the tone, zcr = 2 f / sr, rms = A / sqrt(2);
    silence gives zeros (the unnormalised branch of librosa.util.normalize)."""
    from oracle import spectral_oracle as SO
    sr, n = 22050, 22050 * 2
    f = 100 * sr / 2048.0                      # bin 100
    t = np.arange(n) / sr
    y = (0.5 * np.sin(2 * np.pi * f * t)).astype(np.float32)
    inner = slice(4, -4)
    c = SO.spectral_centroid(y)[0, inner]
    assert np.all(np.abs(c - f) < 2e-3)
    # Hann main lobe: |X| = (1/2, 1, 1/2) at bins 99..101 -> cumsum crosses 0.85 * 2 at bin 101
    assert np.all(SO.spectral_rolloff(y)[0, inner] == 101 * sr / 2048.0)
    bw = SO.spectral_bandwidth(y)[0, inner]
    # S_norm = (1/4, 1/2, 1/4) -> bandwidth = sqrt(1/2) df; the float32 quantisation floor of y spread over
    # 1025 bins adds a few percent (deviations up to 10 kHz weigh it)
    df = sr / 2048.0
    assert np.all((bw > np.sqrt(0.5) * df) & (bw < 1.06 * np.sqrt(0.5) * df))
    np.testing.assert_allclose(SO.zero_crossing_rate(y)[0, inner], 2 * f / sr, atol=1.5 / 2048)
    np.testing.assert_allclose(SO.rms(y)[0, inner], 0.5 / np.sqrt(2), rtol=2e-3)
    z = np.zeros(n, np.float32)
    assert not SO.spectral_stats(z).any()
    stats = SO.spectral_stats(y)
    assert stats.shape == (10,) and np.isfinite(stats).all()


def test_chroma_oracle_properties():
    """Pins the chroma_stft restatement (parity vs librosa unpinned): the filterbank is 12 x 1025 float32 with
    unit-L2 columns before the octave weighting (so every column's norm is that weight); an A tone lands on
    chroma 9 (base_c=True); the tuning estimate follows a detuned tone to within the 0.01-semitone histogram's
    piptrack error; silence gives tuning 0 and all-zero chroma."""
    from oracle import spectral_oracle as SO
    fb = SO.chroma_filterbank()
    assert fb.shape == (12, 1025) and fb.dtype == np.float32
    freqs = np.linspace(0, 22050, 2048, endpoint=False)[1:1025]
    octw = np.exp(-0.5 * (((np.log2(freqs / 27.5) - 5.0) / 2) ** 2))
    np.testing.assert_allclose(np.linalg.norm(fb[:, 1:].astype(np.float64), axis=0), octw, rtol=1e-5)
    t = np.arange(22050 * 3) / 22050
    for det in (0.0, 0.23, -0.31):
        f = 440 * 2 ** (det / 12)
        y = (0.3 * np.sin(2 * np.pi * f * t) + 0.2 * np.sin(2 * np.pi * 1.5 * f * t)).astype(np.float32)
        ch, tun = SO.chroma_stft(y)
        assert abs(tun - det) <= 0.06, (det, tun)
        assert np.argmax(ch[:, 8:-8].mean(1)) == 9
    ch, tun = SO.chroma_stft(np.zeros(8192, np.float32))
    assert tun == 0.0 and not ch.any()


def test_philox_known_answers():
    """oracle/rng_oracle.py Philox4x32-10 against the Random123 known-answer vectors (kat_vectors: philox4x32_10)."""
    from oracle.rng_oracle import normals, philox4x32
    assert philox4x32((0, 0, 0, 0), (0, 0)) == (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)
    assert philox4x32((0xffffffff,) * 4, (0xffffffff,) * 2) == (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)
    assert philox4x32((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0)) == (
        0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)
    a = normals(4096, seed=1234)
    assert abs(float(a.mean())) < 0.05 and abs(float(a.std()) - 1) < 0.05
    np.testing.assert_array_equal(normals(8, seed=1234, offset=4096 - 8), a[-8:])


@pytest.mark.parametrize("name", ["audio_128x128", "hybrid_128x128_td768", "cvae_128x128", "simple_370"])
def test_oracle_training_chain_reproduces_fixture_latents(name):
    """The oracle's 3-step train chain (tests/test_models_gpu._oracle_trained: the fixture generator's Adam steps
    and dropout seeds) then eval-mode encode reproduces the reference classes' fixture eval_mu bit for bit on the
    generating host — the pin of the latent-extraction contract (src/Convolutional_VAE.py:286-303,
    src/Conditional_VAE.py:397-402, src/Simple_VAE.py:225-226) the GPU test compares the engine against."""
    from tests.test_models_gpu import _oracle_trained
    case = FX.case_by_name(name)
    ora = _oracle_trained(case)
    ins, _ = FX.inputs_fn(case)(0)
    with torch.no_grad():
        mu = ora.encode(*ins)[0]
    fx = np.load(f"tests/golden/model_{name}.npz")["eval_mu"]
    err = float(np.abs(mu.numpy() - fx).max())
    # bit-exact where the fixtures were generated (this container's CPU); Adam-amplified rounding elsewhere
    assert err == 0.0 or float(np.linalg.norm(mu.numpy() - fx) / np.linalg.norm(fx)) < 5e-2, err
