"""Cluster-quality metrics on the GPU vs sklearn 1.7.2's recorded outputs
(tests/golden/metrics_*.npz) and the float64 oracle (oracle/metrics_oracle.py).

Tolerances: silhouette score 1e-6 relative, per-sample coefficients 1e-5 relative + 1e-6 absolute (sklearn
rounds the per-cluster distance sums to float32; the kernel keeps fp32 distances and f64 sums);
Davies-Bouldin / Calinski-Harabasz 1e-6 relative (sklearn's centroids are float32 means).  Every kernel
call is deterministic: repeated runs are bit-identical."""
import numpy as np
import pytest
import torch

import hlmc_amd
from oracle import metrics_oracle as MO
from tests.golden import fixtures as FX

pytestmark = pytest.mark.gpu
M = hlmc_amd.metrics


def _case(case):
    n, d, centers, k, n_init = case
    X = FX.blobs(n, d, centers, seed=n + d + k)
    y_pred = np.load(f"tests/golden/{FX.kmeans_fixture_name(case)}")["labels"].astype(np.int64)
    return X, y_pred, np.load(f"tests/golden/{FX.metrics_fixture_name(case)}")


@pytest.mark.parametrize("case", FX.METRICS_CASES, ids=lambda c: f"n{c[0]}_d{c[1]}_k{c[3]}")
def test_silhouette_matches_sklearn(cuda, case):
    X, y, fx = _case(case)
    Xd = torch.from_numpy(X).to(cuda)
    s = M.silhouette_score(Xd, y)
    ref = float(fx["silhouette"])
    assert abs(s - ref) <= 1e-6 * abs(ref) + 1e-8, (s, ref)
    samples = M.silhouette_samples(Xd, y).cpu().numpy()
    np.testing.assert_allclose(samples, fx["silhouette_samples"], rtol=1e-5, atol=1e-6)
    # deterministic: a second run is bit-identical
    assert M.silhouette_score(Xd, y) == s
    assert torch.equal(M.silhouette_samples(Xd, y).cpu(), torch.from_numpy(samples))


@pytest.mark.parametrize("case", FX.METRICS_CASES, ids=lambda c: f"n{c[0]}_d{c[1]}_k{c[3]}")
def test_davies_bouldin_calinski_harabasz_match_sklearn(cuda, case):
    X, y, fx = _case(case)
    Xd = torch.from_numpy(X).to(cuda)
    db, ch = M.davies_bouldin_score(Xd, y), M.calinski_harabasz_score(Xd, y)
    assert abs(db - float(fx["davies_bouldin"])) <= 1e-6 * float(fx["davies_bouldin"]), db
    assert abs(ch - float(fx["calinski_harabasz"])) <= 1e-6 * float(fx["calinski_harabasz"]), ch


def test_silhouette_edge_cases(cuda):
    """Singleton clusters score 0 (sklearn's nan_to_num), string labels are encoded like LabelEncoder,
    k = 2 and a ragged n (not a multiple of the 64-row tiles) against the oracle; k = 1 raises."""
    rng = np.random.default_rng(5)
    X = rng.normal(0, 1, (203, 24)).astype(np.float32)
    y = rng.integers(0, 5, 203)
    y[17] = 9  # a singleton cluster
    s = M.silhouette_samples(X, y).cpu().numpy()
    assert s[17] == 0.0
    np.testing.assert_allclose(s, MO.silhouette_samples(X, y), rtol=1e-5, atol=1e-6)
    names = np.array(["rock", "pop", "jazz"])[rng.integers(0, 3, 203)]
    assert abs(M.silhouette_score(X, names) - MO.silhouette_score(X, names)) < 1e-6
    y2 = (X[:, 0] > 0).astype(np.int64)
    assert abs(M.silhouette_score(X, y2) - MO.silhouette_score(X, y2)) < 1e-6
    with pytest.raises(ValueError):
        M.silhouette_score(X, np.zeros(203, dtype=np.int64))


def test_silhouette_larger_n_vs_oracle(cuda):
    """n = 6000 (94 row tiles, ragged last tile), d = 32, k = 7 against the float64 oracle."""
    X = FX.blobs(6000, 32, 7, seed=21)
    y = FX.blob_labels(6000, 32, 7, seed=21)
    np.testing.assert_allclose(M.silhouette_samples(torch.from_numpy(X).to(cuda), y).cpu().numpy(),
                               MO.silhouette_samples(X, y), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("d", [16, 128])
def test_many_clusters_label_windows(cuda, d):
    """k = 150 > the 64 LDS accumulator rows of one launch: the label windows (silhouette) and the clu_sums
    windows (Davies-Bouldin / Calinski-Harabasz) against the float64 oracle; sklearn allows k up to n - 1."""
    rng = np.random.default_rng(d)
    X = rng.normal(0, 1, (900, d)).astype(np.float32)
    y = rng.integers(0, 150, 900)
    Xd = torch.from_numpy(X).to(cuda)
    np.testing.assert_allclose(M.silhouette_samples(Xd, y).cpu().numpy(), MO.silhouette_samples(X, y),
                               rtol=1e-5, atol=1e-6)
    db, ch = M.davies_bouldin_score(Xd, y), M.calinski_harabasz_score(Xd, y)
    assert abs(db - MO.davies_bouldin_score(X, y)) <= 1e-6 * abs(MO.davies_bouldin_score(X, y))
    assert abs(ch - MO.calinski_harabasz_score(X, y)) <= 1e-6 * abs(MO.calinski_harabasz_score(X, y))
