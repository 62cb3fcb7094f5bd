"""K-Means on the GPU vs sklearn 1.7.2 KMeans(random_state=42) labels recorded in tests/golden
(bit-identical labels required; centres within float32 rounding; ARI vs sklearn == 1)."""
import glob

import numpy as np
import pytest

import hlmc_amd
from tests.golden import fixtures as FX

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", FX.KMEANS_CASES, ids=lambda c: f"n{c[0]}_d{c[1]}_k{c[3]}_i{c[4]}")
def test_kmeans_labels_bitexact(cuda, case):
    n, d, centers, k, n_init = case
    X = FX.blobs(n, d, centers, seed=n + d + k)
    fx = np.load(f"tests/golden/kmeans_n{n}_d{d}_k{k}_i{n_init}.npz")
    km = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
    np.testing.assert_array_equal(km.labels_, fx["labels"])
    np.testing.assert_allclose(km.cluster_centers_, fx["centers"], rtol=1e-5, atol=1e-5)
    assert km.n_iter_ == int(fx["n_iter"])
    assert abs(km.inertia_ - float(fx["inertia"])) <= 1e-4 * float(fx["inertia"])


def test_kmeans_predict_and_auto(cuda):
    X = FX.blobs(2000, 32, 5, seed=3)
    km = hlmc_amd.KMeans(5, random_state=0).fit(X)
    np.testing.assert_array_equal(km.predict(X), km.labels_)


def test_kmeans_empty_cluster_relocation(cuda):
    # duplicated points force empty clusters in early iterations
    X = np.repeat(FX.blobs(40, 8, 3, seed=1), 5, axis=0)
    from sklearn.cluster import KMeans as SK
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        ref = SK(n_clusters=12, random_state=42, n_init=3).fit(X)
    ours = hlmc_amd.KMeans(n_clusters=12, random_state=42, n_init=3).fit(X)
    np.testing.assert_array_equal(ours.labels_, ref.labels_)
