"""TEST INFRASTRUCTURE ONLY (checker, never shipped or measured): numpy float64 restatement of the
sklearn 1.7.2 cluster-quality metrics the reference calls:

  silhouette_samples / silhouette_score  sklearn/metrics/cluster/_unsupervised.py (silhouette_samples,
      _silhouette_reduce): per-row sums of euclidean distances by cluster, a = intra / (n_l - 1),
      b = min over other clusters of mean distance, s = (b - a) / max(a, b), 0 for singletons; mean.
      Called at src/Convolutional_VAE.py:320,337,361,399, src/Conditional_VAE.py:298, src/Simple_VAE.py:247.
  davies_bouldin_score     (_unsupervised.py davies_bouldin_score) src/Convolutional_VAE.py:400
  calinski_harabasz_score  (_unsupervised.py calinski_harabasz_score) src/Simple_VAE.py:257,263

Pinned: tests/test_oracle_cpu.py checks it against the committed sklearn outputs (tests/golden/metrics_*.npz,
made by tests/golden/make_golden.py with sklearn itself).
"""
from __future__ import annotations

import numpy as np


def _encode(labels):
    classes, enc = np.unique(np.asarray(labels), return_inverse=True)
    return enc.reshape(-1), len(classes)


def silhouette_samples(X, labels, chunk=1024):
    X = np.asarray(X, dtype=np.float64)
    lab, k = _encode(labels)
    n = X.shape[0]
    freqs = np.bincount(lab, minlength=k)
    sq = (X * X).sum(1)
    S = np.zeros((n, k))
    for i0 in range(0, n, chunk):
        xi = X[i0:i0 + chunk]
        d2 = sq[i0:i0 + chunk, None] + sq[None, :] - 2.0 * xi @ X.T
        D = np.sqrt(np.maximum(d2, 0.0))
        D[np.arange(xi.shape[0]), np.arange(i0, i0 + xi.shape[0])] = 0.0
        for c in range(k):
            S[i0:i0 + chunk, c] = D[:, lab == c].sum(1)
    intra = S[np.arange(n), lab]
    Sm = S / freqs[None, :]
    Sm[np.arange(n), lab] = np.inf
    inter = Sm.min(1)
    denom = (freqs - 1)[lab]
    with np.errstate(divide="ignore", invalid="ignore"):
        a = intra / denom
        s = (inter - a) / np.maximum(a, inter)
    return np.nan_to_num(s)


def silhouette_score(X, labels):
    return float(np.mean(silhouette_samples(X, labels)))


def davies_bouldin_score(X, labels):
    X = np.asarray(X, dtype=np.float64)
    lab, k = _encode(labels)
    cent = np.stack([X[lab == c].mean(0) for c in range(k)])
    intra = np.array([np.linalg.norm(X[lab == c] - cent[c], axis=1).mean() for c in range(k)])
    cd = np.linalg.norm(cent[:, None, :] - cent[None, :, :], axis=2)
    if np.allclose(intra, 0) or np.allclose(cd, 0):
        return 0.0
    cd[cd == 0] = np.inf
    return float(np.mean(np.max((intra[:, None] + intra[None, :]) / cd, axis=1)))


def calinski_harabasz_score(X, labels):
    X = np.asarray(X, dtype=np.float64)
    lab, k = _encode(labels)
    n = X.shape[0]
    mean = X.mean(0)
    extra, intra = 0.0, 0.0
    for c in range(k):
        xc = X[lab == c]
        mc = xc.mean(0)
        extra += len(xc) * ((mc - mean) ** 2).sum()
        intra += ((xc - mc) ** 2).sum()
    return float(1.0 if intra == 0.0 else extra * (n - k) / (intra * (k - 1.0)))
