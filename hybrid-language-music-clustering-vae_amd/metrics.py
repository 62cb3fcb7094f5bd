"""Clustering evaluation metrics of the reference's k sweep and final report.

GPU (libhlmc metrics kernels):
  silhouette_score / silhouette_samples  sklearn.metrics (metric "euclidean"): src/Convolutional_VAE.py:320,
                                         337,361,399; src/Conditional_VAE.py:298; src/Simple_VAE.py:247,256,262
  davies_bouldin_score                   src/Convolutional_VAE.py:400
  calinski_harabasz_score                src/Simple_VAE.py:257,263
Host (label-only contingency arithmetic on n integers, nothing GPU-shaped):
  adjusted_rand_score, normalized_mutual_info_score   src/Conditional_VAE.py:299-300, src/Convolutional_VAE.py:402
  calculate_purity                                    src/Conditional_VAE.py:279-293

Labels may be any integer / string array: they are encoded to 0..k-1 in sorted order (sklearn's
LabelEncoder) on the host.  X is float32 [n, d] (a torch tensor on the GPU, or anything numpy accepts,
which is uploaded).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib as L


def _encode(labels):
    lab = labels.detach().cpu().numpy() if torch.is_tensor(labels) else np.asarray(labels)
    classes, enc = np.unique(lab, return_inverse=True)
    return enc.astype(np.int32).reshape(-1), len(classes)


def _device_x(X, device=None):
    if torch.is_tensor(X):
        dev = X.device if X.is_cuda else torch.device(device or "cuda")
        return X.detach().to(device=dev, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.asarray(X, dtype=np.float32), device=device or "cuda").contiguous()


def _prepare(X, labels):
    x = _device_x(X)
    if x.dim() != 2:
        raise ValueError("X must be 2-D [n_samples, n_features]")
    enc, k = _encode(labels)
    if enc.shape[0] != x.shape[0]:
        raise ValueError(f"X has {x.shape[0]} rows but labels has {enc.shape[0]} entries")
    n = x.shape[0]
    if not 2 <= k <= n - 1:  # sklearn check_number_of_labels
        raise ValueError(f"Number of labels is {k}. Valid values are 2 to n_samples - 1 (inclusive)")
    return x, torch.from_numpy(enc).to(x.device), k


def silhouette_samples(X, labels, *, metric="euclidean"):
    """Per-sample silhouette coefficients (float64 tensor on the GPU), sklearn semantics."""
    if metric != "euclidean":
        raise ValueError("only metric='euclidean' (the reference's) is implemented")
    x, lab, k = _prepare(X, labels)
    n, d = x.shape
    lib = L.lib()
    ws = torch.empty(int(lib.hlmc_silhouette_workspace(n, k)), dtype=torch.uint8, device=x.device)
    out = torch.empty(n, dtype=torch.float64, device=x.device)
    score = torch.empty(1, dtype=torch.float64, device=x.device)
    L.check(lib.hlmc_silhouette(L.stream(), x.data_ptr(), n, d, lab.data_ptr(), k, out.data_ptr(), score.data_ptr(),
                                ws.data_ptr(), ws.numel()), "hlmc_silhouette")
    return out


def silhouette_score(X, labels, *, metric="euclidean", sample_size=None, random_state=None):
    """Mean silhouette coefficient over all samples (sklearn.metrics.silhouette_score)."""
    if metric != "euclidean":
        raise ValueError("only metric='euclidean' (the reference's) is implemented")
    if sample_size is not None:  # sklearn: random subset without replacement, then the same score
        rs = np.random.RandomState(random_state) if not isinstance(random_state, np.random.RandomState) else random_state
        n = X.shape[0]
        idx = rs.permutation(n)[:sample_size]
        lab = labels.detach().cpu().numpy() if torch.is_tensor(labels) else np.asarray(labels)
        X = X[torch.as_tensor(idx, device=X.device)] if torch.is_tensor(X) else np.asarray(X)[idx]
        labels = lab[idx]
    x, lab, k = _prepare(X, labels)
    n, d = x.shape
    lib = L.lib()
    ws = torch.empty(int(lib.hlmc_silhouette_workspace(n, k)), dtype=torch.uint8, device=x.device)
    score = torch.empty(1, dtype=torch.float64, device=x.device)
    L.check(lib.hlmc_silhouette(L.stream(), x.data_ptr(), n, d, lab.data_ptr(), k, None, score.data_ptr(),
                                ws.data_ptr(), ws.numel()), "hlmc_silhouette")
    return float(score.item())


def _cluster_scores(X, labels):
    x, lab, k = _prepare(X, labels)
    n, d = x.shape
    lib = L.lib()
    ws = torch.empty(int(lib.hlmc_cluster_scores_workspace(k, d)), dtype=torch.uint8, device=x.device)
    out = torch.empty(2, dtype=torch.float64, device=x.device)
    L.check(lib.hlmc_cluster_scores(L.stream(), x.data_ptr(), n, d, lab.data_ptr(), k, out.data_ptr(), ws.data_ptr(),
                                    ws.numel()), "hlmc_cluster_scores")
    return out.cpu().tolist()


def davies_bouldin_score(X, labels):
    """sklearn.metrics.davies_bouldin_score (lower is better)."""
    return _cluster_scores(X, labels)[0]


def calinski_harabasz_score(X, labels):
    """sklearn.metrics.calinski_harabasz_score (higher is better)."""
    return _cluster_scores(X, labels)[1]


# ---------------------------------------------------------------- label-only scores (host)
def _contingency(a, b):
    ea, _ = _encode(a)
    eb, _ = _encode(b)
    na, nb = ea.max() + 1, eb.max() + 1
    c = np.zeros((na, nb), dtype=np.int64)
    np.add.at(c, (ea, eb), 1)
    return c


def _comb2(x):
    x = np.asarray(x, dtype=np.int64)
    return (x * (x - 1) // 2).sum()


def adjusted_rand_score(labels_true, labels_pred):
    """sklearn.metrics.adjusted_rand_score: pair-confusion counts in int64, float64 finish."""
    c = _contingency(labels_true, labels_pred)
    n = int(c.sum())
    sum_sq = int((c * c).sum())
    n_c, n_k = c.sum(1), c.sum(0)
    tp = sum_sq - n
    fp = int((c * n_k[None, :]).sum()) - sum_sq
    fn = int((c * n_c[:, None]).sum()) - sum_sq
    tn = n * n - fp - fn - sum_sq
    if fn == 0 and fp == 0:
        return 1.0
    return 2.0 * (tp * tn - fn * fp) / ((tp + fn) * (fn + tn) + (tp + fp) * (fp + tn))


def _entropy(counts):
    p = counts[counts > 0].astype(np.float64)
    if p.size <= 1:
        return 0.0
    tot = p.sum()
    return float(-np.sum((p / tot) * (np.log(p) - np.log(tot))))


def normalized_mutual_info_score(labels_true, labels_pred, *, average_method="arithmetic"):
    """sklearn.metrics.normalized_mutual_info_score (natural log; arithmetic-mean normaliser by default)."""
    c = _contingency(labels_true, labels_pred)
    if c.shape[0] == c.shape[1] == 1:
        return 1.0
    pi, pj = c.sum(1), c.sum(0)
    if pi.size == 1 or pj.size == 1:
        return 0.0
    nzx, nzy = np.nonzero(c)
    nz = c[nzx, nzy].astype(np.float64)
    tot = float(c.sum())
    cnm = nz / tot
    outer = pi[nzx].astype(np.int64) * pj[nzy].astype(np.int64)
    log_outer = -np.log(outer) + np.log(float(pi.sum())) + np.log(float(pj.sum()))
    mi = cnm * (np.log(nz) - np.log(tot)) + cnm * log_outer
    mi = np.where(np.abs(mi) < np.finfo(np.float64).eps, 0.0, mi)
    mi = float(np.clip(mi.sum(), 0.0, None))
    if mi == 0.0:
        return 0.0
    h_true, h_pred = _entropy(pi), _entropy(pj)
    if average_method == "arithmetic":
        norm = (h_true + h_pred) / 2.0
    elif average_method == "geometric":
        norm = math.sqrt(h_true * h_pred)
    elif average_method == "min":
        norm = min(h_true, h_pred)
    elif average_method == "max":
        norm = max(h_true, h_pred)
    else:
        raise ValueError("average_method must be 'min', 'geometric', 'arithmetic' or 'max'")
    return float(mi / norm)


def calculate_purity(y_true, y_pred):
    """Cluster purity (the reference's own helper, src/Conditional_VAE.py:279-293): sum over clusters of the
    largest true-class count, divided by n."""
    c = _contingency(y_pred, y_true)
    return float(c.max(axis=1).sum() / c.sum())
