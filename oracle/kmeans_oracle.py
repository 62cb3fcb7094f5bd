"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy restatement of sklearn KMeans / StandardScaler.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use this.

Reference call sites (the algorithms themselves live in scikit-learn, a third-party dependency the
reference leaves unpinned, >=1.2 for ``OneHotEncoder(sparse_output=)``; restated here from the
installed scikit-learn 1.7.2):
  * ``KMeans(n_clusters=k, random_state=42, n_init=10).fit_predict`` —
    src/Convolutional_VAE.py:317-319, 379-380; src/Conditional_VAE.py:293-295; src/Simple_VAE.py:244-261
  * ``KMeans(k, random_state=42)`` (n_init='auto' -> 1 for k-means++) — src/Conditional_VAE.py:528
  * ``StandardScaler().fit_transform`` — src/1_preprocessing.py:310-311; src/1_preprocessing_advanced.py:376-391
sklearn semantics restated (sklearn/cluster/_kmeans.py, _k_means_lloyd.pyx, _k_means_common.pyx):
  X (float32) is mean-centred; tol = mean(var(X, axis=0)) * 1e-4; per init one shared RandomState
  stream: k-means++ (first centre ``choice(N, p=w/sum w)``, then per centre ``uniform(size=2+int(ln k))
  * pot`` -> searchsorted(float64 cumsum) -> candidates; distances in float64 rounded to float32);
  Lloyd: dist = ||c||^2 - 2 x.c (float32), first-minimum argmin, empty clusters relocated to the
  farthest points, centres = sum / w, stop on identical labels or sum(shift^2) <= tol, max_iter 300;
  if not strictly converged a final E-step; keep the best inertia unless it is the same clustering.
Pinned against sklearn's own output in tests/golden/kmeans_*.npz (labels bit-identical).
"""
from __future__ import annotations

import numpy as np

CHUNK = 256


def _sqdist_upcast(A: np.ndarray, X: np.ndarray) -> np.ndarray:
    """sklearn _euclidean_distances_upcast: float64 ||a||^2 - 2 a.x + ||x||^2, clipped at 0, float32."""
    A64 = A.astype(np.float64)
    X64 = X.astype(np.float64)
    d = -2.0 * (A64 @ X64.T)
    d += (A64 * A64).sum(1)[:, None]
    d += (X64 * X64).sum(1)[None, :]
    return np.maximum(d.astype(np.float32), np.float32(0))


def kmeans_plusplus(X: np.ndarray, k: int, rs: np.random.RandomState, w: np.ndarray | None = None):
    n = X.shape[0]
    w = np.ones(n, dtype=X.dtype) if w is None else w
    trials = 2 + int(np.log(k))
    cid = rs.choice(n, p=w / w.sum())
    idx = np.full(k, -1, dtype=int)
    centers = np.empty((k, X.shape[1]), dtype=X.dtype)
    centers[0], idx[0] = X[cid], cid
    closest = _sqdist_upcast(X[cid][None, :], X)          # [1, n] f32
    pot = closest @ w
    for c in range(1, k):
        r = rs.uniform(size=trials) * pot
        cand = np.searchsorted(np.cumsum((w * closest).astype(np.float64), dtype=np.float64), r)
        np.clip(cand, None, closest.size - 1, out=cand)
        dc = _sqdist_upcast(X[cand], X)
        np.minimum(closest, dc, out=dc)
        cpot = dc @ w.reshape(-1, 1)
        best = int(np.argmin(cpot))
        pot = cpot[best]
        closest = dc[best]
        centers[c], idx[c] = X[cand[best]], cand[best]
    return centers, idx


def assign_labels(X: np.ndarray, centers: np.ndarray) -> np.ndarray:
    """E-step in float32: ||c||^2 - 2 x.c, first-minimum argmin."""
    cn = np.einsum("ij,ij->i", centers, centers)
    d = cn[None, :] + np.float32(-2.0) * (X @ centers.T)
    return np.argmin(d, axis=1).astype(np.int32)


def _lloyd_iter(X, w, centers, labels, update=True):
    k, D = centers.shape
    labels[:] = assign_labels(X, centers)
    if not update:
        return None, None, None
    new = np.zeros((k, D), np.float64)
    wic = np.zeros(k, np.float64)
    np.add.at(new, labels, X.astype(np.float64) * w[:, None])
    np.add.at(wic, labels, w.astype(np.float64))
    new = new.astype(np.float32)
    wic = wic.astype(np.float32)
    empty = np.where(wic == 0)[0]
    if empty.size:
        dist = ((X - centers[labels]) ** 2).sum(axis=1)
        if dist.max() > 0:
            far = np.argpartition(dist, -empty.size)[:-empty.size - 1:-1]
            for e, f in zip(empty, far):
                old = labels[f]
                new[old] -= X[f] * w[f]
                new[e] = X[f] * w[f]
                wic[e] = w[f]
                wic[old] -= w[f]
    amax = int(np.argmax(wic))
    for j in range(k):
        if wic[j] > 0:
            new[j] *= np.float32(1.0) / wic[j]
        else:
            new[j] = new[amax]
    shift = np.sqrt(((new - centers) ** 2).sum(1))
    return new, wic, shift


def kmeans_single_lloyd(X, w, centers, max_iter=300, tol=0.0):
    labels = np.full(X.shape[0], -1, np.int32)
    labels_old = labels.copy()
    strict = False
    for i in range(max_iter):
        new, _, shift = _lloyd_iter(X, w, centers, labels)
        centers = new
        if np.array_equal(labels, labels_old):
            strict = True
            break
        if (shift ** 2).sum() <= tol:
            break
        labels_old[:] = labels
    if not strict:
        _lloyd_iter(X, w, centers, labels, update=False)
    inertia = float(((X - centers[labels]).astype(np.float32) ** 2).sum(1) @ w)
    return labels, inertia, centers, i + 1


def is_same_clustering(a, b, k):
    mapping = np.full(k, -1)
    for x, y in zip(a, b):
        if mapping[x] == -1:
            mapping[x] = y
        elif mapping[x] != y:
            return False
    return True


class KMeans:
    """sklearn.cluster.KMeans(init='k-means++', algorithm='lloyd') restated for dense float32 X."""

    def __init__(self, n_clusters=8, *, n_init="auto", max_iter=300, tol=1e-4, random_state=None):
        self.n_clusters, self.n_init, self.max_iter, self.tol = n_clusters, n_init, max_iter, tol
        self.random_state = random_state

    def fit(self, X):
        X = np.array(X, dtype=np.float32, copy=True, order="C")
        n_init = 1 if self.n_init == "auto" else int(self.n_init)
        rs = self.random_state if isinstance(self.random_state, np.random.RandomState) \
            else np.random.RandomState(self.random_state)
        tol = float(np.mean(np.var(X, axis=0)) * self.tol) if self.tol else 0.0
        w = np.ones(X.shape[0], dtype=np.float32)
        mean = X.mean(axis=0)
        X -= mean
        best = None
        for _ in range(n_init):
            c0, _ = kmeans_plusplus(X, self.n_clusters, rs, w)
            lab, inert, cen, nit = kmeans_single_lloyd(X, w, c0, self.max_iter, tol)
            if best is None or (inert < best[1] and not is_same_clustering(lab, best[0], self.n_clusters)):
                best = (lab, inert, cen, nit)
        self.labels_, self.inertia_, cen, self.n_iter_ = best
        self.cluster_centers_ = cen + mean
        return self

    def fit_predict(self, X):
        return self.fit(X).labels_


def standard_scaler_fit(X: np.ndarray):
    """StandardScaler.fit: float64 mean/var (ddof=0), scale_=sqrt(var) with near-constant columns -> 1."""
    X64 = np.asarray(X, dtype=np.float64)
    n = X64.shape[0]
    mean = X64.sum(0) / n
    t = X64 - mean
    corr = t.sum(0)
    var = ((t * t).sum(0) - corr * corr / n) / n
    scale = np.sqrt(var)
    eps = np.finfo(np.float64).eps
    upper = n * eps * var + (n * mean * eps) ** 2
    const = var <= upper
    scale[const] = 1.0
    return mean, var, scale


def standard_scaler_transform(X: np.ndarray, mean: np.ndarray, scale: np.ndarray) -> np.ndarray:
    """In-place float32 ``X -= mean_; X /= scale_`` as sklearn does (each op in float64, stored f32)."""
    X = np.array(X, dtype=np.float32, copy=True)
    X -= mean
    X /= scale
    return X
