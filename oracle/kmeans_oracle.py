"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy restatement of sklearn KMeans / StandardScaler.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use this.

Reference call sites (the algorithms themselves live in scikit-learn, a third-party dependency the
reference leaves unpinned, >=1.2 for ``OneHotEncoder(sparse_output=)``; restated here from the
installed scikit-learn 1.7.2 with the OpenBLAS 0.3.28 (SkylakeX kernels) that scipy bundles):
  * ``KMeans(n_clusters=k, random_state=42, n_init=10).fit_predict`` —
    src/Convolutional_VAE.py:317-319, 379-380; src/Conditional_VAE.py:293-295; src/Simple_VAE.py:244-261
  * ``KMeans(k, random_state=42)`` (n_init='auto' -> 1 for k-means++) — src/Conditional_VAE.py:528
  * ``StandardScaler().fit_transform`` — src/1_preprocessing.py:310-311; src/1_preprocessing_advanced.py:376-391
sklearn semantics restated (sklearn/cluster/_kmeans.py, _k_means_lloyd.pyx, _k_means_common.pyx), single
thread (threadpoolctl limits=1, as the fixtures are generated):
  X (float32) is mean-centred; tol = mean(var(X, axis=0)) * 1e-4; per init one shared RandomState
  stream: k-means++ (first centre ``choice(N, p=w/sum w)``, then per centre ``uniform(size=2+int(ln k))
  * pot`` -> searchsorted(float64 cumsum) -> candidates; distances in float64 rounded to float32);
  Lloyd: dist = ||c||^2 - 2 x.c (float32), first-minimum argmin, empty clusters relocated to the
  farthest points, centres = sum / w, stop on identical labels or sum(shift^2) <= tol, max_iter 300;
  if not strictly converged a final E-step; keep the best inertia unless it is the same clustering.

The Lloyd E-step is restated at the bit level (``estep_dist``), because labels are decided by float32
rounding wherever two centres are nearly equidistant (overlapping clusters, real latents):
  * ||c||^2 = ``np.einsum("ij,ij->i", C, C)`` (sklearn row_norms): numpy's baseline-SSE loop, 4 lanes, each
    16-element block added as blocks 3, 2, 1, 0 with a separate multiply and add, zero-filled tail
    vectors, then (l0 + l1) + (l2 + l3);
  * x.c: ``_update_chunk_dense`` calls sgemm per 256-row chunk as column-major TN with M = k, N = rows,
    K = d, alpha = -2, beta = 1 on a buffer holding ||c||^2.  OpenBLAS takes its small-matrix TN kernel
    when M*N <= 1200, K >= 32 and M*N*K <= 1e6: 16 float32 lanes (lane l sums k = l, l+16, ... with fma),
    reduced by an adjacent-pair tree, except elements in both the M and the N remainder of 4 (a single
    ``_mm512_reduce_add_ps``: halves first).  Otherwise its regular kernel: one sequential fma chain over
    k.  Then dist = ||c||^2 + (-2 * dot) with one rounding.
  ``estep_dist_blas`` makes the very sgemm call sklearn makes (scipy's BLAS); tests pin the restatement to
  it on near-tie data.  M-step sums: sequential float32 per cluster in row order (one thread's
  ``centers_new_chunk``), counts exact.
Pinned against sklearn's own output in tests/golden/kmeans_*.npz (labels bit-identical).
"""
from __future__ import annotations

import numpy as np

CHUNK = 256
f32 = np.float32


# ----------------------------------------------------------------------------- E-step arithmetic
def row_norms_sq_f32(C: np.ndarray) -> np.ndarray:
    """np.einsum('ij,ij->i', C, C) for float32 C (numpy baseline-SSE sum_of_products, outstride 0)."""
    C = np.asarray(C, f32)
    k, d = C.shape
    acc = np.zeros((k, 4), f32)
    i = 0
    while d - i >= 16:
        for t in (3, 2, 1, 0):
            a = C[:, i + 4 * t:i + 4 * t + 4]
            acc = (a * a).astype(f32) + acc
        i += 16
    while i < d:
        a = np.zeros((k, 4), f32)
        m = min(4, d - i)
        a[:, :m] = C[:, i:i + m]
        acc = (a * a).astype(f32) + acc
        i += 4
    return ((acc[:, 0] + acc[:, 1]).astype(f32) + (acc[:, 2] + acc[:, 3]).astype(f32)).astype(f32)


def _fma(a, b, c):
    """float32 fused multiply-add (the f32 x f32 product is exact in float64)."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def _tree_adjacent(v):
    while v.shape[-1] > 1:
        v = (v[..., 0::2] + v[..., 1::2]).astype(f32)
    return v[..., 0]


def _tree_halves(v):
    while v.shape[-1] > 1:
        h = v.shape[-1] // 2
        v = (v[..., :h] + v[..., h:]).astype(f32)
    return v[..., 0]


def sgemm_small_path(k: int, rows: int, d: int) -> bool:
    """OpenBLAS (SkylakeX) small-matrix permit for sklearn's TN sgemm call (M = k, N = rows, K = d)."""
    return k * rows <= 1200 and d >= 32 and float(k) * rows * d <= 1e6


def estep_dist(Xc: np.ndarray, C: np.ndarray, cn: np.ndarray) -> np.ndarray:
    """float32 ||c||^2 - 2 x.c of one sklearn chunk (rows of Xc), bit-exact restatement of the sgemm call."""
    N, d = Xc.shape
    k = C.shape[0]
    if sgemm_small_path(k, N, d):
        dp = (d + 15) // 16 * 16
        Xp = np.zeros((N, dp), f32)
        Xp[:, :d] = Xc
        Cp = np.zeros((k, dp), f32)
        Cp[:, :d] = C
        acc = np.zeros((N, k, 16), f32)
        for b in range(0, dp, 16):
            acc = _fma(Xp[:, None, b:b + 16], Cp[None, :, b:b + 16], acc)
        s = _tree_adjacent(acc.copy())
        n4, k4 = 4 * (N // 4), 4 * (k // 4)
        if n4 < N and k4 < k:
            s[n4:, k4:] = _tree_halves(acc[n4:, k4:].copy())
    else:
        s = np.zeros((N, k), f32)
        for t in range(d):
            s = _fma(Xc[:, None, t], C[None, :, t], s)
    return (cn[None, :] + (f32(-2.0) * s).astype(f32)).astype(f32)


def estep_dist_blas(Xc: np.ndarray, C: np.ndarray, cn: np.ndarray) -> np.ndarray:
    """The chunk's distances through the very BLAS call sklearn makes (scipy's sgemm, column-major TN)."""
    from scipy.linalg import blas
    pd = np.asfortranarray(np.tile(cn, (Xc.shape[0], 1)).T)
    return blas.sgemm(-2.0, np.asfortranarray(C.T), np.asfortranarray(Xc.T), beta=1.0, c=pd,
                      trans_a=1, trans_b=0).T


def assign_labels(X: np.ndarray, centers: np.ndarray, dist_fn=estep_dist) -> np.ndarray:
    """lloyd_iter_chunked_dense(update_centers=False): 256-row chunks, first-minimum argmin."""
    X = np.asarray(X, f32)
    C = np.asarray(centers, f32)
    cn = row_norms_sq_f32(C)
    out = [np.argmin(dist_fn(X[s:s + CHUNK], C, cn), axis=1) for s in range(0, X.shape[0], CHUNK)]
    return np.concatenate(out).astype(np.int32)


def cluster_sums_f32(X: np.ndarray, labels: np.ndarray, k: int):
    """Per-cluster float32 sums added in row order (one accumulator per column) and exact counts."""
    order = np.argsort(labels, kind="stable")
    Xs = np.asarray(X, f32)[order]
    ls = labels[order]
    sums = np.zeros((k, X.shape[1]), f32)
    counts = np.bincount(labels, minlength=k).astype(f32)
    start = 0
    for j in range(k):
        m = int(counts[j])
        if m:
            sums[j] = np.add.accumulate(Xs[start:start + m], axis=0)[-1]
        start += m
    assert start == len(ls)
    return sums, counts


def euclidean_dense_dense_sq(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """sklearn _euclidean_dense_dense(squared=True): float32, 4-element groups summed left to right, tail."""
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    d = a.shape[-1]
    q = d // 4
    r = np.zeros(np.broadcast(a[..., 0], b[..., 0]).shape, f32)
    for g in range(q):
        e = [(a[..., 4 * g + t] - b[..., 4 * g + t]).astype(f32) for t in range(4)]
        s = (e[0] * e[0]).astype(f32) + (e[1] * e[1]).astype(f32)
        s = (s + (e[2] * e[2]).astype(f32)).astype(f32)
        s = (s + (e[3] * e[3]).astype(f32)).astype(f32)
        r = (r + s).astype(f32)
    for c in range(4 * q, d):
        e = (a[..., c] - b[..., c]).astype(f32)
        r = (r + (e * e).astype(f32)).astype(f32)
    return r


def _sqdist_upcast(A: np.ndarray, X: np.ndarray) -> np.ndarray:
    """sklearn _euclidean_distances_upcast: float64 (-2 a.x + ||a||^2) + ||x||^2, clipped at 0, float32."""
    A64 = A.astype(np.float64)
    X64 = X.astype(np.float64)
    d = -2.0 * (A64 @ X64.T)
    d += np.einsum("ij,ij->i", A64, A64)[:, None]
    d += np.einsum("ij,ij->i", X64, X64)[None, :]
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


def _lloyd_iter(X, w, centers, labels, update=True):
    k, D = centers.shape
    labels[:] = assign_labels(X, centers)
    if not update:
        return None, None, None
    new, wic = cluster_sums_f32(X, labels, k)
    empty = np.where(wic == 0)[0]
    if empty.size:
        # _relocate_empty_clusters_dense: numpy expression (pairwise row sums)
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
            new[j] *= np.float32(1.0 / float(wic[j]))
        else:
            new[j] = new[amax]
    shift = np.sqrt(euclidean_dense_dense_sq(new, centers))
    return new, wic, shift


def inertia_f32(X, centers, labels) -> float:
    """_inertia_dense, one thread: float32 sequential sum of _euclidean_dense_dense over rows."""
    r = euclidean_dense_dense_sq(X, centers[labels])
    return float(np.add.accumulate(r)[-1])


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
    return labels, inertia_f32(X, centers, labels), centers, i + 1


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
