"""KMeans (sklearn semantics) with the distance / assign / update work on the GPU.

Replaces ``sklearn.cluster.KMeans(n_clusters=k, random_state=42, n_init=10).fit_predict`` at
src/Convolutional_VAE.py:317-319,379-380, src/Conditional_VAE.py:293-295 (and the n_init='auto'
call at :528), src/Simple_VAE.py:244-261.

Host (this file) keeps exactly what sklearn 1.7.2 does on the host side: one numpy RandomState stream
across all inits, k-means++ candidate draws (``choice``, ``uniform * pot``, float64 cumsum +
searchsorted), potentials as float32 BLAS dot products, the best-of-n_init rule with
``_is_same_clustering``, empty-cluster relocation, centre averaging (float32 ``*= 1/w``),
centre shifts and the strict / tolerance convergence tests.  Device kernels (libhlmc) compute the
numpy-order column mean/variance, the float64-upcast candidate distances, the float32 E-step
(||c||^2 - 2 x.c, first minimum) in the exact rounding order of sklearn's einsum row norms and its OpenBLAS
sgemm call (oracle/kmeans_oracle.py estep_dist), per-cluster sums in sklearn's single-thread row order, and
inertia.

Multi-GPU (``process_group=``): the n_init restarts are independent objects, so they shard across ranks
with no collective on the data path.  Every rank holds the same (small, [N, D] f32) latents and runs the
k-means++ seeding and Lloyd iterations of restarts ``i % world == rank`` only.  sklearn draws every restart's
seeds from one RandomState stream; a seeding consumes a data-independent number of doubles
(``seeding_draws``), so a rank skips another rank's seeding by drawing and discarding exactly that many and
its own restarts see the same random numbers as in a single process.  One ``all_gather_object`` of (restart,
labels, inertia, centres, n_iter) at the end feeds sklearn's sequential best-of rule in restart order, so the
result is bit-identical for any world size.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L


def _is_same_clustering(a, b, k):
    mapping = np.full(k, -1, dtype=np.int64)
    for x, y in zip(a, b):
        if mapping[x] == -1:
            mapping[x] = y
        elif mapping[x] != y:
            return False
    return True


def _euclid_f32(a, b):
    """sklearn _euclidean_dense_dense (float32, 4-element groups, no FMA) for each row pair."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    d = a.shape[-1]
    q = d // 4
    r = np.zeros(a.shape[:-1], np.float32)
    for g in range(q):
        s = (a[..., 4 * g] - b[..., 4 * g]) * (a[..., 4 * g] - b[..., 4 * g])
        s = s + (a[..., 4 * g + 1] - b[..., 4 * g + 1]) * (a[..., 4 * g + 1] - b[..., 4 * g + 1])
        s = s + (a[..., 4 * g + 2] - b[..., 4 * g + 2]) * (a[..., 4 * g + 2] - b[..., 4 * g + 2])
        s = s + (a[..., 4 * g + 3] - b[..., 4 * g + 3]) * (a[..., 4 * g + 3] - b[..., 4 * g + 3])
        r = r + s
    for c in range(4 * q, d):
        r = r + (a[..., c] - b[..., c]) * (a[..., c] - b[..., c])
    return r


class KMeans:
    def __init__(self, n_clusters=8, *, init="k-means++", n_init="auto", max_iter=300, tol=1e-4, verbose=0,
                 random_state=None, copy_x=True, algorithm="lloyd", device=None, process_group=None):
        if init != "k-means++" or algorithm not in ("lloyd", "auto"):
            raise ValueError("only init='k-means++', algorithm='lloyd' are implemented (the reference's defaults)")
        self.n_clusters, self.init, self.n_init, self.max_iter, self.tol = n_clusters, init, n_init, max_iter, tol
        self.verbose, self.random_state, self.copy_x, self.algorithm = verbose, random_state, copy_x, algorithm
        self.device = device
        self.process_group = process_group

    # ------------------------------------------------------------------ device helpers
    def _dev(self):
        return torch.device(self.device) if self.device is not None else torch.device("cuda", torch.cuda.current_device())

    def _center(self, Xd):
        n, d = Xd.shape
        mean = torch.empty(d, dtype=torch.float32, device=Xd.device)
        var = torch.empty(d, dtype=torch.float32, device=Xd.device)
        Xc = torch.empty_like(Xd)
        L.check(L.lib().hlmc_km_center(L.stream(), Xd.data_ptr(), n, d, mean.data_ptr(), var.data_ptr(),
                                       Xc.data_ptr()), "hlmc_km_center")
        return mean, var, Xc

    def _sqdist(self, Xc, cand):
        n, d = Xc.shape
        out = torch.empty(len(cand), n, dtype=torch.float32, device=Xc.device)
        L.check(L.lib().hlmc_km_sqdist_rows(L.stream(), Xc.data_ptr(), n, d, L.i64_array(cand), len(cand),
                                            out.data_ptr()), "hlmc_km_sqdist_rows")
        return out

    def _kmeans_plusplus(self, Xc, rs, w):
        n, d = Xc.shape
        k = self.n_clusters
        trials = 2 + int(np.log(k))
        cid = rs.choice(n, p=w / w.sum())
        idx = np.full(k, -1, dtype=int)
        idx[0] = cid
        closest = self._sqdist(Xc, [cid]).cpu().numpy()          # [1, n] float32
        pot = closest @ w
        for c in range(1, k):
            rand_vals = rs.uniform(size=trials) * pot
            cand = np.searchsorted(np.cumsum(w * closest, axis=None, dtype=np.float64), rand_vals)
            np.clip(cand, None, closest.size - 1, out=cand)
            dist = self._sqdist(Xc, [int(x) for x in cand]).cpu().numpy()
            np.minimum(closest, dist, out=dist)
            cpot = dist @ w.reshape(-1, 1)
            best = int(np.argmin(cpot))
            pot = cpot[best]
            closest = dist[best]
            idx[c] = cand[best]
        return Xc[torch.as_tensor(idx, device=Xc.device)].contiguous(), idx

    def _lloyd(self, Xc, centers, tol):
        n, d = Xc.shape
        k = self.n_clusters
        dev = Xc.device
        labels = torch.full((n,), -1, dtype=torch.int32, device=dev)
        labels_new = torch.empty_like(labels)
        # one device buffer [sums k*d | weights k | changed (int32 bits)]: one copy back per iteration
        pack = torch.empty(k * d + k + 1, dtype=torch.float32, device=dev)
        sums, wts = pack[:k * d], pack[k * d:k * d + k]
        changed = pack[k * d + k:].view(torch.int32)
        # M-step workspace: per-tile cluster histograms + bases, cluster offsets, the label-partitioned row list
        ws_bytes = int(L.lib().hlmc_km_sums_workspace(n, k))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        old_c = centers.cpu().numpy()
        strict = False
        it = 0
        for it in range(self.max_iter):
            changed.zero_()
            L.check(L.lib().hlmc_km_assign(L.stream(), Xc.data_ptr(), n, d, centers.data_ptr(), k,
                                           labels_new.data_ptr(), labels.data_ptr(), changed.data_ptr()))
            L.check(L.lib().hlmc_km_sums_part(L.stream(), Xc.data_ptr(), n, d, labels_new.data_ptr(), k,
                                              sums.data_ptr(), wts.data_ptr(), ws.data_ptr(), ws_bytes))
            pack_h = pack.cpu().numpy()
            new = pack_h[:k * d].reshape(k, d)
            wic = pack_h[k * d:k * d + k]
            n_changed = int(pack_h[k * d + k:].view(np.int32)[0])
            empty = np.where(wic == 0)[0]
            if empty.size:
                # _relocate_empty_clusters_dense (sklearn/cluster/_k_means_common.pyx) ranks rows by the numpy
                # expression ((X - C[labels])**2).sum(axis=1) (pairwise row sums): evaluated here on host copies
                # exactly as written, so near-tied farthest points resolve as in sklearn (empty clusters are rare)
                lab_h = labels_new.cpu().numpy()
                Xh = Xc.cpu().numpy()
                dist = ((Xh - old_c[lab_h]) ** 2).sum(axis=1)
                if dist.max() > 0:
                    far = np.argpartition(dist, -empty.size)[:-empty.size - 1:-1]
                    rows = Xh[far]
                    for e, f, xr in zip(empty, far, rows):
                        old = lab_h[f]
                        new[old] -= xr
                        new[e] = xr
                        wic[e] = 1.0
                        wic[old] -= 1.0
            amax = int(np.argmax(wic))
            for j in range(k):
                if wic[j] > 0:
                    new[j] *= np.float32(1.0 / float(wic[j]))
                else:
                    new[j] = new[amax]
            shift = np.sqrt(_euclid_f32(new, old_c)).astype(np.float32)
            centers = torch.from_numpy(new).to(dev)
            old_c = new
            labels, labels_new = labels_new, labels
            if n_changed == 0 and it > 0:
                strict = True
                break
            if (shift ** 2).sum() <= tol:
                break
        if not strict:
            L.check(L.lib().hlmc_km_assign(L.stream(), Xc.data_ptr(), n, d, centers.data_ptr(), k,
                                           labels.data_ptr(), None, None))
        inertia = torch.empty(1, dtype=torch.float32, device=dev)
        tmp = torch.empty(n, dtype=torch.float32, device=dev)
        L.check(L.lib().hlmc_km_inertia(L.stream(), Xc.data_ptr(), n, d, centers.data_ptr(), labels.data_ptr(),
                                        inertia.data_ptr(), tmp.data_ptr()))
        return labels, float(inertia.item()), centers, it + 1

    @staticmethod
    def seeding_draws(k):
        """Doubles one k-means++ seeding takes from the RandomState stream: choice(n, p) draws one, then each of
        the k - 1 further centres draws n_local_trials = 2 + int(ln k) (uniform(size=trials)); the count does
        not depend on the data."""
        return 1 + (k - 1) * (2 + int(np.log(k)))

    @staticmethod
    def _select_best(runs, k):
        """sklearn's best-of-n_init rule applied in restart order (sklearn/cluster/_kmeans.py, KMeans.fit):
        a later restart wins only with strictly lower inertia AND a different partition."""
        best = None
        for r in runs:
            if best is None or (r[2] < best[2] and not _is_same_clustering(r[1], best[1], k)):
                best = r
        return best

    # ------------------------------------------------------------------ sklearn API
    def fit(self, X, y=None, sample_weight=None):
        if sample_weight is not None:
            raise ValueError("sample_weight is not supported (the reference never passes it)")
        dev = self._dev()
        Xd = torch.as_tensor(np.asarray(X, dtype=np.float32) if not torch.is_tensor(X) else X, device=dev)
        Xd = Xd.to(torch.float32).contiguous()
        n, d = Xd.shape
        if n < self.n_clusters:
            raise ValueError(f"n_samples={n} should be >= n_clusters={self.n_clusters}")
        mean, var, Xc = self._center(Xd)
        tol = np.mean(var.cpu().numpy()) * self.tol if self.tol else 0.0
        rs = self.random_state if isinstance(self.random_state, np.random.RandomState) \
            else np.random.RandomState(self.random_state)
        n_init = 1 if self.n_init == "auto" else int(self.n_init)
        w = np.ones(n, dtype=np.float32)
        world, rank = 1, 0
        if self.process_group is not None:
            world = dist.get_world_size(self.process_group)
            rank = dist.get_rank(self.process_group)
        runs = []
        draws = self.seeding_draws(self.n_clusters)
        for i in range(n_init):
            if i % world != rank:
                # another rank's restart: advance the one RandomState stream past its seeding (a fixed count of
                # doubles) instead of computing it, so every rank seeds only its own restarts
                rs.random_sample(draws)
                continue
            c0, _ = self._kmeans_plusplus(Xc, rs, w)
            labels, inertia, centers, n_iter = self._lloyd(Xc, c0, tol)
            runs.append((i, labels.cpu().numpy(), inertia, centers.cpu().numpy(), n_iter))
        if world > 1:
            gathered = [None] * world
            dist.all_gather_object(gathered, runs, group=self.process_group)
            runs = sorted((r for part in gathered for r in part), key=lambda r: r[0])
        best = self._select_best(runs, self.n_clusters)
        self.labels_ = best[1].astype(np.int32)
        self.inertia_ = best[2]
        self.cluster_centers_ = best[3] + mean.cpu().numpy()
        self.n_iter_ = best[4]
        self.n_features_in_ = d
        return self

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).labels_

    def predict(self, X):
        dev = self._dev()
        Xd = torch.as_tensor(np.asarray(X, dtype=np.float32) if not torch.is_tensor(X) else X, device=dev)
        Xd = Xd.to(torch.float32).contiguous()
        n, d = Xd.shape
        C_ = torch.as_tensor(self.cluster_centers_, device=dev).contiguous()
        labels = torch.empty(n, dtype=torch.int32, device=dev)
        L.check(L.lib().hlmc_km_assign(L.stream(), Xd.data_ptr(), n, d, C_.data_ptr(), self.n_clusters,
                                       labels.data_ptr(), None, None))
        return labels.cpu().numpy()
