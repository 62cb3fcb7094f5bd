"""KMeans (sklearn semantics) with the distance / assign / update work on the GPU.

Replaces ``sklearn.cluster.KMeans(n_clusters=k, random_state=42, n_init=10).fit_predict`` at
src/Convolutional_VAE.py:317-319,379-380, src/Conditional_VAE.py:293-295 (and the n_init='auto'
call at :528), src/Simple_VAE.py:244-261.

The n_init restarts run in lockstep on the device (round 5): every stage is one launch for all of them.
sklearn draws every restart's random numbers from one RandomState stream in a data-independent amount
(``seeding_draws``), so they are drawn up front in sklearn's order.  Device kernels (libhlmc) compute the
numpy-order column mean/variance, the k-means++ candidate draw (searchsorted of the float64 cumsum, exact
through an error bracket with a numpy fallback for undecidable draws), the float64-upcast candidate distances
and their running minimum, the float32 E-step (||c||^2 - 2 x.c, first minimum) in the exact rounding order of
sklearn's einsum row norms and its OpenBLAS sgemm call (oracle/kmeans_oracle.py estep_dist), per-cluster sums in
sklearn's single-thread row order, the centre update (float32 ``*= 1/w``) with its shifts, and inertia.  The
host keeps what sklearn's order depends on BLAS for or decides per restart: the float32 potentials (BLAS dot
products of the copied-back distances), the candidate argmin, empty-cluster relocation, the strict / tolerance
convergence tests and the best-of-n_init rule with ``_is_same_clustering``; one copy back per k-means++ step
and per Lloyd iteration serves all restarts.

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

    def _draw_seeds(self, rs, n, n_init, mine):
        """Consume the one RandomState stream exactly as sklearn's sequential restarts do (data-independent
        counts, seeding_draws): per restart the first centre's choice(n, p=w / w.sum()) and the k - 1 per-centre
        uniform(size=trials) vectors -- kept for this rank's restarts, drawn and discarded for the others."""
        k = self.n_clusters
        trials = 2 + int(np.log(k))
        w = np.ones(n, dtype=np.float32)
        # rs.choice(n, p=w / w.sum()) is one random_sample() searched in the normalised float64 cdf of p
        # (numpy mtrand.RandomState.choice); the cdf is the same for every restart, so it is built once
        cdf = np.array(w / w.sum(), dtype=np.float64).cumsum()
        cdf /= cdf[-1]
        draws = {}
        for i in range(n_init):
            if i not in mine:
                rs.random_sample(self.seeding_draws(k))
                continue
            cid = int(cdf.searchsorted(rs.random_sample(), side="right"))
            draws[i] = (cid, [rs.uniform(size=trials) for _ in range(1, k)])
        return draws, trials

    def _kmeans_plusplus_batch(self, Xc, seeds, trials):
        """sklearn _kmeans_plusplus for R restarts in lockstep (one launch per stage for all of them): the
        candidate draw (searchsorted of the float64 cumsum, hlmc_km_pp_search) and the candidates' distances with
        the running minimum (hlmc_km_pp_dist) on the device; the host keeps sklearn's float32 BLAS potentials
        (closest @ w, dist @ w: numpy on the copied-back distances) and argmin, and redoes with numpy the rare
        draws the device's error bracket flags as undecidable."""
        n, d = Xc.shape
        k, R, T = self.n_clusters, len(seeds), trials
        dev = Xc.device
        lib = L.lib()
        w = np.ones(n, dtype=np.float32)
        idx = np.full((R, k), -1, dtype=np.int64)
        idx[:, 0] = [c for c, _ in seeds]
        cand = torch.as_tensor(idx[:, 0].copy(), device=dev)
        prev = torch.empty(R, 1, n, dtype=torch.float32, device=dev)
        L.check(lib.hlmc_km_pp_dist(L.stream(), Xc.data_ptr(), n, d, R, 1, cand.data_ptr(), None, 1, None,
                                    prev.data_ptr()), "hlmc_km_pp_dist")
        prev_h = prev.cpu().numpy()
        pots = [prev_h[r] @ w for r in range(R)]               # closest_dist_sq @ sample_weight: float32 (1,)
        best = np.zeros(R, dtype=np.int32)
        bufs = [torch.empty(R, T, n, dtype=torch.float32, device=dev) for _ in range(2)]
        cand = torch.empty(R * T, dtype=torch.int64, device=dev)
        amb = torch.empty(R * T, dtype=torch.int32, device=dev)
        # two pinned host images of the distances (this step's and the previous step's closest rows)
        pins = [torch.empty(R, T, n, dtype=torch.float32).pin_memory() for _ in range(2)] if dev.type == "cuda" else None
        if pins is not None:
            cpin = torch.empty(R * T, dtype=torch.int64).pin_memory()
            apin = torch.empty(R * T, dtype=torch.int32).pin_memory()
        for c in range(1, k):
            out = bufs[c % 2]
            pin = pins[c % 2] if pins is not None else None
            rv = np.stack([seeds[r][1][c - 1] * pots[r] for r in range(R)]).astype(np.float64)   # rand_vals
            prevT = prev.shape[1]
            bh = best.ctypes.data_as(C.POINTER(C.c_int32))
            L.check(lib.hlmc_km_pp_search(L.stream(), n, R, T, prev.data_ptr(), prevT, bh,
                                          np.ascontiguousarray(rv).ctypes.data_as(C.POINTER(C.c_double)),
                                          cand.data_ptr(), amb.data_ptr()), "hlmc_km_pp_search")
            L.check(lib.hlmc_km_pp_dist(L.stream(), Xc.data_ptr(), n, d, R, T, cand.data_ptr(), prev.data_ptr(),
                                        prevT, bh, out.data_ptr()), "hlmc_km_pp_dist")
            if pin is not None:   # one synchronisation per step: the distances, candidates and flags
                pin.copy_(out, non_blocking=True)
                cpin.copy_(cand, non_blocking=True)
                apin.copy_(amb, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                cand_h, amb_h = cpin.numpy().reshape(R, T).copy(), apin.numpy().reshape(R, T)
                out_h = pin.numpy()
            else:
                cand_h, amb_h = cand.cpu().numpy().reshape(R, T), amb.cpu().numpy().reshape(R, T)
                out_h = out.cpu().numpy()
            for r in range(R):
                closest = prev_h[r, best[r]][None, :]
                dist = out_h[r]
                if amb_h[r].any():
                    # numpy's own cumsum / searchsorted for this restart's draw (the device bracket could not decide)
                    cc = np.searchsorted(np.cumsum(w * closest, axis=None, dtype=np.float64), rv[r])
                    np.clip(cc, None, closest.size - 1, out=cc)
                    cand_h[r] = cc
                    dist = self._sqdist(Xc, [int(x) for x in cc]).cpu().numpy()
                    np.minimum(closest, dist, out=dist)
                    out[r].copy_(torch.from_numpy(dist))
                    out_h[r] = dist
                cpot = dist @ w.reshape(-1, 1)
                b = int(np.argmin(cpot))
                pots[r] = cpot[b]
                best[r] = b
                idx[r, c] = cand_h[r, b]
            prev, prev_h = out, (out_h if pin is not None else out_h.copy())
        cent = Xc[torch.as_tensor(idx.reshape(-1), device=dev)].reshape(R, k, d).contiguous()
        return cent, idx

    def _lloyd_batch(self, Xc, centers, tol):
        """sklearn _kmeans_single_lloyd for R restarts in lockstep: one assign / partitioned-sums / centre-update
        launch per iteration for all running restarts, one small copy back per iteration (label-change counts,
        centre shifts, the new centres) for sklearn's host-side tests: strict convergence (labels unchanged),
        sum(shift^2) <= tol, max_iter; a restart with an empty cluster is updated on the host that iteration
        (sklearn _relocate_empty_clusters_dense on host copies, as before)."""
        n, d = Xc.shape
        k, R = self.n_clusters, centers.shape[0]
        dev = Xc.device
        lib = L.lib()
        cbuf = [centers.contiguous(), torch.empty_like(centers)]
        labels = [torch.full((R, n), -1, dtype=torch.int32, device=dev), torch.empty(R, n, dtype=torch.int32, device=dev)]
        # [info R*(k+1) | changed R (int32 bits)]: one copy back per iteration together with the new centres
        pack = torch.empty(R * (k + 1) + R, dtype=torch.float32, device=dev)
        info = pack[:R * (k + 1)]
        changed = pack[R * (k + 1):].view(torch.int32)
        sums = torch.empty(R, k, d, dtype=torch.float32, device=dev)
        wts = torch.empty(R, k, dtype=torch.float32, device=dev)
        ws_bytes = int(lib.hlmc_km_sums_workspace(n, k)) * R
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        old_c = cbuf[0].cpu().numpy()
        pinned = dev.type == "cuda"
        pack_p = torch.empty(pack.shape, dtype=torch.float32).pin_memory() if pinned else None
        cen_p = torch.empty(centers.shape, dtype=torch.float32).pin_memory() if pinned else None
        final_c = old_c.copy()
        final_lab = torch.empty(R, n, dtype=torch.int32, device=dev)
        n_iter = np.zeros(R, dtype=np.int64)
        strict = np.zeros(R, dtype=bool)
        active = (1 << R) - 1
        Xh = None
        for it in range(self.max_iter):
            if not active:
                break
            cur, nxt = cbuf[it % 2], cbuf[(it + 1) % 2]
            lab_old, lab_new = labels[it % 2], labels[(it + 1) % 2]
            changed.zero_()
            L.check(lib.hlmc_km_assign_batch(L.stream(), Xc.data_ptr(), n, d, cur.data_ptr(), k, R, active,
                                             lab_new.data_ptr(), lab_old.data_ptr(), changed.data_ptr()))
            L.check(lib.hlmc_km_sums_batch(L.stream(), Xc.data_ptr(), n, d, lab_new.data_ptr(), k, R, active,
                                           sums.data_ptr(), wts.data_ptr(), ws.data_ptr(), ws_bytes))
            L.check(lib.hlmc_km_update_batch(L.stream(), k, d, R, active, sums.data_ptr(), wts.data_ptr(),
                                             cur.data_ptr(), nxt.data_ptr(), info.data_ptr()))
            if pinned:   # one synchronisation per iteration: counts, shifts and the new centres
                pack_p.copy_(pack, non_blocking=True)
                cen_p.copy_(nxt, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                pack_h, nxt_h = pack_p.numpy(), cen_p.numpy()
            else:
                pack_h, nxt_h = pack.cpu().numpy(), nxt.cpu().numpy()
            info_h = pack_h[:R * (k + 1)].reshape(R, k + 1)
            chg = pack_h[R * (k + 1):].view(np.int32)
            for r in range(R):
                if not (active >> r) & 1:
                    continue
                if info_h[r, k] != 0:   # an empty cluster: this restart's update on the host, as sklearn does it
                    if Xh is None:
                        Xh = Xc.cpu().numpy()
                    new = sums[r].cpu().numpy()
                    wic = wts[r].cpu().numpy()
                    lab_h = lab_new[r].cpu().numpy()
                    dist = ((Xh - old_c[r][lab_h]) ** 2).sum(axis=1)
                    empty = np.where(wic == 0)[0]
                    if dist.max() > 0:
                        far = np.argpartition(dist, -empty.size)[:-empty.size - 1:-1]
                        for e, f in zip(empty, far):
                            o = lab_h[f]
                            new[o] -= Xh[f]
                            new[e] = Xh[f]
                            wic[e] = 1.0
                            wic[o] -= 1.0
                    amax = int(np.argmax(wic))
                    for j in range(k):
                        if wic[j] > 0:
                            new[j] *= np.float32(1.0 / float(wic[j]))
                        else:
                            new[j] = new[amax]
                    shift = np.sqrt(_euclid_f32(new, old_c[r])).astype(np.float32)
                    nxt[r].copy_(torch.from_numpy(new))
                else:
                    new = nxt_h[r].copy()
                    shift = np.sqrt(info_h[r, :k]).astype(np.float32)
                old_c[r] = new
                done = False
                if chg[r] == 0 and it > 0:
                    strict[r] = done = True
                elif (shift ** 2).sum() <= tol:
                    done = True
                elif it + 1 == self.max_iter:
                    done = True
                if done:
                    n_iter[r] = it + 1
                    final_c[r] = new
                    final_lab[r].copy_(lab_new[r])
                    active &= ~(1 << r)
        fc = torch.from_numpy(final_c).to(dev)
        redo = sum(1 << r for r in range(R) if not strict[r])
        if redo:   # not strictly converged: labels from the final centres (sklearn's last lloyd_iter, no update)
            L.check(lib.hlmc_km_assign_batch(L.stream(), Xc.data_ptr(), n, d, fc.data_ptr(), k, R, redo,
                                             final_lab.data_ptr(), None, None))
        inertia = torch.empty(R, dtype=torch.float32, device=dev)
        tmp = torch.empty(R, n, dtype=torch.float32, device=dev)
        L.check(lib.hlmc_km_inertia_batch(L.stream(), Xc.data_ptr(), n, d, fc.data_ptr(), k, final_lab.data_ptr(), R,
                                          inertia.data_ptr(), tmp.data_ptr()))
        return final_lab.cpu().numpy(), inertia.cpu().numpy().astype(np.float64), final_c, n_iter

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
        world, rank = 1, 0
        if self.process_group is not None:
            world = dist.get_world_size(self.process_group)
            rank = dist.get_rank(self.process_group)
        mine = [i for i in range(n_init) if i % world == rank]
        seeds, trials = self._draw_seeds(rs, n, n_init, set(mine))
        runs = []
        # restarts in lockstep: <= 16 per batch, R x trials <= 64 (hlmc_km_pp_*), their candidate rows in LDS
        g = max(1, min(16, 64 // trials, (150 * 1024) // (8 * trials * (d + 1))))
        for g0 in range(0, len(mine), g):
            grp = mine[g0:g0 + g]
            c0, _ = self._kmeans_plusplus_batch(Xc, [seeds[i] for i in grp], trials)
            labels, inertia, centers, n_iter = self._lloyd_batch(Xc, c0, tol)
            for j, i in enumerate(grp):
                runs.append((i, labels[j], float(inertia[j]), centers[j], int(n_iter[j])))
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
