"""Restart-sharded KMeans(process_group=...) host logic on CPU with world_size-2 gloo.

The device helpers (_center, _sqdist, _kmeans_plusplus_batch, _lloyd_batch) are swapped for the numpy oracle's pieces so the test runs
without a GPU; what is under test is the sharding of the n_init restarts over ranks, the replicated
k-means++ RandomState stream and the gathered best-of rule.  Both ranks must return the single-process
result, and that must equal the oracle KMeans (itself pinned to sklearn 1.7.2 by tests/golden)."""
import os
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import kmeans_oracle as KO
from tests.golden import fixtures as FX

WORLD = 2
N, D, K, N_INIT = 600, 16, 6, 5


def _cpu_kmeans_cls():
    from hlmc_amd.cluster import KMeans

    class CpuKMeans(KMeans):
        def _dev(self):
            return torch.device("cpu")

        def _center(self, Xd):
            X = Xd.numpy()
            mean = X.mean(axis=0)
            var = np.var(X, axis=0)
            return torch.from_numpy(mean), torch.from_numpy(var), torch.from_numpy(X - mean)

        def _sqdist(self, Xc, cand):
            X = Xc.numpy()
            return torch.from_numpy(KO._sqdist_upcast(X[np.asarray(cand)], X))

        def _kmeans_plusplus_batch(self, Xc, seeds, trials):
            # the oracle's k-means++ (sklearn _kmeans_plusplus) fed with the pre-drawn random numbers
            X = Xc.numpy()
            n, k = X.shape[0], self.n_clusters
            w = np.ones(n, np.float32)
            cents = []
            for cid, us in seeds:
                idx = [cid]
                closest = KO._sqdist_upcast(X[cid][None, :], X)
                pot = closest @ w
                for c in range(1, k):
                    cand = np.searchsorted(np.cumsum((w * closest).astype(np.float64), dtype=np.float64), us[c - 1] * pot)
                    np.clip(cand, None, n - 1, out=cand)
                    dc = KO._sqdist_upcast(X[cand], X)
                    np.minimum(closest, dc, out=dc)
                    cpot = dc @ w.reshape(-1, 1)
                    b = int(np.argmin(cpot))
                    pot, closest = cpot[b], dc[b]
                    idx.append(int(cand[b]))
                cents.append(X[idx])
            return torch.from_numpy(np.stack(cents)), None

        def _lloyd_batch(self, Xc, centers, tol):
            X = Xc.numpy()
            w = np.ones(X.shape[0], np.float32)
            res = [KO.kmeans_single_lloyd(X, w, c, self.max_iter, tol) for c in centers.numpy()]
            return (np.stack([r[0] for r in res]), np.array([r[1] for r in res]), np.stack([r[2] for r in res]),
                    np.array([r[3] for r in res]))

    return CpuKMeans


def _data():
    return FX.blobs(N, D, K, seed=11)


def _worker(rank, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    km = _cpu_kmeans_cls()(n_clusters=K, random_state=42, n_init=N_INIT, process_group=dist.group.WORLD)
    km.fit(_data())
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), labels=km.labels_, centers=km.cluster_centers_,
             inertia=km.inertia_, n_iter=km.n_iter_)
    dist.barrier()
    dist.destroy_process_group()


def test_kmeans_restarts_sharded_over_ranks():
    with tempfile.TemporaryDirectory() as outdir:
        port = 29300 + (os.getpid() % 1000)
        mp.spawn(_worker, args=(port, outdir), nprocs=WORLD, join=True)
        res = [dict(np.load(os.path.join(outdir, f"rank{r}.npz"))) for r in range(WORLD)]
    single = _cpu_kmeans_cls()(n_clusters=K, random_state=42, n_init=N_INIT).fit(_data())
    ora = KO.KMeans(K, random_state=42, n_init=N_INIT).fit(_data())
    np.testing.assert_array_equal(single.labels_, ora.labels_)
    for r in res:
        np.testing.assert_array_equal(r["labels"], single.labels_)
        np.testing.assert_array_equal(r["centers"], single.cluster_centers_)
        assert float(r["inertia"]) == single.inertia_
        assert int(r["n_iter"]) == single.n_iter_


def test_select_best_keeps_first_of_equal_partitions():
    from hlmc_amd.cluster import KMeans
    a = np.array([0, 0, 1, 1])
    b = np.array([1, 1, 0, 0])            # same partition, relabelled, lower inertia: sklearn keeps a
    c = np.array([0, 1, 1, 1])
    runs = [(0, a, 5.0, None, 3), (1, b, 4.0, None, 2), (2, c, 6.0, None, 4)]
    assert KMeans._select_best(runs, 2)[0] == 0
    runs = [(0, a, 5.0, None, 3), (1, c, 4.5, None, 2)]
    assert KMeans._select_best(runs, 2)[0] == 1


def test_seeding_draws_match_the_stream():
    """The restarts' random numbers are drawn up front (KMeans._draw_seeds) and a rank skips another rank's seeding
    by drawing KMeans.seeding_draws(k) doubles: either way the RandomState must stand exactly where sklearn's
    sequential k-means++ seedings (the oracle's kmeans_plusplus) leave it, and the kept draws must be the ones that
    seeding consumes (any k, any data)."""
    cls = _cpu_kmeans_cls()
    X = _data()
    Xc = X - X.mean(axis=0)
    for k in (2, 3, 7, 10, 14):
        a, b, c = np.random.RandomState(42), np.random.RandomState(42), np.random.RandomState(42)
        want = [KO.kmeans_plusplus(Xc, k, a)[1] for _ in range(3)]
        seeds, trials = cls(n_clusters=k)._draw_seeds(b, N, 3, {0, 1, 2})
        cls(n_clusters=k)._draw_seeds(c, N, 3, set())
        for rs in (b, c):
            sa, sb = a.get_state(), rs.get_state()
            assert np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:], k
        got, _ = cls(n_clusters=k)._kmeans_plusplus_batch(torch.from_numpy(Xc), [seeds[i] for i in range(3)], trials)
        np.testing.assert_array_equal(got.numpy(), np.stack([Xc[w] for w in want]))
        assert a.random_sample() == b.random_sample() == c.random_sample()
