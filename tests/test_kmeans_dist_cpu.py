"""Restart-sharded KMeans(process_group=...) host logic on CPU with world_size-2 gloo.

The device helpers (_center, _sqdist, _lloyd) are swapped for the numpy oracle's pieces so the test runs
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

        def _lloyd(self, Xc, centers, tol):
            X = Xc.numpy()
            w = np.ones(X.shape[0], np.float32)
            lab, inertia, cen, nit = KO.kmeans_single_lloyd(X, w, centers.numpy(), self.max_iter, tol)
            return torch.from_numpy(lab), inertia, torch.from_numpy(cen), nit

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
    """A rank skips another rank's k-means++ seeding by drawing KMeans.seeding_draws(k) doubles: the RandomState
    must then stand exactly where the seeding itself would have left it (any k, any data)."""
    cls = _cpu_kmeans_cls()
    X = _data()
    Xc = torch.from_numpy(X - X.mean(axis=0))
    w = np.ones(N, np.float32)
    for k in (2, 3, 7, 10, 14):
        a, b = np.random.RandomState(42), np.random.RandomState(42)
        for _ in range(3):
            cls(n_clusters=k)._kmeans_plusplus(Xc, a, w)
        b.random_sample(3 * cls.seeding_draws(k))
        sa, sb = a.get_state(), b.get_state()
        assert np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:], k
        assert a.random_sample() == b.random_sample()
