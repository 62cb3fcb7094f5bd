"""K-Means on the GPU vs sklearn 1.7.2 KMeans(random_state=42) labels recorded in tests/golden
(bit-identical labels required; centres within float32 rounding; ARI vs sklearn == 1).

Besides the well-separated blob cases, the fixtures hold overlapping clusters (near-tie E-steps, where the
label is decided by float32 rounding), eval-mode VAE latents (k = 2..14, the reference's silhouette sweep)
and the config[4] clustering scale (N = 100 000).  Each test reports the near-tie count of the final E-step
(rows whose two smallest distances lie within 8 float32 ulps) and the ARI against sklearn's labels."""
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


def _sharded_worker(rank, port, outdir, case):
    import os
    import sys
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import hlmc_amd
    torch.cuda.set_device(0)
    n, d, centers, k, n_init = case
    X = FX.blobs(n, d, centers, seed=n + d + k)
    km = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=n_init, process_group=dist.group.WORLD).fit(X)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), labels=km.labels_, centers=km.cluster_centers_,
             inertia=km.inertia_, n_iter=km.n_iter_)
    dist.barrier()
    dist.destroy_process_group()


def test_kmeans_restarts_sharded_two_ranks(cuda):
    """n_init restarts sharded over 2 ranks (gloo, both on cuda:0): each rank's result equals the
    single-process fit and the sklearn golden labels bit-for-bit."""
    import os
    import tempfile
    import torch.multiprocessing as mp
    case = [c for c in FX.KMEANS_CASES if c[0] == 1336 and c[1] == 128 and c[3] == 10 and c[4] == 10][0]
    n, d, centers, k, n_init = case
    fx = np.load(f"tests/golden/kmeans_n{n}_d{d}_k{k}_i{n_init}.npz")
    with tempfile.TemporaryDirectory() as outdir:
        mp.spawn(_sharded_worker, args=(29800 + os.getpid() % 100, outdir, case), nprocs=2, join=True)
        res = [dict(np.load(os.path.join(outdir, f"rank{r}.npz"))) for r in range(2)]
    single = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(FX.blobs(n, d, centers, seed=n + d + k))
    for r in res:
        np.testing.assert_array_equal(r["labels"], fx["labels"])
        np.testing.assert_array_equal(r["labels"], single.labels_)
        np.testing.assert_array_equal(r["centers"], single.cluster_centers_)
        assert float(r["inertia"]) == single.inertia_ and int(r["n_iter"]) == single.n_iter_


@pytest.mark.parametrize("path", ["direct", "part"])
@pytest.mark.parametrize("n,d,k", [(20000, 80, 7), (3000, 130, 3), (1025, 64, 1), (5000, 16, 100), (70001, 3, 11),
                                   (300, 200, 40)])
def test_km_sums_row_order_bitexact(cuda, n, d, k, path):
    """hlmc_km_sums / hlmc_km_sums_part = sklearn's single-thread float32 centre sums: per cluster and column a
    strictly sequential row-order add (np.add.accumulate), counts exact; ragged column slabs and tiles, a heavy
    cluster, empty clusters (k > distinct labels at n=300, k=40)."""
    import torch
    from hlmc_amd import _lib as L
    rng = np.random.default_rng(n + d + k)
    X = rng.normal(0, 2.0, (n, d)).astype(np.float32)
    lab = rng.integers(0, k, n).astype(np.int32)
    lab[: n // 3] = 0                                     # one heavy cluster
    if k == 40:
        lab[lab % 3 == 1] = 2                             # some clusters left empty
    Xd, ld = torch.as_tensor(X, device="cuda"), torch.as_tensor(lab, device="cuda")
    sums = torch.empty(k, d, device="cuda")
    w = torch.empty(k, device="cuda")
    sums.fill_(float("nan"))
    w.fill_(float("nan"))
    if path == "direct":
        L.check(L.lib().hlmc_km_sums(L.stream(), Xd.data_ptr(), n, d, ld.data_ptr(), k, sums.data_ptr(), w.data_ptr()))
    else:
        nb = int(L.lib().hlmc_km_sums_workspace(n, k))
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        L.check(L.lib().hlmc_km_sums_part(L.stream(), Xd.data_ptr(), n, d, ld.data_ptr(), k, sums.data_ptr(),
                                          w.data_ptr(), ws.data_ptr(), nb))
    got = sums.cpu().numpy()
    for j in range(k):
        rows = X[lab == j]
        ref = np.add.accumulate(rows, axis=0)[-1] if len(rows) else np.zeros(d, np.float32)
        np.testing.assert_array_equal(got[j], ref)
        assert float(w[j]) == float((lab == j).sum())


@pytest.mark.parametrize("n,d", [(20000, 80), (1337, 128), (70, 3)])
def test_km_center_numpy_order_bitexact(cuda, n, d):
    """hlmc_km_center = numpy's X.mean(axis=0) / np.var(X, axis=0) (row-sequential float32) bit for bit."""
    import torch
    from hlmc_amd import _lib as L
    X = np.random.default_rng(n * d).normal(0.5, 2.0, (n, d)).astype(np.float32)
    Xd = torch.as_tensor(X, device="cuda")
    mean, var, Xc = torch.empty(d, device="cuda"), torch.empty(d, device="cuda"), torch.empty_like(Xd)
    L.check(L.lib().hlmc_km_center(L.stream(), Xd.data_ptr(), n, d, mean.data_ptr(), var.data_ptr(), Xc.data_ptr()))
    np.testing.assert_array_equal(mean.cpu().numpy(), X.mean(axis=0))
    np.testing.assert_array_equal(var.cpu().numpy(), np.var(X, axis=0))
    np.testing.assert_array_equal(Xc.cpu().numpy(), X - X.mean(axis=0))


def _near_ties(X, centers, ulps=8):
    """Rows whose two smallest E-step distances lie within `ulps` float32 ulps (oracle arithmetic)."""
    from oracle import kmeans_oracle as KO
    Xc = (X - X.mean(axis=0)).astype(np.float32)
    C = (centers - X.mean(axis=0)).astype(np.float32)
    cn = KO.row_norms_sq_f32(C)
    cnt = 0
    for s in range(0, Xc.shape[0], KO.CHUNK):
        dd = np.sort(KO.estep_dist(Xc[s:s + KO.CHUNK], C, cn), axis=1)
        if dd.shape[1] > 1:
            cnt += int((dd[:, 1] - dd[:, 0] <= ulps * np.spacing(np.abs(dd[:, 1]))).sum())
    return cnt


def _check_against_fixture(km, labels, centers, inertia, n_iter, X, what):
    from sklearn.metrics import adjusted_rand_score
    ari = adjusted_rand_score(labels, km.labels_)
    ties = _near_ties(X, centers) if X.shape[0] <= 5000 else -1
    print(f"{what}: near-tie rows {ties}, ARI vs sklearn {ari:.6f}, n_iter {km.n_iter_}/{n_iter}")
    np.testing.assert_array_equal(km.labels_, labels)
    np.testing.assert_allclose(km.cluster_centers_, centers, rtol=1e-5, atol=1e-5)
    assert km.n_iter_ == n_iter
    assert km.inertia_ == inertia


@pytest.mark.parametrize("case", FX.KMEANS_OVERLAP_CASES, ids=lambda c: f"n{c[0]}_d{c[1]}_s{c[3]}_k{c[4]}_i{c[5]}")
def test_kmeans_overlapping_clusters_bitexact(cuda, case):
    n, d, true_k, spread, k, n_init = case
    X = FX.overlap_blobs(n, d, true_k, spread, FX.overlap_seed(case))
    fx = np.load("tests/golden/" + FX.overlap_fixture_name(case))
    km = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
    _check_against_fixture(km, fx["labels"], fx["centers"], float(fx["inertia"]), int(fx["n_iter"]), X,
                           FX.overlap_fixture_name(case))


def test_kmeans_vae_latents_k_sweep(cuda):
    """src/Convolutional_VAE.py:311-327: KMeans(k, random_state=42, n_init=10) for k = 2..14 on eval-mode
    latents of the (oracle) HybridVAE, labels bit-identical to sklearn for every k."""
    fx = np.load("tests/golden/kmeans_latents_n1336_d128.npz")
    X = fx["X"]
    for k in FX.LATENT_KS:
        km = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=10).fit(X)
        _check_against_fixture(km, fx[f"labels_k{k}"], fx[f"centers_k{k}"], float(fx[f"inertia_k{k}"]),
                               int(fx[f"n_iter_k{k}"]), X, f"latents k={k}")


def test_kmeans_100k_config4_scale(cuda):
    """BASELINE config[4]'s clustering scale: N = 100 000 latents-like rows, D = 128, k = 10, n_init = 10."""
    case = FX.KMEANS_BIG_CASE
    n, d, true_k, spread, k, n_init = case
    X = FX.overlap_blobs(n, d, true_k, spread, FX.overlap_seed(case))
    fx = np.load("tests/golden/" + FX.overlap_fixture_name(case))
    km = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
    _check_against_fixture(km, fx["labels"], fx["centers"], float(fx["inertia"]), int(fx["n_iter"]), X, "N=100k")


@pytest.mark.parametrize("n,d,k", [(1336, 128, 2), (1336, 128, 10), (1000, 64, 5), (513, 100, 13), (257, 32, 16),
                                   (300, 130, 3), (4096, 128, 14), (77, 40, 1)])
def test_km_assign_matches_sklearn_estep(cuda, n, d, k):
    """hlmc_km_assign on near-tie data (points on the bisector of two centres) equals the oracle's
    restatement of sklearn's E-step (einsum norms + the OpenBLAS sgemm kernel sklearn's call takes) label
    for label, including the short last chunk and the small-matrix kernel's remainder elements."""
    import torch
    from hlmc_amd import _lib as L
    from oracle import kmeans_oracle as KO
    rng = np.random.default_rng(n * 31 + d * 7 + k)
    C = rng.standard_normal((k, d)).astype(np.float32)
    t = rng.standard_normal((n, d)).astype(np.float32)
    if k >= 2:
        m, u = (C[0] + C[1]) / 2, C[1] - C[0]
        u = u / np.linalg.norm(u)
        t = t - np.outer(t @ u, u)
        X = (m + 0.3 * t + np.outer(rng.standard_normal(n) * 1e-6, u)).astype(np.float32)
    else:
        X = t
    ref = KO.assign_labels(X, C)
    Xd, Cd = torch.as_tensor(X, device="cuda"), torch.as_tensor(C, device="cuda")
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    L.check(L.lib().hlmc_km_assign(L.stream(), Xd.data_ptr(), n, d, Cd.data_ptr(), k, lab.data_ptr(), None, None))
    np.testing.assert_array_equal(lab.cpu().numpy(), ref)


def test_kmeans_pp_search_bracket_flags_exact_prefixes(cuda):
    """hlmc_km_pp_search (include/hlmc.h): a draw lying exactly on a float64 cumsum prefix -- here also inside a run of
    zero distances from duplicate rows, where several prefixes are equal -- cannot be decided by the device's error
    bracket and must be flagged (amb = 1) for the numpy redo; every draw it does decide equals np.searchsorted of
    numpy's own float64 cumsum (sklearn _kmeans_plusplus)."""
    import ctypes as C
    import torch
    from hlmc_amd import _lib as L
    n = 5000
    g = np.random.default_rng(3)
    d = g.random(n).astype(np.float32)
    d[1000:1040] = 0.0                          # duplicate rows of an already-chosen centre: zero distance
    cs = np.cumsum(d, dtype=np.float64)
    exact = [cs[10], cs[1000], cs[1020], cs[2500], cs[n - 1]]
    between = [0.5 * (cs[99] + cs[100]), 0.5 * (cs[3999] + cs[4000]), 0.25 * cs[0]]
    rv = np.array(exact + between, dtype=np.float64)
    T = len(rv)
    prev = torch.from_numpy(d).reshape(1, 1, n).cuda()
    best = np.zeros(1, dtype=np.int32)
    cand = torch.empty(T, dtype=torch.int64, device="cuda")
    amb = torch.empty(T, dtype=torch.int32, device="cuda")
    L.check(L.lib().hlmc_km_pp_search(L.stream(), n, 1, T, prev.data_ptr(), 1, best.ctypes.data_as(C.POINTER(C.c_int32)),
                                      rv.ctypes.data_as(C.POINTER(C.c_double)), cand.data_ptr(), amb.data_ptr()))
    torch.cuda.synchronize()
    cand, amb = cand.cpu().numpy(), amb.cpu().numpy()
    ref = np.minimum(np.searchsorted(cs, rv), n - 1)
    print(f"amb flags {amb.tolist()}, candidates {cand.tolist()} vs numpy {ref.tolist()}")
    assert amb[:len(exact)].all(), amb
    assert not amb[len(exact):].any(), amb
    decided = amb == 0
    np.testing.assert_array_equal(cand[decided], ref[decided])


def test_kmeans_pp_numpy_redo_matches_oracle(cuda, monkeypatch):
    """The k-means++ fallback where the device bracket cannot decide (KMeans._kmeans_plusplus_batch): with every draw
    forced ambiguous, each restart's candidates come from numpy's cumsum / searchsorted, the distances are recomputed
    and written back into the device buffer and the pinned host image -- the chosen centres must still equal the
    oracle's sklearn _kmeans_plusplus (oracle/kmeans_oracle.kmeans_plusplus) restart by restart, on data with duplicate
    rows (zero distances)."""
    import ctypes as C
    import torch
    from hlmc_amd import _lib as L
    from oracle import kmeans_oracle as KO
    X = FX.blobs(3000, 16, 6, seed=12)
    X = np.concatenate([X, np.repeat(X[:50], 4, axis=0)]).astype(np.float32)
    k, n_init = 8, 4
    km = hlmc_amd.KMeans(n_clusters=k, random_state=7, n_init=n_init)
    Xd = torch.as_tensor(X, device="cuda")
    _, _, Xc = km._center(Xd)
    lib = L.lib()
    orig = lib.hlmc_km_pp_search
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    forced = []

    def always_ambiguous(stream, n, R, T, prev, prevT, best, rvals, cand, amb):
        st = orig(stream, n, R, T, prev, prevT, best, rvals, cand, amb)
        assert hip.hipMemsetAsync(amb, 1, 4 * R * T, stream) == 0
        forced.append(R * T)
        return st

    rs = np.random.RandomState(7)
    seeds, trials = km._draw_seeds(rs, X.shape[0], n_init, set(range(n_init)))
    monkeypatch.setattr(lib, "hlmc_km_pp_search", always_ambiguous)
    _, idx = km._kmeans_plusplus_batch(Xc, [seeds[i] for i in range(n_init)], trials)
    monkeypatch.setattr(lib, "hlmc_km_pp_search", orig)
    assert len(forced) == k - 1
    _, idx_dev = km._kmeans_plusplus_batch(Xc, [seeds[i] for i in range(n_init)], trials)
    Xh = Xc.cpu().numpy()
    rs = np.random.RandomState(7)
    for i in range(n_init):
        _, ref = KO.kmeans_plusplus(Xh, k, rs)
        np.testing.assert_array_equal(idx[i], ref, err_msg=f"restart {i} (numpy redo)")
        np.testing.assert_array_equal(idx_dev[i], ref, err_msg=f"restart {i} (device draws)")
