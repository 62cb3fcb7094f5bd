"""K-Means benchmark (SURVEY §8(d) "K-Means Lloyd iter" row): KMeans(k, random_state=42, n_init=10).fit on
latent-like blobs [N, D] f32, the reference's call (src/Convolutional_VAE.py:317-319, cfg 5 at N=100k).

Prints one JSON line per case: whole-fit wall time, Lloyd iterations run (all restarts), and the E-step
(hlmc_km_assign) and M-step (hlmc_km_sums direct, hlmc_km_sums_part partitioned -- the fit's) kernels timed alone with HIP events on the launch stream,
each against the HBM roofline (algorithmic bytes per launch = N*D*4 read + N*4 labels written / read).
sklearn (threadpool default) is timed beside it where it finishes in seconds."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hlmc_amd  # noqa: E402
from hlmc_amd import _lib as L  # noqa: E402
from tests.golden import fixtures as FX  # noqa: E402

HBM_PEAK_GBS = 8000.0


def _time_kernel(fn, reps=50):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3   # us


def case(n, d, k, n_init, sklearn_too):
    X = FX.blobs(n, d, k, seed=n + d + k)
    km = hlmc_amd.KMeans(n_clusters=k, random_state=42, n_init=n_init)
    km.fit(X)                                   # warm-up (library load, allocations)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    km.fit(X)
    torch.cuda.synchronize()
    fit_ms = (time.perf_counter() - t0) * 1e3
    iters = 0
    orig = km._lloyd_batch

    def counting(*a, **kw):
        nonlocal iters
        r = orig(*a, **kw)
        iters += int(np.sum(r[3]))
        return r
    km._lloyd_batch = counting
    km.fit(X)
    Xd = torch.as_tensor(X, device="cuda")
    C = Xd[:k].contiguous()
    lab = torch.as_tensor(km.labels_.astype(np.int32), device="cuda")     # the fit's own partition
    heavy = torch.zeros_like(lab)                                         # worst case: one cluster
    old = torch.zeros_like(lab)
    changed = torch.zeros(1, dtype=torch.int32, device="cuda")
    sums = torch.empty(k, d, device="cuda")
    wts = torch.empty(k, device="cuda")
    lib = L.lib()
    assign_us = _time_kernel(lambda: L.check(lib.hlmc_km_assign(L.stream(), Xd.data_ptr(), n, d, C.data_ptr(), k,
                                                                lab.data_ptr(), old.data_ptr(), changed.data_ptr())))
    sums_us = _time_kernel(lambda: L.check(lib.hlmc_km_sums(L.stream(), Xd.data_ptr(), n, d, lab.data_ptr(), k,
                                                            sums.data_ptr(), wts.data_ptr())))
    heavy_us = _time_kernel(lambda: L.check(lib.hlmc_km_sums(L.stream(), Xd.data_ptr(), n, d, heavy.data_ptr(), k,
                                                             sums.data_ptr(), wts.data_ptr())))
    nb = int(lib.hlmc_km_sums_workspace(n, k))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    part_us = _time_kernel(lambda: L.check(lib.hlmc_km_sums_part(L.stream(), Xd.data_ptr(), n, d, lab.data_ptr(), k,
                                                                 sums.data_ptr(), wts.data_ptr(), ws.data_ptr(), nb)))
    part_heavy_us = _time_kernel(lambda: L.check(lib.hlmc_km_sums_part(L.stream(), Xd.data_ptr(), n, d,
                                                                       heavy.data_ptr(), k, sums.data_ptr(),
                                                                       wts.data_ptr(), ws.data_ptr(), nb)))
    a_bytes = n * d * 4 + 2 * n * 4
    s_bytes = n * d * 4 + n * 4
    out = {"case": f"N={n} D={d} k={k} n_init={n_init}", "fit_ms": round(fit_ms, 2), "lloyd_iters": iters,
           "ms_per_lloyd_iter": round(fit_ms / max(iters, 1), 4),
           "assign_us": round(assign_us, 2), "assign_GBs": round(a_bytes / assign_us / 1e3, 1),
           "assign_frac": round(a_bytes / assign_us / 1e3 / HBM_PEAK_GBS, 4),
           "sums_us": round(sums_us, 2), "sums_GBs": round(s_bytes / sums_us / 1e3, 1),
           "sums_frac": round(s_bytes / sums_us / 1e3 / HBM_PEAK_GBS, 4),
           "sums_one_cluster_us": round(heavy_us, 2),
           "sums_part_us": round(part_us, 2), "sums_part_frac": round(s_bytes / part_us / 1e3 / HBM_PEAK_GBS, 4),
           "sums_part_one_cluster_us": round(part_heavy_us, 2)}
    if sklearn_too:
        from sklearn.cluster import KMeans as SK
        t0 = time.perf_counter()
        ref = SK(n_clusters=k, random_state=42, n_init=n_init).fit(X)
        out["sklearn_fit_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        out["labels_equal_sklearn"] = bool(np.array_equal(ref.labels_, km.labels_))
        out["cpu_cores"] = len(os.sched_getaffinity(0))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    assert torch.cuda.is_available()
    case(1336, 128, 10, 10, True)
    case(10000, 128, 10, 10, True)
    case(100000, 128, 10, 10, "--sklearn-100k" in sys.argv)
    case(100000, 64, 14, 10, False)
