"""Cluster-metric timings: GPU silhouette / Davies-Bouldin / Calinski-Harabasz on
latent-like blobs (N up to 100 000 x 128, k = 10 — BASELINE config 5's clustering scale) against sklearn on
the host for the sizes it finishes in seconds.  Prints one JSON line per case.

Roofline of the silhouette kernel: N^2 pairs x D x 3 flops (sub, fma) on fp32 VALU (MI355X ~157 TFLOP/s
fp32 vector); bytes are negligible (X is re-read from L2 per row tile)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402
from tests.golden import fixtures as FX  # noqa: E402

M = hlmc_amd.metrics
PEAK_VALU = 157.3e12


def gpu_time(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


for n, d, k in [(1336, 128, 10), (10000, 128, 10), (100000, 128, 10), (100000, 64, 14)]:
    X = FX.blobs(n, d, k, seed=n + d)
    y = FX.blob_labels(n, d, k, seed=n + d)
    Xd = torch.from_numpy(X).cuda()
    t_sil = gpu_time(lambda: M.silhouette_score(Xd, y))
    t_dbch = gpu_time(lambda: (M.davies_bouldin_score(Xd, y), M.calinski_harabasz_score(Xd, y)))
    flops = 3.0 * n * n * d
    rec = {"case": f"N={n} D={d} k={k}", "silhouette_ms": round(t_sil * 1e3, 3),
           "silhouette_valu_frac": round(flops / t_sil / PEAK_VALU, 4), "db_ch_ms": round(t_dbch * 1e3, 3)}
    if n <= 10000:
        from sklearn import metrics as skm
        t0 = time.perf_counter()
        skm.silhouette_score(X, y)
        rec["sklearn_silhouette_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        rec["cpu_cores"] = len(os.sched_getaffinity(0))
    print(json.dumps(rec), flush=True)
