import sys, time, numpy as np, torch
sys.path.insert(0, '/root/repo')
import hlmc_amd
from tests.golden import fixtures as FX
from oracle import kmeans_oracle as KO
X = FX.overlap_blobs(100000, 128, 10, 0.3, 5)
km = hlmc_amd.KMeans(n_clusters=10, random_state=42, n_init=10)
km.fit(X); torch.cuda.synchronize()
import cProfile, pstats
t0=time.perf_counter(); km.fit(X); torch.cuda.synchronize(); print('fit ms', (time.perf_counter()-t0)*1e3, 'n_iter', km.n_iter_)
orig_pp, orig_ll = km._kmeans_plusplus_batch, km._lloyd_batch
def tpp(*a, **k):
    torch.cuda.synchronize(); t=time.perf_counter(); r=orig_pp(*a, **k); torch.cuda.synchronize(); print('seeding ms', (time.perf_counter()-t)*1e3); return r
def tll(*a, **k):
    torch.cuda.synchronize(); t=time.perf_counter(); r=orig_ll(*a, **k); torch.cuda.synchronize(); print('lloyd ms', (time.perf_counter()-t)*1e3, 'iters', r[3]); return r
km._kmeans_plusplus_batch, km._lloyd_batch = tpp, tll
km.fit(X)
pr = cProfile.Profile(); pr.enable(); km.fit(X); torch.cuda.synchronize(); pr.disable()
pstats.Stats(pr).sort_stats('cumulative').print_stats(18)
