"""Data-parallel host logic on CPU with world_size-2 gloo (the GPU path uses the same code over RCCL).

* Trainer.allreduce_grads: SUM of the flat gradient buffer across ranks.  With the reference's sum-reduced
  loss, the DP gradient of the global batch is the sum of the per-shard gradients (BatchNorm statistics per
  rank = DDP semantics, so each shard's gradient is that of the reference model run on the shard).  Checked
  bit-exact against the single-process sum of the oracle model's per-shard gradients.
* Trainer's DDP broadcast_buffers: the model's BatchNorm running statistics are re-pointed at one flat tensor
  (state_dict unchanged) and rank 0's values reach every rank through one broadcast.
* StandardScaler(process_group): the two f64 passes are all-reduced and finalised with scaler_finalize; the
  result equals sklearn's StandardScaler on the concatenated shards.
"""
import os
import tempfile
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import models_oracle as OM

WORLD = 2


def _shard_grads(rank):
    """Flat fp32 gradient of the oracle audio-only HybridVAE (seed-42 init) on shard `rank` (2 clips)."""
    torch.manual_seed(42)
    model = OM.HybridVAE(128, 768, (128, 128), audio_only=True)
    g = torch.Generator().manual_seed(100 + rank)
    audio = torch.randn(2, 1, 128, 128, generator=g)
    eps = torch.randn(2, 128, generator=g)
    out = model(audio, None, eps=eps)
    loss = OM.loss_function(out[0], audio, None, None, out[2], out[3])[0]
    loss.backward()
    return torch.cat([p.grad.reshape(-1) for p in model.parameters()])


def _engine_buckets(total):
    """Flat ranges of libhlmc's gradient buckets for the audio-only HybridVAE (host-only C-ABI calls)."""
    import ctypes
    from hlmc_amd import _lib as L
    from hlmc_amd.train import bucket_ranges
    lib = L.lib()
    h = ctypes.c_void_p()
    L.check(lib.hlmc_net_create(L.NET_HYBRID, L.i64_array([128, 0, 128, 128]), 4, L.HLMC_F32, ctypes.byref(h)))
    try:
        offs = [0]
        shape = (L.c_i64 * 8)()
        nd = ctypes.c_int()
        name = ctypes.create_string_buffer(256)
        for i in range(lib.hlmc_net_num_params(h)):
            L.check(lib.hlmc_net_param_info(h, i, name, 256, ctypes.byref(nd), shape))
            n = 1
            for d in shape[:nd.value]:
                n *= d
            offs.append(offs[-1] + n)
        starts = (ctypes.c_int * 16)()
        nb = lib.hlmc_net_grad_buckets(h, starts, 16)
        assert nb >= 2, nb
        ranges = bucket_ranges(list(starts)[:nb], offs)
    finally:
        lib.hlmc_net_destroy(h)
    assert offs[-1] == total
    assert sorted(ranges) == [(a, b) for a, b in sorted(ranges)] and sum(b - a for a, b in ranges) == total
    return ranges


def _scaler_shard(rank):
    rng = np.random.default_rng(3)
    X = (rng.standard_normal((61, 40)) * rng.uniform(0.1, 4, 40) + rng.uniform(-2, 2, 40)).astype(np.float32)
    X[:, 3] = 0.75  # constant column -> scale 1
    return X, np.array_split(X, WORLD)[rank]


def _worker(rank, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import hlmc_amd
    from hlmc_amd.features import scaler_finalize

    # ---- gradient SUM all-reduce through Trainer.allreduce_grads, bucket by bucket over the engine's own
    #      gradient buckets (fp32 and bf16 wire formats)
    flat = _shard_grads(rank)
    buckets = _engine_buckets(flat.numel())
    ns = types.SimpleNamespace(gflat=flat.clone(), grad_dtype=torch.float32, process_group=None, buckets=buckets)
    hlmc_amd.Trainer.allreduce_grads(ns)
    ns16 = types.SimpleNamespace(gflat=flat.clone(), grad_dtype=torch.bfloat16, process_group=None, buckets=buckets)
    hlmc_amd.Trainer.allreduce_grads(ns16)
    # the asynchronous bf16 wire handle: every bucket in flight first, then wait() copies the reduced wire back
    from hlmc_amd.train import _allreduce_sum
    ga = flat.clone()
    works = [_allreduce_sum(ga[lo:hi], torch.bfloat16, None, async_op=True) for lo, hi in buckets]
    for w in works:
        assert w.wait() and w.wait()          # a second wait is a no-op

    # ---- BatchNorm running statistics: flat views + rank 0 broadcast (DDP broadcast_buffers)
    torch.manual_seed(42)
    model = hlmc_amd.HybridVAE(128, 768, (128, 128), audio_only=True)
    keys = list(model.state_dict())
    for i, b in enumerate(m for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)):
        b.running_mean.fill_(10.0 * rank + i)
        b.running_var.fill_(1.0 + rank)
    flat = model._flatten_bn_buffers()
    assert list(model.state_dict()) == keys
    trn = types.SimpleNamespace(bn_flat=flat, _comm=None, process_group=None)
    hlmc_amd.Trainer._broadcast_buffers_after_forward(trn)
    bn_state = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}

    # ---- distributed StandardScaler statistics (numpy stands in for the f64 column-sum kernels)
    _, shard = _scaler_shard(rank)
    n = torch.tensor([float(shard.shape[0])], dtype=torch.float64)
    s = torch.from_numpy(shard.astype(np.float64).sum(0))
    dist.all_reduce(n)
    dist.all_reduce(s)
    mean = s / float(n.item())
    d = torch.from_numpy(shard.astype(np.float64)) - mean
    corr, m2 = d.sum(0), (d * d).sum(0)
    dist.all_reduce(corr)
    dist.all_reduce(m2)
    mean, var, scale = scaler_finalize(float(n.item()), s, corr, m2)
    torch.save({"g32": ns.gflat, "g16": ns16.gflat, "g16a": ga, "mean": mean, "var": var, "scale": scale, "bn": bn_state},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_and_distributed_scaler():
    from sklearn.preprocessing import StandardScaler as SkScaler
    with tempfile.TemporaryDirectory() as outdir:
        port = 29500 + (os.getpid() % 2000)
        mp.spawn(_worker, args=(port, outdir), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    ref = _shard_grads(0) + _shard_grads(1)
    for r in res:
        assert torch.equal(r["g32"], ref), "fp32 SUM all-reduce must equal the per-shard gradient sum exactly"
        rel = float((r["g16"] - ref).norm() / ref.norm())
        assert rel < 1e-2, rel
        assert torch.equal(r["g16a"], r["g16"]), "async bf16 wire == blocking bf16 wire"
    assert torch.equal(res[0]["g32"], res[1]["g32"])
    X, _ = _scaler_shard(0)
    sk = SkScaler().fit(X)
    for r in res:
        np.testing.assert_allclose(r["mean"].numpy(), sk.mean_, rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(r["var"].numpy(), sk.var_, rtol=1e-9, atol=1e-15)
        np.testing.assert_allclose(r["scale"].numpy(), sk.scale_, rtol=1e-9)
    assert res[0]["scale"][3] == 1.0
    for k, v in res[1]["bn"].items():   # every rank holds rank 0's running statistics
        assert torch.equal(v, res[0]["bn"][k]), k
    means = [float(v.reshape(-1)[0]) for k, v in res[1]["bn"].items() if k.endswith("running_mean")]
    assert means == [float(i) for i in range(len(means))]           # rank 0 filled 10 * 0 + i
    assert all(float(v.max()) == float(v.min()) == 1.0 for k, v in res[1]["bn"].items() if k.endswith("running_var"))


def test_pipeline_shards_and_equal_step_counts():
    """run_pipeline's data-parallel split: contiguous shards covering every clip once, and every rank taking the
    same number of train steps (each step all-reduces) with >= 2 rows per batch and every shard clip trained."""
    from hlmc_amd.pipeline import local_batches, shard_bounds
    for n, world, batch in [(16, 1, 16), (16, 2, 8), (17, 2, 8), (100, 8, 4), (9, 2, 4), (10, 3, 2), (7, 2, 2),
                            (100000, 8, 256), (20000, 8, 256), (5, 2, 8), (3, 1, 2)]:
        bounds = shard_bounds(n, world)
        assert bounds[0][0] == 0 and bounds[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
        sizes = [hi - lo for lo, hi in bounds]
        assert max(sizes) - min(sizes) <= 1
        plans = [local_batches(sizes, r, batch) for r in range(world)]
        assert len({len(p) for p in plans}) == 1
        for p, size in zip(plans, sizes):
            assert p[0][0] == 0 and p[-1][1] == size and all(a[1] == b[0] for a, b in zip(p, p[1:]))
            assert all(b - a >= 2 for a, b in p)


def test_checkpoint_rng_keying_round_trip():
    """Trainer.state_dict stores the un-keyed Philox seed; load_state_dict re-keys it for the loading rank
    (hlmc_amd.train.keyed_seed / rank_rng_key): rank 0's checkpoint gives every rank its own stream back."""
    from hlmc_amd.train import keyed_seed, rank_rng_key
    base = 0x1234_5678_9ABC_DEF0
    assert rank_rng_key(0) == 0
    keys = [rank_rng_key(r) for r in range(8)]
    assert len(set(keys)) == 8
    for r, k in enumerate(keys):
        live = keyed_seed(base, k)
        assert keyed_seed(live, -k) == base                     # rank r saves the base
        assert keyed_seed(keyed_seed(live, -k), k) == live      # and gets its own stream back
    assert keyed_seed(2 ** 64 - 1, 1) == 0
