"""Data-parallel Trainer on the GPU with 2 ranks (both on cuda:0, gloo process group — a 1-GPU box cannot
host two RCCL ranks on one device): the bucketed all-reduce path of Trainer(distributed=True) — per-bucket
comm-stream all_reduce gated by the engine's backward events, Adam waiting on the work handles — must leave
both ranks with identical parameters equal to a single-process replay that sums the two shards' gradients
explicitly.  RCCL itself is covered by the 1-rank NCCL test in test_trainer_gpu.py."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2


def _batch(rank, step):
    g = torch.Generator().manual_seed(100 * step + rank)
    return (torch.randn(8, 1, 128, 128, generator=g), torch.randn(8, 128, generator=g))


def _worker(rank, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import hlmc_amd
    torch.cuda.set_device(0)
    torch.manual_seed(42)
    m = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True, compute_dtype="bf16").cuda()
    tr = hlmc_amd.Trainer(m, lr=1e-3, distributed=True)
    assert tr._comm is not None and len(tr.buckets) == 4
    for step in range(2):
        audio, eps = _batch(rank, step)
        tr.step(audio.cuda(), None, eps=eps.cuda())
    torch.cuda.synchronize()
    torch.save({n: p.detach().cpu() for n, p in m.named_parameters()}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_two_ranks_bucketed_allreduce(cuda):
    import hlmc_amd
    with tempfile.TemporaryDirectory() as outdir:
        port = 29700 + (os.getpid() % 1000)
        mp.spawn(_worker, args=(port, outdir), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    for n in res[0]:
        assert torch.equal(res[0][n], res[1][n]), f"ranks diverged at {n}"
    # single-process replay: per-shard gradients through the autograd path, summed, then the same Adam
    torch.manual_seed(42)
    m = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True, compute_dtype="bf16").cuda()
    opt = hlmc_amd.Adam(m.parameters(), lr=1e-3)
    for step in range(2):
        total = None
        for rank in range(WORLD):
            audio, eps = _batch(rank, step)
            audio = audio.cuda()
            opt.zero_grad()
            out = m(audio, None, eps=eps.cuda())
            loss = hlmc_amd.loss_function(out[0], audio, None, None, out[2], out[3])
            loss[0].backward()
            g = [p.grad.detach().clone() for p in m.parameters()]
            total = g if total is None else [a + b for a, b in zip(total, g)]
        for p, g in zip(m.parameters(), total):
            p.grad.copy_(g)
        opt.step()
    torch.cuda.synchronize()
    for n, p in m.named_parameters():
        torch.testing.assert_close(res[0][n], p.detach().cpu(), rtol=1e-5, atol=1e-6, msg=n)
