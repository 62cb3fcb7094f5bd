"""Data-parallel Trainer on the GPU with 2 ranks (both on cuda:0, gloo process group — a 1-GPU box cannot
host two RCCL ranks on one device) checked against the ORACLE: the bucketed all-reduce path of
Trainer(distributed=True) — per-bucket comm-stream all_reduce gated by the engine's backward events, the BN
buffer broadcast, Adam waiting on the comm stream — must leave both ranks with

  * the SUM of the per-shard gradients of the oracle model (tests/golden-pinned restatement of the reference
    HybridVAE, seed-42 weights) — global relative L2 <= 1e-3 in fp32 (conv biases feeding train-mode BN have
    a zero true gradient and are compared absolutely), <= 2e-2 for the bf16 wire;
  * identical parameters, equal to torch.optim.Adam applied to that reduced gradient;
  * identical BatchNorm running statistics equal to rank 0's (DDP broadcast_buffers), i.e. the oracle's
    statistics after rank 0's shard.
RCCL itself is covered by the 1-rank NCCL test in test_trainer_gpu.py."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2
B = 4


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(B, 1, 128, 128, generator=g), torch.randn(B, 128, generator=g)


def _worker(rank, port, outdir, grad_dtype):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import hlmc_amd
    torch.cuda.set_device(0)
    torch.manual_seed(42)
    m = hlmc_amd.HybridVAE(128, 768, (128, 128), audio_only=True).cuda()
    tr = hlmc_amd.Trainer(m, lr=1e-4, distributed=True, grad_dtype=grad_dtype)
    assert tr._comm is not None and len(tr.buckets) == 4 and tr.broadcast_buffers
    audio, eps = _batch(rank)
    tr.step(audio.cuda(), None, eps=eps.cuda())
    torch.cuda.synchronize()
    torch.save({"grad": tr.gflat.detach().cpu().clone(),
                "params": {n: p.detach().cpu() for n, p in m.named_parameters()},
                "buffers": {n: b.detach().cpu().clone() for n, b in m.named_buffers()}},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _oracle_shards():
    """Per-shard gradients of the oracle model, their sum, and rank 0's BN statistics after its forward."""
    from oracle import models_oracle as OM
    total, buf0 = None, None
    for rank in range(WORLD):
        torch.manual_seed(42)
        ora = OM.HybridVAE(128, 768, (128, 128), audio_only=True)
        audio, eps = _batch(rank)
        out = ora(audio, None, eps=eps)
        OM.loss_function(out[0], audio, None, None, out[2], out[3])[0].backward()
        g = torch.cat([p.grad.reshape(-1) for p in ora.parameters()])
        total = g if total is None else total + g
        if rank == 0:
            buf0 = {n: b.clone() for n, b in ora.named_buffers()}
            names = [n for n, _ in ora.named_parameters()]
            shapes = [p.shape for p in ora.parameters()]
    return total, buf0, names, shapes


def _bn_fed_bias(name):
    # audio_encoder.{0,3,...}.bias / audio_decoder.{1,4,...,13}.bias: conv biases directly followed by a BatchNorm
    parts = name.split(".")
    if parts[-1] != "bias" or parts[0] not in ("audio_encoder", "audio_decoder"):
        return False
    i = int(parts[1])
    return (i % 3 == 0) if parts[0] == "audio_encoder" else (i % 3 == 1 and i < 16)


@pytest.mark.parametrize("grad_dtype", [torch.float32, torch.bfloat16], ids=["fp32_wire", "bf16_wire"])
def test_dp_two_ranks_match_oracle(cuda, grad_dtype):
    with tempfile.TemporaryDirectory() as outdir:
        port = 29700 + (os.getpid() % 500) + (0 if grad_dtype == torch.float32 else 500)
        mp.spawn(_worker, args=(port, outdir, grad_dtype), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    # ranks agree bit for bit
    assert torch.equal(res[0]["grad"], res[1]["grad"])
    for n in res[0]["params"]:
        assert torch.equal(res[0]["params"][n], res[1]["params"][n]), f"ranks diverged at {n}"
    for n in res[0]["buffers"]:
        assert torch.equal(res[0]["buffers"][n], res[1]["buffers"][n]), f"BN buffer {n} differs across ranks"
    # reduced gradient = oracle per-shard SUM
    ref, buf0, names, shapes = _oracle_shards()
    got = res[0]["grad"]
    offs, o = [], 0
    for s in shapes:
        offs.append((o, o + s.numel()))
        o += s.numel()
    keep = torch.ones_like(ref, dtype=torch.bool)
    for name, (a, b) in zip(names, offs):
        if _bn_fed_bias(name):
            keep[a:b] = False
            wa, wb = offs[names.index(name[:-4] + "weight")]
            assert float((got[a:b] - ref[a:b]).abs().max()) <= 1e-3 * float(ref[wa:wb].abs().max()) + 1e-5, name
    tol = 1e-3 if grad_dtype == torch.float32 else 2e-2
    err = float((got[keep] - ref[keep]).norm() / ref[keep].norm())
    print(f"DP gradient vs oracle shard sum ({grad_dtype}): rel L2 {err:.2e}")
    assert err <= tol
    # parameters = torch Adam on the reduced gradient
    torch.manual_seed(42)
    from oracle import models_oracle as OM
    init = OM.HybridVAE(128, 768, (128, 128), audio_only=True)
    ps = [p.detach().clone().requires_grad_(True) for p in init.parameters()]
    for p, (a, b) in zip(ps, offs):
        p.grad = got[a:b].view_as(p).clone()
    torch.optim.Adam(ps, lr=1e-4).step()
    for name, p in zip(names, ps):
        torch.testing.assert_close(res[0]["params"][name], p.detach(), rtol=1e-6, atol=1e-7, msg=name)
    # running statistics = rank 0's (DDP broadcast_buffers)
    for n, b in buf0.items():
        if b.dtype.is_floating_point:
            assert float((res[1]["buffers"][n] - b).norm() / max(float(b.norm()), 1e-30)) < 1e-4, n
        else:
            assert torch.equal(res[1]["buffers"][n], b), n
