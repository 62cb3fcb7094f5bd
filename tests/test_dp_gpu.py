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
Over STEPS consecutive steps (a fresh batch per rank and step): every step's forward on every rank starts from
rank 0's post-previous-step statistics (the broadcast overlapping the next forward), so after step k both ranks
hold the oracle chain's statistics — rank 0's shard run through the chain's parameters from rank 0's step-(k-1)
statistics — and the step-k reduced gradient equals the oracle's shard sum at the chain parameters (which are
torch Adam applied to the reduced gradients of steps 0..k-1).
The bf16-compute case (the N > 1 bench's arithmetic: bf16 activations / MFMA operands, fp32 wire) runs the same chain
with the f64 yardstick at bf16's tolerance: the reduced gradient within 0.15 relative L2 of the float64 shard sum (the
B = 4 bound of test_models_gpu.test_bf16_mode_tracks_fp32) and no further from it than 8x the fp32 oracle's own error
or 0.15, whichever is larger; ranks bit-identical; parameters = torch Adam on the reduced gradient.
Every worker also checks the checkpoint noise contract: Trainer.state_dict() stores the un-keyed Philox seed (equal on
every rank), and loading rank 0's checkpoint on every rank restores each rank's own keyed stream (ranks keep drawing
different eps after a resume).
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
STEPS = 3


def _batch(rank, step=0):
    g = torch.Generator().manual_seed(100 + rank + 10 * step)
    return torch.randn(B, 1, 128, 128, generator=g), torch.randn(B, 128, generator=g)


def _worker(rank, port, outdir, grad_dtype, compute="fp32"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import hlmc_amd
    torch.cuda.set_device(0)
    torch.manual_seed(42)
    m = hlmc_amd.HybridVAE(128, 768, (128, 128), audio_only=True, compute_dtype=compute).cuda()
    tr = hlmc_amd.Trainer(m, lr=1e-4, distributed=True, grad_dtype=grad_dtype)
    assert tr._comm is not None and len(tr.buckets) == 4 and tr.broadcast_buffers
    steps = []
    for k in range(STEPS):
        audio, eps = _batch(rank, k)
        tr.step(audio.cuda(), None, eps=eps.cuda())
        torch.cuda.synchronize()
        steps.append({"grad": tr.gflat.detach().cpu().clone(),
                      "params": {n: p.detach().cpu().clone() for n, p in m.named_parameters()},
                      "buffers": {n: b.detach().cpu().clone() for n, b in m.named_buffers()}})
    # checkpoint noise contract (Trainer.state_dict / load_state_dict under DP)
    from hlmc_amd.train import keyed_seed, rank_rng_key
    sd = tr.state_dict()
    live = m.get_rng_state()
    bases = [None] * WORLD
    dist.all_gather_object(bases, tuple(sd["rng"]))
    lives = [None] * WORLD
    dist.all_gather_object(lives, live)
    box = [sd if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    tr.load_state_dict(box[0])
    resumed = m.get_rng_state()
    steps.append({"rng": {"bases": bases, "lives": lives, "live": live, "resumed": resumed,
                          "expect": (keyed_seed(bases[0][0], rank_rng_key(rank)), bases[0][1])}})
    torch.save(steps, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _oracle_shards(params, buffers, step):
    """Per-shard gradients of the oracle model at the given parameters / BN buffers (every rank's forward starts from
    the same broadcast statistics), their sum, the float64 sum and its kink-flipped twin (the yardstick of
    test_models_gpu.compare_step), and rank 0's BN statistics after its forward."""
    from oracle import models_oracle as OM
    from tests.test_models_gpu import oracle64_with_kink_envelope
    total, buf0, t64, t64f = None, None, None, None
    for rank in range(WORLD):
        torch.manual_seed(42)
        ora = OM.HybridVAE(128, 768, (128, 128), audio_only=True)
        with torch.no_grad():
            for n, p in ora.named_parameters():
                p.copy_(params[n])
            for n, b in ora.named_buffers():
                b.copy_(buffers[n])
        audio, eps = _batch(rank, step)
        m64, m64f = oracle64_with_kink_envelope({"kind": "hybrid"}, ora, [audio, None], eps, None)
        g64 = torch.cat([p.grad.reshape(-1) for p in m64.parameters()])
        g64f = torch.cat([p.grad.reshape(-1) for p in m64f.parameters()])
        t64 = g64 if t64 is None else t64 + g64
        t64f = g64f if t64f is None else t64f + g64f
        out = ora(audio, None, eps=eps)
        OM.loss_function(out[0], audio, None, None, out[2], out[3])[0].backward()
        g = torch.cat([p.grad.reshape(-1) for p in ora.parameters()])
        total = g if total is None else total + g
        if rank == 0:
            buf0 = {n: b.clone() for n, b in ora.named_buffers()}
    return total, buf0, t64, t64f


def _bn_fed_bias(name):
    # audio_encoder.{0,3,...}.bias / audio_decoder.{1,4,...,13}.bias: conv biases directly followed by a BatchNorm
    parts = name.split(".")
    if parts[-1] != "bias" or parts[0] not in ("audio_encoder", "audio_decoder"):
        return False
    i = int(parts[1])
    return (i % 3 == 0) if parts[0] == "audio_encoder" else (i % 3 == 1 and i < 16)


@pytest.mark.parametrize("grad_dtype,compute", [(torch.float32, "fp32"), (torch.bfloat16, "fp32"),
                                                (torch.float32, "bf16")],
                         ids=["fp32_wire", "bf16_wire", "bf16_compute"])
def test_dp_two_ranks_match_oracle(cuda, grad_dtype, compute):
    with tempfile.TemporaryDirectory() as outdir:
        port = 29700 + (os.getpid() % 300) + {"fp32_wire": 0, "bf16_wire": 300, "bf16_compute": 600}[
            ("bf16_compute" if compute == "bf16" else "fp32_wire" if grad_dtype == torch.float32 else "bf16_wire")]
        mp.spawn(_worker, args=(port, outdir, grad_dtype, compute), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    # the checkpoint noise contract: un-keyed base seed on every rank, each rank's own keyed stream after the resume
    rngs = [r[-1]["rng"] for r in res]
    assert rngs[0]["bases"][0] == rngs[0]["bases"][1] and rngs[0]["lives"][0] != rngs[0]["lives"][1]
    for r in rngs:
        assert tuple(r["resumed"]) == tuple(r["expect"]) == tuple(r["live"]), r
    assert rngs[0]["resumed"][0] != rngs[1]["resumed"][0]
    from oracle import models_oracle as OM
    torch.manual_seed(42)
    chain = OM.HybridVAE(128, 768, (128, 128), audio_only=True)
    names = [n for n, _ in chain.named_parameters()]
    shapes = [p.shape for p in chain.parameters()]
    offs, o = [], 0
    for sh in shapes:
        offs.append((o, o + sh.numel()))
        o += sh.numel()
    ps = [p.detach().clone().requires_grad_(True) for p in chain.parameters()]
    opt = torch.optim.Adam(ps, lr=1e-4)
    bufs = {n: b.detach().clone() for n, b in chain.named_buffers()}
    for k in range(STEPS):  # the chain follows the engine's own parameters (checked = torch Adam on its gradient)
        r0, r1 = res[0][k], res[1][k]
        # ranks agree bit for bit
        assert torch.equal(r0["grad"], r1["grad"]), k
        for n in r0["params"]:
            assert torch.equal(r0["params"][n], r1["params"][n]), f"step {k}: ranks diverged at {n}"
        for n in r0["buffers"]:
            assert torch.equal(r0["buffers"][n], r1["buffers"][n]), f"step {k}: BN buffer {n} differs across ranks"
        # reduced gradient = oracle per-shard SUM at the chain's parameters and broadcast statistics
        ref, buf0, ref64, ref64f = _oracle_shards({n: p.detach() for n, p in zip(names, ps)}, bufs, k)
        got = r0["grad"]
        keep = torch.ones_like(ref, dtype=torch.bool)
        for name, (a, b) in zip(names, offs):
            if _bn_fed_bias(name):
                keep[a:b] = False
                wa, wb = offs[names.index(name[:-4] + "weight")]
                btol_b = 2e-2 if compute == "bf16" else 1e-3
                assert float((got[a:b] - ref[a:b]).abs().max()) <= btol_b * float(ref[wa:wb].abs().max()) + 1e-5, name
        err = float((got[keep] - ref[keep]).norm() / ref[keep].norm())
        def rel64(a):
            a = a[keep].double()
            return float((a - ref64[keep]).norm() / ref64[keep].norm())
        if compute == "bf16":
            e_ours, e_ref = rel64(got), rel64(ref)
            bound = max(0.15, 8 * e_ref)
            print(f"step {k}: bf16-compute DP gradient vs f64 shard sum: ours {e_ours:.2e}, fp32 oracle {e_ref:.2e} "
                  f"(bound {bound:.2e})")
            assert e_ours <= bound, k
        elif grad_dtype == torch.float32:
            e_ours, e_ref, e_kink = rel64(got), rel64(ref), rel64(ref64f)
            bound = max(1e-3, 8 * e_ref) + 1.5 * e_kink
            print(f"step {k}: DP gradient vs f64 shard sum: ours {e_ours:.2e}, fp32 oracle {e_ref:.2e}, "
                  f"kink envelope {e_kink:.2e} (bound {bound:.2e}); vs fp32 oracle {err:.2e}")
            assert e_ours <= bound, k
        else:
            print(f"step {k}: DP gradient vs oracle shard sum (bf16 wire): rel L2 {err:.2e}")
            assert err <= 2e-2, k
        # parameters = torch Adam on the reduced gradient (the chain continues from them)
        for p, (a, b) in zip(ps, offs):
            p.grad = got[a:b].view_as(p).clone()
        opt.step()
        for name, p in zip(names, ps):
            torch.testing.assert_close(r0["params"][name], p.detach(), rtol=1e-6, atol=1e-7, msg=f"step {k}: {name}")
        # running statistics = rank 0's after its forward from the broadcast statistics (DDP broadcast_buffers)
        btol = 5e-2 if compute == "bf16" else 1e-4  # bf16: test_models_gpu.test_bf16_mode_tracks_fp32's buffer bound
        for n, b in buf0.items():
            if b.dtype.is_floating_point:
                assert float((r1["buffers"][n] - b).norm() / max(float(b.norm()), 1e-30)) < btol, (k, n)
            else:
                assert torch.equal(r1["buffers"][n], b), (k, n)
        bufs = buf0
