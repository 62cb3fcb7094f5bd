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
The three model families of BASELINE configs[1]-[3] run this chain: the audio-only ConvVAE (fp32 wire, bf16 wire,
bf16 compute), the hybrid ConvVAE with 384-d lyrics (config[2], "DDP 8x": its text encoder's BatchNorm1d buffers ride the
same broadcast and its text decoder heads the first bucket, engine.cpp HybridNet bucket_starts) and the genre-conditioned
ConditionalVAE (config[3], "DDP 8x": latent 64, 768-d lyrics, one-hot genres); reference models
src/Convolutional_VAE.py:75-194 and src/Conditional_VAE.py:109-246.
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


# model family -> (engine constructor, oracle constructor, latent dim, lyric dim or None, genre classes or None)
MODELS = {
    "audio": (lambda h, c: h.HybridVAE(128, 768, (128, 128), audio_only=True, compute_dtype=c),
              lambda OM: OM.HybridVAE(128, 768, (128, 128), audio_only=True), 128, None, None),
    "hybrid384": (lambda h, c: h.HybridVAE(128, 384, (128, 128), compute_dtype=c),
                  lambda OM: OM.HybridVAE(128, 384, (128, 128)), 128, 384, None),
    "cvae": (lambda h, c: h.ConditionalVAE(64, 768, 10, (128, 128), compute_dtype=c),
             lambda OM: OM.ConditionalVAE(64, 768, 10, (128, 128)), 64, 768, 10),
}


def _batch(kind, rank, step=0):
    """(audio, text or None, one-hot genres or None, eps) of one rank's shard at one step."""
    _, _, lat, td, nc = MODELS[kind]
    g = torch.Generator().manual_seed(100 + rank + 10 * step)
    audio = torch.randn(B, 1, 128, 128, generator=g)
    eps = torch.randn(B, lat, generator=g)
    text = torch.randn(B, td, generator=g) / td ** 0.5 if td else None
    cond = torch.nn.functional.one_hot(torch.randint(0, nc, (B,), generator=g), nc).float() if nc else None
    return audio, text, cond, eps


def _oracle_loss(kind, out, audio, text):
    from oracle import models_oracle as OM
    if kind == "cvae":
        return OM.cvae_loss_function(out[0], audio, out[1], text, out[2], out[3], beta=4.0)
    return OM.loss_function(out[0], audio, out[1], text, out[2], out[3])


def _worker(rank, port, outdir, grad_dtype, compute="fp32", kind="audio"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import hlmc_amd
    torch.cuda.set_device(0)
    torch.manual_seed(42)
    m = MODELS[kind][0](hlmc_amd, compute).cuda()
    tr = hlmc_amd.Trainer(m, lr=1e-4, distributed=True, grad_dtype=grad_dtype)
    assert tr._comm is not None and len(tr.buckets) == 4 and tr.broadcast_buffers
    steps = []
    for k in range(STEPS):
        audio, text, cond, eps = _batch(kind, rank, k)
        tr.step(audio.cuda(), None if text is None else text.cuda(), None if cond is None else cond.cuda(),
                eps=eps.cuda())
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


def _oracle_shards(kind, params, buffers, step):
    """Per-shard gradients of the oracle model at the given parameters / BN buffers (every rank's forward starts from
    the same broadcast statistics), their sum, the float64 sum and its kink-flipped twin (the yardstick of
    test_models_gpu.compare_step), and rank 0's BN statistics after its forward."""
    from oracle import models_oracle as OM
    from tests.test_models_gpu import oracle64_with_kink_envelope
    total, buf0, t64, t64f = None, None, None, None
    for rank in range(WORLD):
        torch.manual_seed(42)
        ora = MODELS[kind][1](OM)
        with torch.no_grad():
            for n, p in ora.named_parameters():
                p.copy_(params[n])
            for n, b in ora.named_buffers():
                b.copy_(buffers[n])
        audio, text, cond, eps = _batch(kind, rank, step)
        ins = [audio, text, cond] if kind == "cvae" else [audio, text]
        m64, m64f = oracle64_with_kink_envelope({"kind": "cvae" if kind == "cvae" else "hybrid"}, ora, ins, eps, None)
        g64 = torch.cat([p.grad.reshape(-1) for p in m64.parameters()])
        g64f = torch.cat([p.grad.reshape(-1) for p in m64f.parameters()])
        t64 = g64 if t64 is None else t64 + g64
        t64f = g64f if t64f is None else t64f + g64f
        out = ora(*ins, eps=eps)
        _oracle_loss(kind, out, audio, text)[0].backward()
        g = torch.cat([p.grad.reshape(-1) for p in ora.parameters()])
        total = g if total is None else total + g
        if rank == 0:
            buf0 = {n: b.clone() for n, b in ora.named_buffers()}
    return total, buf0, t64, t64f


CASES = {"fp32_wire": (torch.float32, "fp32", "audio"), "bf16_wire": (torch.bfloat16, "fp32", "audio"),
         "bf16_compute": (torch.float32, "bf16", "audio"), "hybrid384_fp32_wire": (torch.float32, "fp32", "hybrid384"),
         "cvae_fp32_wire": (torch.float32, "fp32", "cvae")}


@pytest.mark.parametrize("case", list(CASES))
def test_dp_two_ranks_match_oracle(cuda, case):
    grad_dtype, compute, kind = CASES[case]
    with tempfile.TemporaryDirectory() as outdir:
        port = 29700 + (os.getpid() % 300) + 300 * list(CASES).index(case)
        mp.spawn(_worker, args=(port, outdir, grad_dtype, compute, kind), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    # the checkpoint noise contract: un-keyed base seed on every rank, each rank's own keyed stream after the resume
    rngs = [r[-1]["rng"] for r in res]
    assert rngs[0]["bases"][0] == rngs[0]["bases"][1] and rngs[0]["lives"][0] != rngs[0]["lives"][1]
    for r in rngs:
        assert tuple(r["resumed"]) == tuple(r["expect"]) == tuple(r["live"]), r
    assert rngs[0]["resumed"][0] != rngs[1]["resumed"][0]
    from oracle import models_oracle as OM
    from tests.test_models_gpu import _bias_feeds_bn
    torch.manual_seed(42)
    chain = MODELS[kind][1](OM)
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
        ref, buf0, ref64, ref64f = _oracle_shards(kind, {n: p.detach() for n, p in zip(names, ps)}, bufs, k)
        got = r0["grad"]
        keep = torch.ones_like(ref, dtype=torch.bool)
        for name, (a, b) in zip(names, offs):
            if _bias_feeds_bn(chain, name):
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
