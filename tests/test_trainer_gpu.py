"""The fused Trainer step (one native call sequence, no host sync) equals the autograd path
(model -> loss_function -> backward -> hlmc Adam) bit-for-bit up to float rounding."""
import pytest
import torch

import hlmc_amd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("audio_only", [False, True])
def test_trainer_equals_autograd_path(cuda, audio_only):
    torch.manual_seed(42)
    a = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=audio_only).cuda()
    torch.manual_seed(42)
    b = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=audio_only).cuda()
    opt = hlmc_amd.Adam(a.parameters(), lr=1e-4)
    tr = hlmc_amd.Trainer(b, lr=1e-4)
    g = torch.Generator().manual_seed(0)
    for step in range(3):
        audio = torch.randn(8, 1, 128, 128, generator=g).cuda()
        text = (torch.randn(8, 384, generator=g) / 384 ** 0.5).cuda()
        eps = torch.randn(8, 128, generator=g).cuda()
        opt.zero_grad()
        out = a(audio, None if audio_only else text, eps=eps)
        loss = hlmc_amd.loss_function(out[0], audio, out[1], None if audio_only else text, out[2], out[3])
        loss[0].backward()
        opt.step()
        sums = tr.step(audio, None if audio_only else text, eps=eps)
        tot = tr.loss_tuple(sums)[0]
        assert abs(tot - float(loss[0])) <= 1e-6 * abs(float(loss[0]))
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-7, msg=n)


def test_trainer_bf16_loss_decreases(cuda):
    torch.manual_seed(0)
    m = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True, compute_dtype="bf16").cuda()
    tr = hlmc_amd.Trainer(m, lr=1e-3)
    g = torch.Generator(device=cuda).manual_seed(1)
    audio = torch.randn(32, 1, 128, 128, device=cuda, generator=g)
    first = last = None
    for i in range(20):
        tot = tr.loss_tuple(tr.step(audio))[0]
        first = tot if first is None else first
        last = tot
    assert last < 0.9 * first


@pytest.mark.parametrize("kind", ["hybrid", "cvae"])
def test_trainer_dp_overlapped_allreduce_world1(cuda, kind):
    """The DP path (per-bucket RCCL all-reduces on a comm stream gated on backward's bucket events, Adam
    waiting on them) in a 1-rank NCCL group: parameters must equal the non-distributed Trainer's exactly."""
    import os
    import torch.distributed as dist
    own = not dist.is_initialized()
    if own:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29600 + os.getpid() % 1000))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda)
    try:
        def make():
            torch.manual_seed(42)
            if kind == "hybrid":
                m = hlmc_amd.HybridVAE(128, 384, (128, 128), compute_dtype="bf16").cuda()
            else:
                m = hlmc_amd.ConditionalVAE(64, 384, 10, (128, 128), compute_dtype="bf16").cuda()
            return m
        a, b = make(), make()
        ta = hlmc_amd.Trainer(a, lr=1e-3)
        tb = hlmc_amd.Trainer(b, lr=1e-3, distributed=True)
        assert len(tb.buckets) >= 3
        g = torch.Generator().manual_seed(0)
        for _ in range(3):
            audio = torch.randn(16, 1, 128, 128, generator=g).cuda()
            text = (torch.randn(16, 384, generator=g) / 384 ** 0.5).cuda()
            eps = torch.randn(16, a.latent_dim, generator=g).cuda()
            extra = ()
            if kind == "cvae":
                extra = (torch.nn.functional.one_hot(torch.arange(16) % 10, 10).float().cuda(),)
            sa = ta.step(audio, text, *extra, eps=eps)
            sb = tb.step(audio, text, *extra, eps=eps)
            assert torch.equal(sa, sb)
        torch.cuda.synchronize()
        for (n, p), q in zip(a.named_parameters(), b.parameters()):
            assert torch.equal(p, q), n
    finally:
        if own:
            dist.destroy_process_group()


def test_graphed_step_equals_eager(cuda):
    """GraphedStep (whole step captured into a HIP graph, Adam coefficients staged per replay) updates the
    parameters exactly like eager Trainer.step on the same batches."""
    def make():
        torch.manual_seed(42)
        return hlmc_amd.HybridVAE(128, 384, (128, 128), compute_dtype="bf16").cuda()
    a, b = make(), make()
    ta = hlmc_amd.Trainer(a, lr=1e-3)
    tb = hlmc_amd.Trainer(b, lr=1e-3)
    g = torch.Generator().manual_seed(3)
    batches = [(torch.randn(8, 1, 128, 128, generator=g), torch.randn(8, 384, generator=g) / 384 ** 0.5,
                torch.randn(8, 128, generator=g)) for _ in range(4)]
    audio, text, eps = (t.clone().cuda() for t in batches[0])

    def body():
        return tb.step(audio, text, eps=eps)

    gs = hlmc_amd.GraphedStep(tb, body, warmup=1)   # the warmup is batch 0's real step
    for i, (x, t, e) in enumerate(batches):
        sa = ta.step(x.cuda(), t.cuda(), eps=e.cuda())
        if i > 0:
            audio.copy_(x)
            text.copy_(t)
            eps.copy_(e)
            sb = gs()
            torch.cuda.synchronize()
            assert torch.equal(sa, sb), i
    torch.cuda.synchronize()
    assert ta.step_count == tb.step_count == 4
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n
    gs.release()


def test_checkpoint_resume_restores_noise_stream(cuda):
    """model.state_dict() + Trainer.state_dict() (Adam moments, step count, the engine's Philox (seed, offset))
    resume a run bit for bit, device-drawn reparameterisation noise included."""
    def make():
        torch.manual_seed(42)
        m = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True).cuda()
        return m, hlmc_amd.Trainer(m, lr=1e-3)

    g = torch.Generator().manual_seed(3)
    batches = [torch.randn(8, 1, 128, 128, generator=g).cuda() for _ in range(3)]
    m, tr = make()
    for x in batches[:2]:
        tr.step(x)
    ck_model = {k: v.clone() for k, v in m.state_dict().items()}
    ck_tr = tr.state_dict()
    assert ck_tr["rng"][1] > 0   # the offset advanced past the two steps' draws
    tr.step(batches[2])
    want = {k: v.clone() for k, v in m.state_dict().items()}
    m2, tr2 = make()
    m2.load_state_dict(ck_model)
    tr2.load_state_dict(ck_tr)
    tr2.step(batches[2])
    for k, v in m2.state_dict().items():
        assert torch.equal(v, want[k]), k


def test_rng_state_round_trip(cuda):
    torch.manual_seed(7)
    m = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True).cuda()
    st = m.get_rng_state()
    assert st[0] == 7
    m.set_rng_state((123, 456))
    assert m.get_rng_state() == (123, 456)
