"""Model-level parity: hlmc_amd.{HybridVAE, ConditionalVAE, VAE} (HIP engine, fp32 mode) vs the torch-CPU
oracle (oracle/models_oracle.py, itself pinned bit-exact to the AST-loaded reference classes by
tests/golden/make_golden.py) on the golden fixture cases, from identical weights / inputs / eps.

Tolerances (fp32, per step from shared state — SURVEY §0.6):
  * mu, logvar, reconstructions, ELBO terms: relative error <= 1e-4 (north_star), typically ~1e-6.
  * parameter gradients: relative L2 error vs a float64 run of the oracle <= max(1e-3, 8 x the fp32 oracle's
    own error) per tensor (sum-reduced losses leave a few gradients ill-conditioned in any fp32 order), plus
    a kink envelope: pre-activations within ~8 fp32 ulps of a (Leaky)ReLU kink (|z| <= 1e-6 max|z|; several
    per layer at these sizes) have a rounding-decided derivative, so the allowance adds 1.5 x the change a
    float64 run shows when those derivatives are flipped;
    conv biases that feed train-mode BatchNorm
    have a mathematically-zero gradient (pure rounding noise) and are checked absolutely against the
    scale of their layer's weight gradient.
  * BatchNorm running statistics after the step: relative <= 1e-4.
"""
import copy

import numpy as np
import pytest
import torch

import hlmc_amd
from oracle import models_oracle as OM
from tests.golden import fixtures as FX

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _bias_feeds_bn(model, name):
    """conv / linear biases directly followed by a BatchNorm (zero true gradient)."""
    mods = dict(model.named_modules())
    parent, idx, leaf = name.rsplit(".", 2) if name.count(".") >= 2 else (None, None, None)
    if leaf != "bias" or parent is None:
        return False
    seq = mods.get(parent)
    if not isinstance(seq, torch.nn.Sequential):
        return False
    i = int(idx)
    return i + 1 < len(seq) and isinstance(seq[i + 1], torch.nn.modules.batchnorm._BatchNorm) and not isinstance(
        seq[i], torch.nn.modules.batchnorm._BatchNorm)


def build(case, dtype="fp32"):
    ctor = FX.oracle_ctor(case)
    torch.manual_seed(42)
    ora = {"hybrid": OM.HybridVAE, "cvae": OM.ConditionalVAE, "simple": OM.VAE}[case["kind"]](**ctor)
    torch.manual_seed(42)
    cls = {"hybrid": hlmc_amd.HybridVAE, "cvae": hlmc_amd.ConditionalVAE, "simple": hlmc_amd.VAE}[case["kind"]]
    ours = cls(**ctor, compute_dtype=dtype)
    so, sm = ora.state_dict(), ours.state_dict()
    assert list(so) == list(sm)
    for k in so:
        assert torch.equal(so[k], sm[k]), f"init differs at {k}"
    return ora, ours.cuda()


def run_oracle_step(case, ora, ins, eps, masks=None):
    ora.train()
    if case["kind"] == "simple":
        hooks = []
        it = iter(masks)

        def hook(mod, inp, out):
            m = next(it)
            return inp[0] * m.to(inp[0].dtype) / 0.8

        for mod in ora.modules():
            if isinstance(mod, torch.nn.Dropout):
                hooks.append(mod.register_forward_hook(hook))
        out = ora(*ins, eps=eps)
        for h in hooks:
            h.remove()
        loss = OM.vae_loss(out[0], ins[0], out[1], out[2], beta=0.8)
    else:
        out = ora(*ins, eps=eps)
        if case["kind"] == "hybrid":
            loss = OM.loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3])
        else:
            loss = OM.cvae_loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3], beta=4.0)
    loss[0].backward()
    return out, loss


def run_ours_step(case, ours, ins, eps, mask=None):
    ours.train()
    cins = [None if t is None else t.cuda() for t in ins]
    if case["kind"] == "simple":
        out = ours(cins[0], eps=eps.cuda(), dropout_mask=mask)
        loss = hlmc_amd.vae_loss(out[0], cins[0], out[1], out[2], beta=0.8)
    else:
        out = ours(*cins, eps=eps.cuda())
        if case["kind"] == "hybrid":
            loss = hlmc_amd.loss_function(out[0], cins[0], out[1], cins[1], out[2], out[3])
        else:
            loss = hlmc_amd.cvae_loss_function(out[0], cins[0], out[1], cins[1], out[2], out[3], beta=4.0)
    loss[0].backward()
    return out, loss


def simple_masks(case, B, seed=5):
    g = torch.Generator().manual_seed(seed)
    widths = case["ctor"]["hidden_dims"] + case["ctor"]["hidden_dims"][::-1]
    masks = [(torch.rand(B, w, generator=g) >= 0.2) for w in widths]
    flat = torch.cat([m.reshape(-1) for m in masks]).to(torch.uint8).cuda()
    return masks, flat


KINK_REL = 1e-6  # |z| <= KINK_REL * max|z| of its layer: within ~8 fp32 ulps of a (Leaky)ReLU kink


def _act_modules(model):
    return [m for m in model.modules() if isinstance(m, (torch.nn.LeakyReLU, torch.nn.ReLU))]


def oracle64_with_kink_envelope(case, ora, ins, eps, masks):
    """float64 oracle step, plus a second float64 step with the activation derivative flipped at every
    pre-activation within rounding distance of the kink (where an fp32 implementation's derivative is
    decided by rounding, e.g. |z| = 7e-8 max|z|).  Returns (model64, model64_flipped)."""
    base = copy.deepcopy(ora).double()
    flip = copy.deepcopy(ora).double()
    zs = {}
    hooks = []
    for i, m in enumerate(_act_modules(base)):
        hooks.append(m.register_forward_hook(lambda mod, inp, out, i=i: zs.__setitem__(i, inp[0].detach())))
    run_oracle_step(case, base, [None if t is None else t.double() for t in ins], eps.double(), masks)
    for h in hooks:
        h.remove()
    for i, m in enumerate(_act_modules(flip)):
        z = zs.get(i)
        if z is None:
            continue
        amb = z.abs() <= KINK_REL * z.abs().max()
        if not bool(amb.any()):
            continue
        slope = getattr(m, "negative_slope", 0.0)
        other = torch.where(z > 0, torch.full_like(z, slope), torch.ones_like(z))

        def bhook(mod, gin, gout, amb=amb, other=other):
            g = gin[0].clone()
            g[amb] = gout[0][amb] * other[amb]
            return (g,)
        m.register_full_backward_hook(bhook)
    run_oracle_step(case, flip, [None if t is None else t.double() for t in ins], eps.double(), masks)
    return base, flip


def compare_step(case, ora, ours, tol_out=1e-4, tol_grad=1e-3):
    ins, eps = FX.inputs_fn(case)(0)
    masks, flat = (simple_masks(case, case["B"]) if case["kind"] == "simple" else (None, None))
    # float64 runs of the same oracle: the exact-arithmetic yardstick for the gradient check, and its
    # kink envelope (derivatives flipped where fp32 rounding decides the side of a (Leaky)ReLU kink)
    ora64, ora64f = oracle64_with_kink_envelope(case, ora, ins, eps, masks)
    o_out, o_loss = run_oracle_step(case, ora, ins, eps, masks)
    m_out, m_loss = run_ours_step(case, ours, ins, eps, flat)
    for i, (a, b) in enumerate(zip(m_out, o_out)):
        if a is None or b is None or (case["kind"] == "simple" and i == 3):
            continue
        assert rel(a.detach(), b.detach()) < tol_out, f"output {i}: {rel(a.detach(), b.detach())}"
    for i, (a, b) in enumerate(zip(m_loss, o_loss)):
        if float(b) != 0.0:
            assert abs(float(a) - float(b)) <= tol_out * abs(float(b)) + 1e-6, f"loss {i}: {float(a)} vs {float(b)}"
    onames = dict(ora.named_parameters())
    o64 = dict(ora64.named_parameters())
    o64f = dict(ora64f.named_parameters())
    mparams = dict(ours.named_parameters())
    for name, po in onames.items():
        gm, go = mparams[name].grad, po.grad
        assert gm is not None, name
        if _bias_feeds_bn(ora, name):
            wname = name[:-4] + "weight"
            scale = float(onames[wname].grad.abs().max())
            assert float((gm.cpu() - go).abs().max()) <= 1e-4 * scale + 1e-6, name
        else:
            # as accurate as the reference's own fp32 computation: error vs the float64 gradient within
            # max(tol_grad, 8 x the fp32 oracle's error) (sum-reduced losses make some gradients ill-conditioned),
            # plus the kink envelope (1.5 x the change from flipping the rounding-decided derivatives)
            g64 = o64[name].grad
            e_ref, e_ours, e_kink = rel(go, g64), rel(gm, g64), rel(o64f[name].grad, g64)
            assert e_ours <= max(tol_grad, 8 * e_ref) + 1.5 * e_kink, \
                f"grad {name}: {e_ours:.3e} vs fp32 oracle {e_ref:.3e}, kink envelope {e_kink:.3e}"
    for (n, bo), (_, bm) in zip(ora.named_buffers(), ours.named_buffers()):
        if bo.dtype.is_floating_point:
            assert rel(bm, bo) < tol_out, f"buffer {n}: {rel(bm, bo)}"
        else:
            assert torch.equal(bm.cpu(), bo), n
    return o_loss, m_loss


@pytest.mark.parametrize("name", ["audio_128x128", "hybrid_128x128_td768", "hybrid_128x128_td384", "cvae_128x128",
                                  "simple_370", "hybrid_128x1024_td768", "cvae_128x1024"])
def test_model_step_matches_oracle(cuda, name):
    """One fp32 train step vs the oracle at the 1e-4 contract.  ``audio_128x128`` is BASELINE config[1], the
    benchmarked model: its fixture comes from the reference HybridVAE with the text branch, fusion slice and text
    loss removed by an AST rewrite (tests/golden/make_golden.py ``_AudioOnlyRewrite``), against which the
    restatement is bit-exact."""
    case = FX.case_by_name(name)
    ora, ours = build(case)
    o_loss, m_loss = compare_step(case, ora, ours)
    # the fixture pins the oracle itself (bit-exact to the reference at generation time)
    fx = np.load(f"tests/golden/model_{name}.npz")
    if case["kind"] != "simple":
        np.testing.assert_allclose([float(t) for t in m_loss], fx["loss_step0"], rtol=1e-4, atol=1e-6)


def test_hybrid_audio_only_and_adam(cuda):
    """Audio-only ConvVAE (BASELINE config[1]): one fwd/bwd vs the oracle, then hlmc Adam vs torch Adam on
    the SAME gradients (first-step Adam moves a weight by ~lr*sign(g), so comparing updates across two
    gradient computations would only test the sign of near-zero gradients)."""
    ctor = dict(latent_dim=128, text_dim=768, input_hw=(128, 128), audio_only=True)
    torch.manual_seed(42)
    ora = OM.HybridVAE(**ctor)
    torch.manual_seed(42)
    ours = hlmc_amd.HybridVAE(**ctor).cuda()
    g = torch.Generator().manual_seed(3)
    audio = torch.randn(4, 1, 128, 128, generator=g)
    eps = torch.randn(4, 128, generator=g)
    o = ora(audio, None, eps=eps)
    lo = OM.loss_function(o[0], audio, None, None, o[2], o[3])
    lo[0].backward()
    m = ours(audio.cuda(), None, eps=eps.cuda())
    lm = hlmc_amd.loss_function(m[0], audio.cuda(), None, None, m[2], m[3])
    lm[0].backward()
    assert rel(m[2].detach(), o[2].detach()) < 1e-4
    assert abs(float(lm[0]) - float(lo[0])) < 1e-4 * abs(float(lo[0]))
    # optimizer parity: torch Adam on a CPU copy fed with our gradients
    ref = [p.detach().cpu().clone().requires_grad_(True) for p in ours.parameters()]
    opt_t = torch.optim.Adam(ref, lr=1e-4)
    opt_m = hlmc_amd.Adam(ours.parameters(), lr=1e-4)
    for step in range(3):
        for r, p in zip(ref, ours.parameters()):
            r.grad = p.grad.detach().cpu().clone()
        opt_t.step()
        opt_m.step()
        for r, p in zip(ref, ours.parameters()):
            torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=1e-6, atol=1e-7)
        for p in ours.parameters():
            p.grad.mul_(0.5)


def test_eval_encode_matches_oracle(cuda):
    case = FX.case_by_name("hybrid_128x128_td768")
    ora, ours = build(case)
    ins, _ = FX.inputs_fn(case)(0)
    ora.eval()
    ours.eval()
    with torch.no_grad():
        mo, lo = ora.encode(*ins)
        mm, lm = ours.encode(*[t.cuda() for t in ins])
    assert rel(mm, mo) < 1e-5 and rel(lm, lo) < 1e-5


def _oracle_trained(case, steps=3):
    """The fixture generator's chain on the oracle (tests/golden/make_golden.py run_case): `steps` train-mode
    Adam(lr 1e-4) steps on the per-step fixture inputs, torch.manual_seed(7 + step) before each forward (the
    Simple VAE's dropout masks), so BatchNorm running statistics and weights are the reference's own after
    training.  Returns the oracle in eval mode."""
    torch.manual_seed(42)
    ora = {"hybrid": OM.HybridVAE, "cvae": OM.ConditionalVAE, "simple": OM.VAE}[case["kind"]](**FX.oracle_ctor(case))
    opt = torch.optim.Adam(ora.parameters(), lr=1e-4)
    for step in range(steps):
        ins, eps = FX.inputs_fn(case)(step)
        ora.train()
        opt.zero_grad()
        torch.manual_seed(7 + step)
        out = ora(*ins, eps=eps)
        if case["kind"] == "simple":
            lo = OM.vae_loss(out[0], ins[0], out[1], out[2], beta=0.8)
        elif case["kind"] == "hybrid":
            lo = OM.loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3])
        else:
            lo = OM.cvae_loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3], beta=4.0)
        lo[0].backward()
        opt.step()
    return ora.eval()


@pytest.mark.parametrize("name", ["audio_128x128", "hybrid_128x128_td768", "cvae_128x128", "cvae_128x1024",
                                  "simple_370", "hybrid_128x1024_td768"])
def test_eval_mode_matches_fixture_chain(cuda, name):
    """Latent extraction and the validation forward (row a14): src/Convolutional_VAE.py:286-303 (model.eval();
    encode -> mu), src/Conditional_VAE.py:397-402 (cvae.encode over the whole set under no_grad),
    src/Simple_VAE.py:103-105,225-226 (vae.get_latent_features) and the per-epoch validation loop
    model(audio, text) under model.eval() (src/Convolutional_VAE.py:245-256, src/Conditional_VAE.py:336-345).

      1. the oracle trained by the reference's own 3 Adam steps reproduces the fixture's eval_mu (the reference
         classes' latents): bit-exact on the generating host (tests/test_oracle_cpu.py); another host's CPU
         kernels move it by Adam-amplified rounding (first-step Adam turns rounding noise in the
         zero true gradients of BN-fed conv biases into +-lr moves; measured 8e-5 .. 3.2e-2 on the MI355X box's
         host), bounded at 5e-2;
      2. the engine holding that oracle state (weights + BatchNorm running statistics, load_state_dict): eval
         encode (and get_latent_features) vs the oracle's at 1e-5 relative, and the eval-mode full forward +
         loss (running statistics, eps as given) at the 1e-4 contract."""
    case = FX.case_by_name(name)
    ora = _oracle_trained(case)
    ours = build(case)[1]
    ours.load_state_dict(ora.state_dict())
    ours.eval()
    ins, eps = FX.inputs_fn(case)(0)
    cins = [None if t is None else t.cuda() for t in ins]
    fx = np.load(f"tests/golden/model_{name}.npz")["eval_mu"]
    with torch.no_grad():
        mo, lo = ora.encode(*ins)
        mm, lm = ours.encode(*cins)
    e_fx = rel(mo, torch.from_numpy(fx))
    print(f"{name}: oracle-on-host vs fixture eval_mu {e_fx:.2e}; engine eval mu {rel(mm, mo):.2e}, logvar "
          f"{rel(lm, lo):.2e}; engine vs fixture {rel(mm, torch.from_numpy(fx)):.2e}")
    assert e_fx < 5e-2
    assert rel(mm, mo) < 1e-5 and rel(lm, lo) < 1e-5
    if case["kind"] == "simple":
        with torch.no_grad():
            assert rel(ours.get_latent_features(cins[0]), ora.get_latent_features(ins[0])) < 1e-5
    # the validation loop: eval-mode forward (BatchNorm running statistics, no dropout) + the loss tuple
    with torch.no_grad():
        o_out = ora(*ins, eps=eps)
        m_out = ours(*cins, eps=eps.cuda())
    for i, (a, b) in enumerate(zip(m_out, o_out)):
        if a is None or b is None:
            continue
        assert rel(a, b) < 1e-4, f"eval output {i}: {rel(a, b):.2e}"
    if case["kind"] == "simple":
        lo_, lm_ = (OM.vae_loss(o_out[0], ins[0], o_out[1], o_out[2], beta=0.8),
                    hlmc_amd.vae_loss(m_out[0], cins[0], m_out[1], m_out[2], beta=0.8))
    elif case["kind"] == "hybrid":
        lo_ = OM.loss_function(o_out[0], ins[0], o_out[1], ins[1], o_out[2], o_out[3])
        lm_ = hlmc_amd.loss_function(m_out[0], cins[0], m_out[1], cins[1], m_out[2], m_out[3])
    else:
        lo_ = OM.cvae_loss_function(o_out[0], ins[0], o_out[1], ins[1], o_out[2], o_out[3], beta=4.0)
        lm_ = hlmc_amd.cvae_loss_function(m_out[0], cins[0], m_out[1], cins[1], m_out[2], m_out[3], beta=4.0)
    for a, b in zip(lm_, lo_):
        if float(b) != 0.0:
            assert abs(float(a) - float(b)) <= 1e-4 * abs(float(b)), (float(a), float(b))
    # the running statistics were read, not updated
    for (n, bo), (_, bm) in zip(ora.named_buffers(), ours.named_buffers()):
        assert torch.equal(bm.cpu(), bo), n


def test_bf16_mode_tracks_fp32(cuda):
    """Throughput mode (bf16 activations / MFMA operands, fp32 accumulate + master weights): outputs and
    the ELBO stay within 3e-2 / 2e-2 of the fp32 oracle; gradients within 0.15 relative L2 overall at
    B=4 (BatchNorm over 4-64 rows amplifies bf16 rounding of activations)."""
    case = FX.case_by_name("hybrid_128x128_td768")
    ora, ours = build(case, "bf16")
    ins, eps = FX.inputs_fn(case)(0)
    o_out, o_loss = run_oracle_step(case, ora, ins, eps)
    m_out, m_loss = run_ours_step(case, ours, ins, eps)
    assert rel(m_out[2].detach(), o_out[2].detach()) < 3e-2
    assert abs(float(m_loss[0]) - float(o_loss[0])) < 2e-2 * abs(float(o_loss[0]))
    errs = {n: rel(p.grad, q.grad) for (n, p), q in zip(ours.named_parameters(), ora.parameters())
            if not _bias_feeds_bn(ora, n)}
    print("bf16 per-parameter grad rel err (worst 8):", sorted(errs.items(), key=lambda kv: -kv[1])[:8])
    gm = torch.cat([p.grad.reshape(-1).cpu() for p in ours.parameters()])
    go = torch.cat([p.grad.reshape(-1) for p in ora.parameters()])
    assert rel(gm, go) < 0.15
    # every BatchNorm layer's running statistics (the statistics path of each layer: producer epilogue, split-K
    # moments pass, consumer-side finalize or the next halo kernel's input staging) track the oracle's
    bo = dict(ora.named_buffers())
    for n, b in ours.named_buffers():
        if b.dtype.is_floating_point:
            assert rel(b.detach(), bo[n]) < 5e-2, n
        else:
            assert torch.equal(b.detach().cpu(), bo[n]), n


@pytest.mark.parametrize("train", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("name", ["hybrid_128x128_td768", "cvae_128x128", "simple_370", "hybrid_128x1024_td768"])
def test_decode_matches_oracle(cuda, name, train):
    """decode(z) / decode(z, condition) (src/Convolutional_VAE.py:167-179, src/Conditional_VAE.py:206-225,
    src/Simple_VAE.py:95-96) vs the oracle's decode from identical weights; train mode also checks the
    decoder BatchNorms' running-statistics update."""
    case = FX.case_by_name(name)
    ora, ours = build(case)
    B, Ld = case["B"], case["ctor"]["latent_dim"]
    g = torch.Generator().manual_seed(77)
    z = torch.randn(B, Ld, generator=g)
    ora.train(train)
    ours.train(train)
    if case["kind"] == "cvae":
        cond = torch.nn.functional.one_hot(torch.randint(0, 10, (B,), generator=g), 10).float()
        with torch.no_grad():
            ro = ora.decode(z, cond)
        rm = ours.decode(z.cuda(), cond.cuda())
    elif case["kind"] == "simple":
        masks, flat = simple_masks(case, B)
        nh = len(case["ctor"]["hidden_dims"])
        it = iter(masks[nh:])
        hooks = [m.register_forward_hook(lambda mod, inp, out: inp[0] * next(it).to(inp[0].dtype) / 0.8)
                 for m in ora.decoder.modules() if isinstance(m, torch.nn.Dropout)] if train else []
        with torch.no_grad():
            ro = (ora.decode(z),)
        for h in hooks:
            h.remove()
        rm = (ours.decode(z.cuda(), dropout_mask=flat if train else None),)
    else:
        with torch.no_grad():
            ro = ora.decode(z)
        rm = ours.decode(z.cuda())
    for a, b in zip(rm, ro):
        assert not a.requires_grad
        assert rel(a, b) < 1e-4, f"{name} decode: {rel(a, b)}"
    for (n, bo), (_, bm) in zip(ora.named_buffers(), ours.named_buffers()):
        if bo.dtype.is_floating_point:
            assert rel(bm, bo) < 1e-4, f"buffer {n}: {rel(bm, bo)}"
        else:
            assert torch.equal(bm.cpu(), bo), n


def test_decode_audio_only_and_backward_guard(cuda):
    """Audio-only HybridVAE (config[1]) decode returns (recon, None); a backward without a full forward fails
    loudly instead of reading a decode-only workspace."""
    ctor = dict(latent_dim=128, text_dim=768, input_hw=(128, 128), audio_only=True)
    torch.manual_seed(42)
    ora = OM.HybridVAE(**ctor)
    torch.manual_seed(42)
    ours = hlmc_amd.HybridVAE(**ctor).cuda().eval()
    ora.eval()
    z = torch.randn(3, 128, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ro = ora.decode(z)
    ra, rt = ours.decode(z.cuda())
    assert rt is None and rel(ra, ro[0]) < 1e-4
    from hlmc_amd import _lib as L
    net = ours._native_net()
    ws = net.new_workspace(3, z.device if z.is_cuda else torch.device("cuda"))
    d = torch.zeros(3, 1, 128, 128, device="cuda")
    dm = torch.zeros(3, 128, device="cuda")
    L.check(L.lib().hlmc_net_decode(net.h, L.stream(), 3, 0, L.ptr(z.cuda()), None, None, L.ptr(d), None, ws.data_ptr()))
    with pytest.raises(L.HLMCError, match="full hlmc_net_forward"):
        L.check(L.lib().hlmc_net_backward(net.h, L.stream(), 3, L.ptr(d), None, L.ptr(dm), L.ptr(dm), ws.data_ptr()))


@pytest.mark.parametrize("name", ["audio_128x128", "hybrid_128x128_td768"])
def test_three_adam_steps_match_fixture_trajectory(cuda, name):
    """Three train steps (fwd → ELBO → bwd → hlmc Adam, lr 1e-4) on the fixture's per-step inputs, against the
    reference's own parameter / BN-buffer summaries after steps 1 and 3 (tests/golden/make_golden.py
    run_case: torch.optim.Adam on the AST-loaded reference classes).

    Step-1 Adam moves every weight by lr·g/(|g|+eps) ≈ ±lr, so an entry whose gradient sign is decided by
    rounding (conv biases feeding train-mode BN: true gradient 0; pre-activations at a LeakyReLU kink) can
    differ by 2·lr.  Contract: those BN-fed biases are excluded; of the sampled entries of every other
    parameter ≥ 97% agree within 1e-2·lr after step 1 (≥ 90% after step 3) and all within 2·lr·steps; the
    per-tensor sum rows are not asserted (a few flips move them by 2·lr each).  BN running stats: within
    1e-4 relative + 10·lr absolute (the running means carry the BN-fed biases' drift).

    How many entries a differently-rounded computation keeps within 1e-2·lr after 3 steps depends on the model:
    the float64 oracle (the same chain in exact-er arithmetic) keeps 94 % for the hybrid but only 65 % for the
    audio-only model, whose fusion layer feeds on the audio branch alone.  So the step-3 bar is the float64
    yardstick's own fraction less 0.10 (capped at 0.90), computed here from the oracle chain in float64."""
    case = FX.case_by_name(name)
    fx = np.load(f"tests/golden/model_{name}.npz")
    ora, ours = build(case)
    lr = 1e-4
    yard = _f64_trajectory_fractions(case, fx, lr)
    bars = {0: min(0.97, yard[0] - 0.03), 2: min(0.90, yard[2] - 0.10)}
    opt = hlmc_amd.Adam(ours.parameters(), lr=lr)
    names = [n for n, _ in ours.named_parameters()]
    assert list(fx["param_names"]) == names
    keep = [i for i, n in enumerate(names) if not _bias_feeds_bn(ora, n)]
    for step in range(3):
        ins, eps = FX.inputs_fn(case)(step)
        opt.zero_grad()
        run_ours_step(case, ours, ins, eps)
        opt.step()
        if step in (0, 2):
            got = FX.param_summary(_cpu_copy(ours))
            ref = fx[f"param_summary_after{step + 1}"]
            samp_g, samp_r = got[keep, 2:], ref[keep, 2:]
            d = np.abs(samp_g - samp_r)
            assert float(d.max()) <= 2 * lr * (step + 1) + 1e-6, float(d.max())
            frac = float((d <= 1e-2 * lr).mean())
            print(f"{name} step {step + 1}: {frac:.3f} of samples within 1e-2·lr (float64 oracle {yard[step]:.3f})")
            assert frac >= bars[step], f"step {step + 1}: {frac:.3f} of samples within 1e-2·lr (bar {bars[step]:.3f})"
            bg = FX.buffer_summary(_cpu_copy(ours))[:, 2:]
            br = fx[f"buffer_summary_after{step + 1}"][:, 2:]
            np.testing.assert_allclose(bg, br, rtol=1e-4, atol=10 * lr)


def _f64_trajectory_fractions(case, fx, lr):
    """{0: f, 2: f}: the fraction of the fixture's sampled parameter entries (BN-fed biases excluded) that the
    float64 oracle chain (same init, inputs, eps, torch Adam) keeps within 1e-2·lr of the reference's fp32 chain
    after steps 1 and 3 -- the yardstick of how rounding-sensitive the trajectory is."""
    torch.manual_seed(42)
    ora = OM.HybridVAE(**FX.oracle_ctor(case)).double()
    opt = torch.optim.Adam(ora.parameters(), lr=lr)
    keep = [i for i, (n, _) in enumerate(ora.named_parameters()) if not _bias_feeds_bn(ora, n)]
    out = {}
    for step in range(3):
        ins, eps = FX.inputs_fn(case)(step)
        ins = [None if t is None else t.double() for t in ins]
        ora.train()
        opt.zero_grad()
        o = ora(*ins, eps=eps.double())
        OM.loss_function(o[0], ins[0], o[1], ins[1], o[2], o[3])[0].backward()
        opt.step()
        if step in (0, 2):
            d = np.abs(FX.param_summary(ora)[keep, 2:] - fx[f"param_summary_after{step + 1}"][keep, 2:])
            out[step] = float((d <= 1e-2 * lr).mean())
    return out


class _cpu_copy:
    """Host view of a module's parameters / buffers for the fixture summaries (no module copy)."""

    def __init__(self, model):
        self._p = [(n, p.detach().cpu()) for n, p in model.named_parameters()]
        self._b = [(n, b.detach().cpu()) for n, b in model.named_buffers()]

    def named_parameters(self):
        return iter(self._p)

    def named_buffers(self):
        return iter(self._b)
