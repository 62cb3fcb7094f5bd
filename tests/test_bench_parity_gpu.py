"""Parity of the EXACT benchmarked configuration (bench.py, BASELINE config[1]): 256 clips of synthetic PCM
(bench.synthetic_pcm, generated on the GPU as the bench does) -> bench.MelStage (HIP mel-dB 128x128 with the
HIP StandardScaler z-score fused into the dB pass) -> audio-only HybridVAE 128x128 -> one fused Trainer.step (forward, ELBO sums,
backward, Adam), the B = 256 GEMM plans (split-K factors, sub-pixel tiles, LDS-DMA variants) the bench
times.  Compared with the oracle chain: oracle/mel_oracle.py (numpy librosa restatement) for the mel stage,
oracle/models_oracle.py (pinned bit-exact to the AST-loaded reference classes) for the step, seed-42
weights, eps from torch.Generator().manual_seed(1); reference step:
src/Convolutional_VAE.py:224-240.

Tolerances:
  * mel-dB vs the oracle: atol 0.05 dB, <= 2e-3 dB above -60 dB (fp32 vs float64 STFT, as test_features_gpu);
  * fp32 engine from the same z-scored input: mu / logvar / ELBO terms <= 1e-4 relative (north_star);
    gradients by the f64-yardstick rule of test_models_gpu.compare_step; Adam exact vs torch.optim.Adam on
    the same gradient; BatchNorm running statistics <= 1e-4;
  * bf16 engine (the bench dtype): mu / ELBO / global gradient within BF16_TOL (about 3x the measured errors:
    ELBO 5e-4) and no tensor's gradient farther than 0.6 relative L2 from the fp32 oracle's;
  * configs[2] (hybrid, 384-d lyrics) and [3] (CVAE) at the same B = 256 shapes, fp32 and bf16;
  * the whole oracle chain (oracle mel -> oracle f64 scaler -> oracle model) vs the HIP chain: the inputs
    differ by the mel tolerance, so ELBO / mu are compared at 1e-3 (fp32 engine).
"""
import json
import os

import numpy as np
import pytest
import torch

import bench
import hlmc_amd
from oracle import kmeans_oracle as KO
from oracle import mel_oracle as MO
from oracle import models_oracle as OM
from tests.test_models_gpu import _bias_feeds_bn, oracle64_with_kink_envelope, rel

pytestmark = pytest.mark.gpu
B = 256


LATENT = {"audio": 128, "hybrid": 128, "cvae": 64}


def _hip_chain(dtype, workload="audio"):
    """The bench's own chain for one BASELINE workload (bench.build_workload: seed-42 model, fused Trainer, the
    synthetic lyrics / one-hot genres) on the bench's PCM, one train step from eps ~ Generator(1)."""
    dev = torch.device("cuda", 0)
    pcm = bench.synthetic_pcm(B, bench.N_SAMPLES, seed=1000, device=dev)
    calib = hlmc_amd.extract_mel_spectrogram(pcm, fixed_time_steps=bench.FRAMES)
    scaler = hlmc_amd.StandardScaler().fit(calib.reshape(B, -1))
    stage = bench.MelStage(B, dev, scaler)
    x = stage(pcm)
    # the fused dB + z-score pass is bit-identical to hlmc_mel_db followed by hlmc_zscore_apply
    assert torch.equal(x.reshape(B, -1), scaler.transform(calib.reshape(B, -1)))
    model, trainer, text, cond = bench.build_workload(workload, dtype, B, dev, 1)
    eps = torch.randn(B, LATENT[workload], generator=torch.Generator().manual_seed(1))
    init = [p.detach().cpu().clone() for p in model.parameters()]
    sums = trainer.step(x, text, cond, eps=eps.to(dev))
    out = trainer._cache[B]["out"]
    torch.cuda.synchronize()
    return dict(pcm=pcm.cpu().numpy(), mel=calib.cpu().numpy(), x=x.detach().cpu().clone(), eps=eps,
                text=None if text is None else text.cpu(), cond=None if cond is None else cond.cpu(),
                loss=trainer.loss_tuple(sums), mu=out["mu"].cpu(), logvar=out["logvar"].cpu(),
                recon=out["recon"].cpu(), recon_text=out["recon_text"].cpu() if "recon_text" in out else None,
                grad=trainer.gflat.detach().cpu().clone(), init=init, model=model)


def _oracle_model(workload="audio"):
    torch.manual_seed(42)
    if workload == "cvae":
        return OM.ConditionalVAE(64, 768, 10, (128, 128))
    return OM.HybridVAE(128, 384, (128, 128), audio_only=workload == "audio")


def _case(workload):
    return {"kind": "cvae" if workload == "cvae" else "hybrid"}


def _ins(h, workload):
    if workload == "cvae":
        return (h["x"], h["text"], h["cond"])
    return (h["x"], h["text"])


def _oracle_step(ora, h, workload):
    ins = _ins(h, workload)
    out = ora(*ins, eps=h["eps"])
    if workload == "cvae":
        lo = OM.cvae_loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3], beta=4.0)
    else:
        lo = OM.loss_function(out[0], ins[0], out[1], ins[1], out[2], out[3])
    lo[0].backward()
    return out, lo


def test_bench_mel_stage_matches_oracle(cuda):
    h = _hip_chain("bf16")
    ref = np.stack([MO.extract_mel_spectrogram(c, fixed_time_steps=bench.FRAMES) for c in h["pcm"]])
    assert h["mel"].shape == ref.shape == (B, 128, 128)
    err = np.abs(h["mel"] - ref)
    print(f"mel-dB B={B}: max abs err {err.max():.2e} dB, above -60 dB {err[ref > -60].max():.2e} dB")
    assert err.max() < 0.05 and err[ref > -60].max() < 2e-3
    # z-score: the HIP StandardScaler (fitted on this batch) vs sklearn's float64 fit of the same mel
    mean, var, scale = KO.standard_scaler_fit(h["mel"].reshape(B, -1))
    z = KO.standard_scaler_transform(h["mel"].reshape(B, -1), mean, scale).reshape(B, 1, 128, 128)
    np.testing.assert_allclose(h["x"].numpy(), z, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("workload", ["audio", "hybrid", "cvae"])
def test_bench_train_step_fp32_matches_oracle(cuda, workload):
    """BASELINE configs[1] (audio), [2] (hybrid, 384-d lyrics) and [3] (CVAE, 10 genres) at the bench's B = 256
    shapes and GEMM plans, fp32 engine: one fused Trainer.step vs the oracle (src/Convolutional_VAE.py:224-240,
    src/Conditional_VAE.py:321-331)."""
    h = _hip_chain("fp32", workload)
    ora = _oracle_model(workload)
    for p, q in zip(ora.parameters(), h["init"]):
        assert torch.equal(p.detach(), q)
    ora64, ora64f = oracle64_with_kink_envelope(_case(workload), ora, _ins(h, workload), h["eps"], None)
    out, lo = _oracle_step(ora, h, workload)
    _check_fp32_step(workload, h, ora, ora64, ora64f, out, lo)


def _check_fp32_step(label, h, ora, ora64, ora64f, out, lo):
    """fp32 engine step vs the oracle step from the same weights / inputs / eps: outputs and ELBO terms at the 1e-4
    contract, gradients by the f64-yardstick + kink-envelope rule (BN-fed conv / linear biases absolutely), Adam exact
    vs torch.optim.Adam on the engine's own gradient, BatchNorm running statistics <= 1e-4."""
    print(f"{label} B={B} fp32: rel mu {rel(h['mu'], out[2].detach()):.2e}, rel logvar "
          f"{rel(h['logvar'], out[3].detach()):.2e}, ELBO {h['loss'][0]:.6e} vs {float(lo[0]):.6e}")
    assert rel(h["mu"], out[2].detach()) < 1e-4 and rel(h["logvar"], out[3].detach()) < 1e-4
    assert rel(h["recon"], out[0].detach()) < 1e-4
    if h["recon_text"] is not None:
        assert rel(h["recon_text"], out[1].detach()) < 1e-4
    for a, b in zip(h["loss"], lo):
        if b is not None and float(b) != 0.0:
            assert abs(a - float(b)) <= 1e-4 * abs(float(b)), (a, float(b))
    # gradients: f64 yardstick + kink envelope, BN-fed conv biases absolutely
    off = 0
    names = dict(ora.named_parameters())
    o64, o64f = dict(ora64.named_parameters()), dict(ora64f.named_parameters())
    worst = 0.0
    for name, p in ora.named_parameters():
        g = h["grad"][off:off + p.numel()].view_as(p)
        off += p.numel()
        if _bias_feeds_bn(ora, name):
            scale = float(names[name[:-4] + "weight"].grad.abs().max())
            assert float((g - p.grad).abs().max()) <= 1e-4 * scale + 1e-6, name
            continue
        g64 = o64[name].grad
        e_ref, e_ours, e_kink = rel(p.grad, g64), rel(g, g64), rel(o64f[name].grad, g64)
        worst = max(worst, e_ours)
        assert e_ours <= max(1e-3, 8 * e_ref) + 1.5 * e_kink, f"grad {name}: {e_ours:.3e} vs {e_ref:.3e} / {e_kink:.3e}"
    print(f"{label} B={B} fp32: worst per-tensor gradient error vs float64 {worst:.2e}")
    # Adam: exact torch.optim.Adam on the engine's own gradient
    ps = [q.clone().requires_grad_(True) for q in h["init"]]
    off = 0
    for p in ps:
        p.grad = h["grad"][off:off + p.numel()].view_as(p).clone()
        off += p.numel()
    torch.optim.Adam(ps, lr=1e-4).step()
    for (name, pm), p in zip(h["model"].named_parameters(), ps):
        torch.testing.assert_close(pm.detach().cpu(), p.detach(), rtol=1e-6, atol=1e-7, msg=name)
    for (n, bo), (_, bm) in zip(ora.named_buffers(), h["model"].named_buffers()):
        if bo.dtype.is_floating_point:
            assert rel(bm, bo) < 1e-4, n
        else:
            assert torch.equal(bm.cpu(), bo), n


# bf16 engine (the bench dtype) vs the fp32 oracle at B = 256: (mu, ELBO, global gradient) relative bounds, each
# about 3x the error measured on MI355X.  Inputs are identical, so the gap is the bf16 rounding of
# activations / MFMA operands (fp32 accumulation, fp32 BN statistics); a kernel that drops a K-split slab of one
# layer moves the gradient of that layer by >= 1/S and the ELBO by far more than these bounds.
# measured (MI355X, round 3): audio 1.19e-2 / 9.4e-5 / 1.38e-2, hybrid 1.03e-2 / 3.9e-6 / 1.58e-2, cvae 1.14e-2 /
# 1.42e-4 / 2.23e-2.  Per tensor the bf16 gradients of the shallow conv layers and BN parameters differ from the fp32
# ones by up to 0.36 relative L2 (B = 256 BatchNorm reductions of bf16 activations), so a dropped split-K slab is
# caught by the op-level tests at these exact shapes (test_ops_gpu *_bench_shapes_bf16, fp32-accumulation exact)
# and here only a garbage tensor (>= 0.6) is.
BF16_TOL = {"audio": (3.5e-2, 5e-4, 5e-2), "hybrid": (3.5e-2, 5e-4, 5e-2), "cvae": (3.5e-2, 5e-4, 6e-2)}
# BatchNorm running buffers after the bf16 step (worst layer): batch-mean error in batch standard deviations,
# batch-variance error relative; about 3x the MI355X measurement (round 4: audio 3.4e-3 / 5.0e-3, hybrid 6.6e-3 /
# 4.5e-3, cvae 3.4e-3 / 3.0e-3)
BF16_BN_TOL = {"audio": (1e-2, 1.5e-2), "hybrid": (2e-2, 1.5e-2), "cvae": (1e-2, 1e-2)}


# Per-tensor bf16 gradient errors vs the fp32 oracle, measured on MI355X for every workload and committed as a fixture
# (tests/golden/bf16_tensor_err.json, written by a run with HLMC_RECORD_BF16=<path>): each tensor must stay within
# 3x its own measured error + 0.01.  The shallow conv layers and BN parameters reach ~0.36 (B = 256 BatchNorm reductions
# of bf16 activations), the deep layers are at 1e-2 or below, so a wrong tile in one small layer (relative L2 ~1) is
# caught there instead of hiding under a blanket 0.6.
TENSOR_ERR_FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "bf16_tensor_err.json")


def _tensor_bounds(label):
    try:
        with open(TENSOR_ERR_FIXTURE) as f:
            meas = json.load(f)[label]
    except (OSError, KeyError):
        return None
    return {n: 3.0 * e + 0.01 for n, e in meas.items()}


def _record_tensor_errors(label, per):
    path = os.environ.get("HLMC_RECORD_BF16")
    if not path:
        return
    d = {}
    if os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
    d[label] = {n: round(e, 6) for n, e in per.items()}
    with open(path, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


@pytest.mark.parametrize("workload", ["audio", "hybrid", "cvae"])
def test_bench_train_step_bf16_tracks_oracle(cuda, workload):
    h = _hip_chain("bf16", workload)
    ora = _oracle_model(workload)
    out, lo = _oracle_step(ora, h, workload)
    _check_bf16_step(workload, h, ora, out, lo, BF16_TOL[workload], BF16_BN_TOL[workload])


def _check_bf16_step(label, h, ora, out, lo, tol, bn_tol):
    go = torch.cat([p.grad.reshape(-1) for p in ora.parameters()])
    e_mu, e_elbo, e_g = rel(h["mu"], out[2].detach()), abs(h["loss"][0] - float(lo[0])) / abs(float(lo[0])), rel(h["grad"], go)
    # per-tensor gradient errors (BN-fed conv biases excluded: zero true gradient)
    per = {}
    off = 0
    for name, p in ora.named_parameters():
        g = h["grad"][off:off + p.numel()].view_as(p)
        off += p.numel()
        if not _bias_feeds_bn(ora, name):
            per[name] = rel(g, p.grad)
    _record_tensor_errors(label, per)
    worst = sorted(per.items(), key=lambda kv: -kv[1])[:4]
    print(f"{label} B={B} bf16: rel mu {e_mu:.2e}, rel ELBO {e_elbo:.2e}, global grad rel L2 {e_g:.2e}; "
          f"worst tensors {[(n, round(e, 4)) for n, e in worst]}")
    t_mu, t_elbo, t_g = tol
    assert e_mu < t_mu and e_elbo < t_elbo and e_g < t_g
    # every tensor within 3x its measured error (+0.01); no tensor's gradient garbage in any case
    bounds = _tensor_bounds(label)
    bad = {n: e for n, e in per.items() if e > 0.6 or (bounds is not None and e > bounds[n])}
    assert not bad, {n: (e, None if bounds is None else bounds[n]) for n, e in bad.items()}
    # every BatchNorm running buffer after the step vs the oracle's (src/Convolutional_VAE.py:80-100, 124-139):
    # from the zero / one initialisation, running_mean = 0.1 * batch mean and running_var = 0.9 + 0.1 * unbiased
    # batch variance, so the error is reported in the batch statistics' own units -- the mean error in batch standard
    # deviations, the variance error relative to the batch variance.  These come from the halo kernels' multi-tile
    # epilogue statistics, the BnInput staging, the split-K reduce's statistics and col_moments.
    worst_m, worst_v = (0.0, ""), (0.0, "")
    ora_b = dict(ora.named_buffers())
    for n, bm in h["model"].named_buffers():
        bo, bm = ora_b[n], bm.detach().cpu()
        if n.endswith("num_batches_tracked"):
            assert torch.equal(bm, bo), n
            continue
        if n.endswith("running_mean"):
            var = (ora_b[n[:-4] + "var"].double() - 0.9) / 0.1
            e = float(((bm.double() - bo.double()).abs() / (0.1 * var.clamp_min(1e-12).sqrt())).max())
            worst_m = max(worst_m, (e, n))
        else:
            var = (bo.double() - 0.9) / 0.1
            e = float(((bm.double() - bo.double()).abs() / (0.1 * var.clamp_min(1e-12))).max())
            worst_v = max(worst_v, (e, n))
    print(f"{label} B={B} bf16 BN buffers: worst mean error {worst_m[0]:.2e} sd ({worst_m[1]}), worst variance "
          f"error {worst_v[0]:.2e} rel ({worst_v[1]})")
    t_m, t_v = bn_tol
    assert worst_m[0] < t_m and worst_v[0] < t_v, (worst_m, worst_v)


# ---- BASELINE configs[4]'s training shape: HybridVAE 128 x 1024 with 768-d lyrics at B = 256, the model, trainer and
# GEMM plans pipeline.run_pipeline times in bench.py's config[4] extra (split-K factors, halo / sub-pixel tiles chosen
# by M = 256 * H * W at 8x the 128 x 128 pixel count).  Input: the pipeline's own chain on 256 synthetic 30 s clips
# (HIP mel-dB with 1024 kept frames -> per-pixel StandardScaler), lyrics ~ N(0, 1/768), eps ~ Generator(1).  The oracle
# step (fp32 + the float64 yardstick and its kink envelope) runs once for both dtypes.  Reference:
# src/Convolutional_VAE.py:207-240 at its native 128 x 1024 (src/1_preprocessing_advanced.py:34, fixed_time_steps=1024).
C4_TOL = (3.5e-2, 5e-4, 5e-2)
C4_BN_TOL = (2e-2, 1.5e-2)


@pytest.fixture(scope="module")
def config4_case(cuda):
    from hlmc_amd import pipeline as P
    dev = torch.device("cuda", 0)
    pcm = P.synthetic_clips(B, P.CLIP_SAMPLES, seed=4242, device=dev)
    mel = hlmc_amd.extract_mel_spectrogram(pcm, fixed_time_steps=P.KEEP_FRAMES)
    del pcm
    x = hlmc_amd.StandardScaler().fit(mel.reshape(B, -1)).transform(mel.reshape(B, -1)).reshape(B, 1, 128, 1024)
    g = torch.Generator().manual_seed(17)
    text = torch.randn(B, 768, generator=g) / 768 ** 0.5
    eps = torch.randn(B, 128, generator=torch.Generator().manual_seed(1))
    x = x.cpu()
    torch.manual_seed(42)
    ora = OM.HybridVAE(128, 768, (128, 1024))
    ora64, ora64f = oracle64_with_kink_envelope({"kind": "hybrid"}, ora, [x, text], eps, None)
    out = ora(x, text, eps=eps)
    lo = OM.loss_function(out[0], x, out[1], text, out[2], out[3])
    lo[0].backward()
    return dict(x=x, text=text, eps=eps, ora=ora, ora64=ora64, ora64f=ora64f, out=out, lo=lo)


def _config4_engine(c, dtype):
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = hlmc_amd.HybridVAE(128, 768, (128, 1024), compute_dtype=dtype).to(dev)
    trainer = hlmc_amd.Trainer(model, lr=1e-4)
    init = [p.detach().cpu().clone() for p in model.parameters()]
    for p, q in zip(c["ora"].parameters(), init):
        assert torch.equal(p.detach(), q)
    sums = trainer.step(c["x"].to(dev), c["text"].to(dev), eps=c["eps"].to(dev))
    out = trainer._cache[B]["out"]
    torch.cuda.synchronize()
    h = dict(loss=trainer.loss_tuple(sums), mu=out["mu"].cpu(), logvar=out["logvar"].cpu(), recon=out["recon"].cpu(),
             recon_text=out["recon_text"].cpu(), grad=trainer.gflat.detach().cpu().clone(), init=init, model=model)
    trainer.release()
    return h


def test_config4_train_step_fp32_matches_oracle(config4_case):
    c = config4_case
    h = _config4_engine(c, "fp32")
    _check_fp32_step("config4 128x1024 td768", h, c["ora"], c["ora64"], c["ora64f"], c["out"], c["lo"])


def test_config4_train_step_bf16_tracks_oracle(config4_case):
    c = config4_case
    h = _config4_engine(c, "bf16")
    _check_bf16_step("config4", h, c["ora"], c["out"], c["lo"], C4_TOL, C4_BN_TOL)


def test_bench_whole_oracle_chain(cuda):
    """PCM -> oracle mel -> oracle (sklearn-f64) z-score -> oracle model vs the HIP chain end to end (fp32)."""
    h = _hip_chain("fp32")
    mel = np.stack([MO.extract_mel_spectrogram(c, fixed_time_steps=bench.FRAMES) for c in h["pcm"]])
    mean, var, scale = KO.standard_scaler_fit(mel.reshape(B, -1))
    x = torch.from_numpy(KO.standard_scaler_transform(mel.reshape(B, -1), mean, scale).reshape(B, 1, 128, 128))
    print(f"input (z-score) max abs diff HIP vs oracle chain: {float((x - h['x']).abs().max()):.2e}")
    ora = _oracle_model()
    out = ora(x, None, eps=h["eps"])
    lo = OM.loss_function(out[0], x, None, None, out[2], out[3])
    e_mu, e_elbo = rel(h["mu"], out[2].detach()), abs(h["loss"][0] - float(lo[0])) / abs(float(lo[0]))
    print(f"whole chain B={B}: rel mu {e_mu:.2e}, rel ELBO {e_elbo:.2e}")
    assert e_mu < 1e-3 and e_elbo < 1e-3
