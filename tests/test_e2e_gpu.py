"""BASELINE config[4] end to end (hlmc_amd.pipeline.run_pipeline) at small N against the oracle chain:
30 s PCM -> mel-dB (1024 kept frames; dB reference over all 1292) -> per-pixel StandardScaler -> HybridVAE
(128 x 1024, lyrics 768) train step -> eval-mode latents -> KMeans(k, random_state=42, n_init=10).
Reference chain: src/1_preprocessing_advanced.py:286-421 then src/Convolutional_VAE.py:217-327.

Checks (fp32 engine):
  * mel-dB vs oracle/mel_oracle.py: atol 0.05 dB, <= 2e-3 dB above -60 dB (test_features_gpu's contract);
  * scaler statistics vs the oracle's sklearn-f64 fit of the same mel: rtol 1e-9;
  * the model path from the same z-scored input and the same eps: after the single Adam step the eval-mode
    latents agree to 2e-3 relative L2 (Adam turns rounding noise in the zero true gradients of the
    BatchNorm-fed conv biases into +-lr moves; one step measured ~2e-4 fp32 vs fp64);
  * K-Means on the engine's latents: labels bit-identical to the oracle's sklearn restatement on the same latents;
    against the whole oracle chain (its own latents) ARI >= 0.99 (north_star: ARI delta <= 0.01).
"""
import numpy as np
import pytest
import torch

import hlmc_amd
from oracle import kmeans_oracle as KO
from oracle import mel_oracle as MO
from oracle import models_oracle as OM

pytestmark = pytest.mark.gpu
N, K = 16, 3


def test_config4_pipeline_matches_oracle_chain(cuda):
    pcm = MO.synthetic_pcm(N, hlmc_amd.pipeline.CLIP_SAMPLES, seed=44)
    g = torch.Generator().manual_seed(9)
    lyrics = torch.randn(N, 768, generator=g) / 768 ** 0.5
    eps = torch.randn(N, 128, generator=g)
    pcm_d = torch.from_numpy(pcm).cuda()
    r = hlmc_amd.pipeline.run_pipeline(N, batch=N, epochs=1, compute_dtype="fp32", k=K, n_init=10,
                                       pcm_fn=lambda i, b: pcm_d[i:i + b], lyrics=lyrics.cuda(),
                                       eps_fn=lambda step, b: eps[:b].cuda(), order_fn=lambda ep: torch.arange(N),
                                       keep_outputs=True)
    print("stages (s):", {k: round(v, 3) for k, v in r["stages_s"].items()})
    # ---- mel
    mel = r["mel"].cpu().numpy()
    ref = np.stack([MO.extract_mel_spectrogram(c, fixed_time_steps=1024) for c in pcm])
    err = np.abs(mel - ref)
    print(f"mel-dB 30 s x {N}: max err {err.max():.2e} dB, above -60 dB {err[ref > -60].max():.2e}")
    assert err.max() < 0.05 and err[ref > -60].max() < 2e-3
    # ---- scaler on the engine's mel
    mean, var, scale = KO.standard_scaler_fit(mel.reshape(N, -1))
    np.testing.assert_allclose(r["scaler"].mean_, mean, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(r["scaler"].scale_, scale, rtol=1e-9)
    x = torch.from_numpy(KO.standard_scaler_transform(mel.reshape(N, -1), mean, scale).reshape(N, 1, 128, 1024))
    # ---- oracle model: one Adam step on the same batch / eps, then eval-mode latents
    torch.manual_seed(42)
    ora = OM.HybridVAE(128, 768, (128, 1024))
    opt = torch.optim.Adam(ora.parameters(), lr=1e-4)
    out = ora(x, lyrics, eps=eps)
    OM.loss_function(out[0], x, out[1], lyrics, out[2], out[3])[0].backward()
    opt.step()
    ora.eval()
    with torch.no_grad():
        mu_o = ora.encode(x, lyrics)[0]
    mu_h = r["latents"].cpu()
    rel = float((mu_h - mu_o).norm() / mu_o.norm())
    print(f"eval latents after one step: rel L2 {rel:.2e}")
    assert rel < 2e-3
    # the engine isolated from Adam amplification: the pipeline's model holding the oracle's post-step state
    # (weights + running statistics) encodes the same z-scored 128 x 1024 input to the 1e-4 contract
    eng = r["model"]
    eng.load_state_dict(ora.state_dict())
    eng.eval()
    with torch.no_grad():
        mu_e = eng.encode(x.cuda(), lyrics.cuda())[0].cpu()
    rel_e = float((mu_e - mu_o).norm() / mu_o.norm())
    print(f"engine eval latents from the oracle's state: rel L2 {rel_e:.2e}")
    assert rel_e < 1e-4
    # ---- K-Means: engine == sklearn restatement on the engine's latents; ARI vs the whole oracle chain
    lab_o = KO.KMeans(K, random_state=42, n_init=10).fit(mu_h.numpy()).labels_
    np.testing.assert_array_equal(r["labels"], lab_o)
    lab_chain = KO.KMeans(K, random_state=42, n_init=10).fit(mu_o.numpy()).labels_
    from sklearn.metrics import adjusted_rand_score
    ari = adjusted_rand_score(lab_chain, r["labels"])
    print(f"ARI(engine chain, oracle chain) = {ari:.4f}")
    assert ari >= 0.99


# ---------------------------------------------------------------------------------------------- data parallel
WORLD2, N2, B2, K2 = 2, 16, 4, 3


def _dp_inputs():
    pcm = MO.synthetic_pcm(N2, hlmc_amd.pipeline.CLIP_SAMPLES, seed=45)
    g = torch.Generator().manual_seed(19)
    lyrics = torch.randn(N2, 768, generator=g) / 768 ** 0.5
    eps = torch.randn(64, B2 + 1, 128, generator=g)   # per (rank, step) noise, indexed below
    return pcm, lyrics, eps


def _dp_worker(rank, port, outdir):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD2)
    torch.cuda.set_device(0)
    pcm, lyrics, eps = _dp_inputs()
    pcm_d = torch.from_numpy(pcm).cuda()
    r = hlmc_amd.pipeline.run_pipeline(N2, batch=B2, epochs=1, compute_dtype="fp32", k=K2, n_init=4,
                                       pcm_fn=lambda i, b: pcm_d[i:i + b], lyrics=lyrics.cuda(),
                                       eps_fn=lambda step, b: eps[8 * rank + step, :b].cuda(),
                                       order_fn=lambda ep: torch.arange(N2 // WORLD2), keep_outputs=True,
                                       process_group=dist.group.WORLD)
    torch.save({"labels": torch.from_numpy(r["labels"].astype("int64")), "latents": r["latents"].cpu(),
                "mean": torch.from_numpy(r["scaler"].mean_), "scale": torch.from_numpy(r["scaler"].scale_),
                "mel": r["mel"].cpu(), "shard": torch.tensor(r["shard"]), "steps": r["train_steps"],
                "state": {k: v.detach().cpu() for k, v in r["model"].state_dict().items()}},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_config4_pipeline_two_ranks(cuda):
    """run_pipeline(process_group=...) with 2 ranks (gloo, both on cuda:0; a 1-GPU box cannot host two RCCL
    ranks): each rank computes the mel of its own 8-clip shard, the scaler statistics are all-reduced, training is
    the data-parallel Trainer (SUM all-reduce + BN buffer broadcast, oracle-checked in test_dp_gpu.py), latents are
    gathered in clip order and KMeans shards its restarts.  Checks: the ranks agree bit for bit (weights, BN
    statistics, latents, labels); the shard mels equal the single-process mel of the same clips bit for bit; the
    all-reduced scaler equals the single-process fit on all 16 clips (f64 sums in a different order: 1e-12);
    the gathered latents equal the single-process eval encode of all clips with the trained state; the labels
    equal the single-process KMeans of those latents bit for bit (restarts sharded, one RandomState stream)."""
    import os
    import tempfile

    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as outdir:
        port = 30300 + (os.getpid() % 500)
        mp.spawn(_dp_worker, args=(port, outdir), nprocs=WORLD2, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(WORLD2)]
    r0, r1 = res
    assert r0["steps"] == r1["steps"] == 2
    for key in ("labels", "latents", "mean", "scale"):
        assert torch.equal(r0[key], r1[key]), key
    for k in r0["state"]:
        assert torch.equal(r0["state"][k], r1["state"][k]), f"ranks diverged at {k}"
    # single process, same clips
    pcm, lyrics, _ = _dp_inputs()
    mel = hlmc_amd.extract_mel_spectrogram(torch.from_numpy(pcm).cuda(), fixed_time_steps=1024)
    for r in res:
        lo, hi = r["shard"].tolist()
        assert torch.equal(r["mel"], mel[lo:hi].cpu())
    sc = hlmc_amd.StandardScaler().fit(mel.view(N2, -1))
    np.testing.assert_allclose(r0["mean"].numpy(), sc.mean_, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(r0["scale"].numpy(), sc.scale_, rtol=1e-12)
    torch.manual_seed(42)
    model = hlmc_amd.HybridVAE(128, 768, (128, 1024)).cuda()
    model.load_state_dict(r0["state"])
    model.eval()
    x = sc.transform(mel.view(N2, -1)).view(N2, 1, 128, 1024)
    with torch.no_grad():
        mu = torch.cat([model.encode(x[i:i + B2], lyrics[i:i + B2].cuda())[0] for i in range(0, N2, B2)]).cpu()
    e = float((r0["latents"] - mu).norm() / mu.norm())
    print(f"gathered latents vs single-process encode: rel L2 {e:.2e}")
    assert e < 1e-6
    km = hlmc_amd.KMeans(K2, random_state=42, n_init=4).fit(r0["latents"].cuda())
    np.testing.assert_array_equal(r0["labels"].numpy(), km.labels_)
