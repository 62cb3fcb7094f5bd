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
    # ---- K-Means: engine == sklearn restatement on the engine's latents; ARI vs the whole oracle chain
    lab_o = KO.KMeans(K, random_state=42, n_init=10).fit(mu_h.numpy()).labels_
    np.testing.assert_array_equal(r["labels"], lab_o)
    lab_chain = KO.KMeans(K, random_state=42, n_init=10).fit(mu_o.numpy()).labels_
    from sklearn.metrics import adjusted_rand_score
    ari = adjusted_rand_score(lab_chain, r["labels"])
    print(f"ARI(engine chain, oracle chain) = {ari:.4f}")
    assert ari >= 0.99
