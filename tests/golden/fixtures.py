"""Fixture case definitions shared by make_golden.py (generator) and the tests (consumers).

Inputs are regenerated from seeds on every machine (torch CPU / numpy generators are deterministic),
so the .npz files hold only expected outputs and compact summaries.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch

MODEL_CASES = [
    # BASELINE config[1] (the benchmarked model): the reference HybridVAE with its text branch, fusion slice and
    # text loss term removed by an AST rewrite (make_golden._AudioOnlyRewrite); inputs (audio, None)
    dict(name="audio_128x128", kind="hybrid", hw=(128, 128), B=4, audio_only=True,
         ctor=dict(latent_dim=128, text_dim=768)),
    dict(name="hybrid_128x128_td768", kind="hybrid", hw=(128, 128), B=4, ctor=dict(latent_dim=128, text_dim=768)),
    dict(name="hybrid_128x128_td384", kind="hybrid", hw=(128, 128), B=4, ctor=dict(latent_dim=128, text_dim=384)),
    dict(name="hybrid_128x1024_td768", kind="hybrid", hw=(128, 1024), B=2, ctor=dict(latent_dim=128, text_dim=768)),
    dict(name="cvae_128x128", kind="cvae", hw=(128, 128), B=4, ctor=dict(latent_dim=64, text_dim=768, num_classes=10)),
    dict(name="cvae_128x1024", kind="cvae", hw=(128, 1024), B=2, ctor=dict(latent_dim=64, text_dim=768, num_classes=10)),
    dict(name="simple_370", kind="simple", B=32, ctor=dict(input_dim=370, hidden_dims=[128, 64, 32], latent_dim=32)),
]

# (N, D, blob centres, k, n_init)
KMEANS_CASES = [
    (1336, 128, 10, 10, 10),
    (1336, 128, 10, 2, 10),
    (1336, 128, 10, 14, 10),
    (1336, 64, 10, 10, 10),
    (4096, 128, 8, 10, 10),
    (4096, 64, 12, 14, 10),
    (1336, 64, 10, 10, 1),
]

# Overlapping-cluster cases (labels decided by float32 rounding at near-ties): (N, D, true clusters, centre std,
# k, n_init).  Points are N(0, 1) around centres ~ N(0, spread^2): spread 1 = "blob spread = centre spread";
# spread 0.15 = heavy overlap (every point nearly equidistant from several centres).
KMEANS_OVERLAP_CASES = [
    (1336, 128, 10, 1.0, 10, 10),
    (1336, 128, 10, 0.15, 10, 10),
    (4096, 64, 10, 0.15, 14, 10),
    (1336, 64, 6, 0.15, 2, 10),
    (1000, 128, 8, 0.15, 3, 10),
    (999, 128, 8, 0.15, 5, 1),
]
# config[4] clustering scale: N = 100 000 latents-like rows (D = 128), k = 10, n_init = 10 (labels stored int16)
KMEANS_BIG_CASE = (100000, 128, 10, 0.3, 10, 10)
# eval-mode latents of the oracle HybridVAE (128x128, text 768) on 1336 synthetic clips; k = 2..14 sweep
# (src/Convolutional_VAE.py:311-327); the latents themselves are stored in the fixture
LATENT_N, LATENT_KS = 1336, list(range(2, 15))

N_SAMPLES = 16


def oracle_ctor(case):
    ctor = dict(case["ctor"])
    if case["kind"] in ("hybrid", "cvae"):
        ctor["input_hw"] = tuple(case["hw"])
    if case.get("audio_only"):
        ctor["audio_only"] = True
    return ctor


def case_by_name(name):
    return next(c for c in MODEL_CASES if c["name"] == name)


def inputs_fn(case):
    """step -> (inputs tuple, eps) on CPU float32, seeded per (case, step)."""
    B = case["B"]
    kind = case["kind"]

    def fn(step):
        g = torch.Generator().manual_seed(1000 + 17 * step)
        if kind == "simple":
            x = torch.randn(B, case["ctor"]["input_dim"], generator=g)
            eps = torch.randn(B, case["ctor"]["latent_dim"], generator=g)
            return (x,), eps
        H, W = case["hw"]
        td = case["ctor"]["text_dim"]
        audio = torch.randn(B, 1, H, W, generator=g)
        text = torch.randn(B, td, generator=g) / td ** 0.5
        eps = torch.randn(B, case["ctor"]["latent_dim"], generator=g)
        if case.get("audio_only"):
            return (audio, None), eps
        if kind == "cvae":
            C = case["ctor"]["num_classes"]
            cls = torch.randint(0, C, (B,), generator=g)
            cond = torch.nn.functional.one_hot(cls, C).float()
            return (audio, text, cond), eps
        return (audio, text), eps

    return fn


def loss_args(kind, outs, ins):
    if kind == "simple":
        recon, mu, logvar, _ = outs
        return recon, ins[0], mu, logvar
    ra, rt, mu, logvar = outs
    return ra, ins[0], rt, ins[1], mu, logvar


def encode_args(kind, ins):
    return ins


def _sample_idx(name, numel):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    return rng.integers(0, numel, size=min(N_SAMPLES, numel))


def _summ(name, t):
    a = t.detach().reshape(-1).double().numpy()
    idx = _sample_idx(name, a.size)
    row = np.zeros(2 + N_SAMPLES)
    row[0], row[1] = a.sum(), (a * a).sum()
    row[2:2 + idx.size] = a[idx]
    return row


def grad_summary(model):
    return np.stack([_summ(n, p.grad) for n, p in model.named_parameters()])


def param_summary(model):
    return np.stack([_summ(n, p) for n, p in model.named_parameters()])


def buffer_summary(model):
    rows = [_summ(n, b) for n, b in model.named_buffers() if b.dtype.is_floating_point]
    return np.stack(rows) if rows else np.zeros((0, 2 + N_SAMPLES))


def blobs(n, d, k, seed):
    """Latent-like float32 data: k Gaussian blobs (std 1) around N(0, 3^2) centres."""
    rng = np.random.default_rng(seed)
    c = rng.normal(0, 3.0, (k, d))
    lab = rng.integers(0, k, n)
    return (c[lab] + rng.normal(0, 1.0, (n, d))).astype(np.float32)


def overlap_blobs(n, d, k, spread, seed):
    """Overlapping clusters: N(0, 1) points around k centres drawn from N(0, spread^2), float32."""
    rng = np.random.default_rng(seed)
    c = rng.normal(0, spread, (k, d))
    lab = rng.integers(0, k, n)
    return (c[lab] + rng.normal(0, 1.0, (n, d))).astype(np.float32)


def overlap_fixture_name(case):
    n, d, true_k, spread, k, n_init = case
    return f"kmeans_overlap_n{n}_d{d}_s{int(round(spread * 100))}_k{k}_i{n_init}.npz"


def overlap_seed(case):
    n, d, true_k, spread, k, n_init = case
    return 7 * n + 3 * d + 11 * true_k + int(round(spread * 100))


def blob_labels(n, d, k, seed):
    """The blob membership of blobs(n, d, k, seed) (same generator sequence): ground-truth labels."""
    rng = np.random.default_rng(seed)
    rng.normal(0, 3.0, (k, d))
    return rng.integers(0, k, n)


# cluster-quality metric cases: the KMEANS_CASES entries whose sklearn labels are scored
METRICS_CASES = [KMEANS_CASES[0], KMEANS_CASES[1], KMEANS_CASES[3], KMEANS_CASES[5]]


def kmeans_fixture_name(case):
    n, d, centers, k, n_init = case
    return f"kmeans_n{n}_d{d}_k{k}_i{n_init}.npz"


def metrics_fixture_name(case):
    n, d, centers, k, n_init = case
    return f"metrics_n{n}_d{d}_k{k}.npz"

