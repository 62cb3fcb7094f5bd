"""BASELINE config[4] end to end on the GPU: raw 30 s clips -> HIP STFT / mel-dB (1024 kept frames) -> per-pixel
StandardScaler -> ConvVAE (HybridVAE 128 x 1024 with lyrics) training -> eval-mode latent extraction -> KMeans.

The reference runs this as three scripts with files in between:
  * src/1_preprocessing_advanced.py:286-421 — joblib pool over clips: load + pad to 30 s (:79-94),
    extract_mel_spectrogram(fixed_time_steps=1024) (:97-114), np.array gather, StandardScaler over
    [N, 128 * 1024] pixels (:376-382), np.save processed_data2/mel_spectrograms_normalized.npy;
  * src/Convolutional_VAE.py:217-271 — HybridVAE(128) + Adam(1e-4), bs 32, train loop (the early stopping
    and validation split are host policy, not the hot path);
  * src/Convolutional_VAE.py:286-303 — model.eval(); encode -> mu per batch -> hybrid_latent_features.npy;
  * src/Convolutional_VAE.py:317-319 / 379-380 — KMeans(n_clusters=k, random_state=42, n_init=10).fit_predict.
Here every stage stays resident in HBM (100 000 clips of mel-dB = 52 GB f32 of the 288 GB), nothing goes
through files or host memory, and each stage is timed.  Decoding WAV files is out of scope: the
clips are synthetic PCM generated on the device in batches (SURVEY §8d recipe), 30 s at 22.05 kHz.
"""
from __future__ import annotations

import time

import torch

from . import _lib as L
from .cluster import KMeans
from .features import StandardScaler, extract_mel_spectrogram
from .models import HybridVAE
from .train import Trainer

SR = 22050
CLIP_SAMPLES = 30 * SR      # 661 500 (load_audio_file pads / trims to 30 s)
KEEP_FRAMES = 1024          # fixed_time_steps (src/1_preprocessing_advanced.py:34)


def synthetic_clips(batch, n_samples, seed, device):
    """Seeded sum of 8 sinusoids (50-8000 Hz, amplitude U(0.02, 0.1)) + N(0, 0.01^2) noise per clip, on the
    device, clipped to [-1, 1]."""
    g = torch.Generator(device=device).manual_seed(seed)
    t = torch.arange(n_samples, device=device, dtype=torch.float32) / SR
    f = torch.rand(batch, 8, device=device, generator=g) * 7950 + 50
    a = torch.rand(batch, 8, device=device, generator=g) * 0.08 + 0.02
    ph = torch.rand(batch, 8, device=device, generator=g) * 6.2831853
    y = 0.01 * torch.randn(batch, n_samples, device=device, generator=g)
    for j in range(8):
        y += a[:, j:j + 1] * torch.sin(6.2831853 * f[:, j:j + 1] * t + ph[:, j:j + 1])
    return y.clamp_(-1, 1)


def _sync():
    torch.cuda.synchronize()
    return time.perf_counter()


def shard_bounds(n_clips, world):
    """Contiguous clip shards [lo, hi) per rank: sizes n // world, the first n % world ranks one more."""
    q, r = divmod(n_clips, world)
    out, lo = [], 0
    for k in range(world):
        hi = lo + q + (1 if k < r else 0)
        out.append((lo, hi))
        lo = hi
    return out


def local_batches(shard_sizes, rank, batch):
    """Per-step slices [a, b) of rank `rank`'s epoch order such that every rank takes the SAME number of steps
    (each step all-reduces gradients): steps = ceil(smallest shard / batch); a larger shard (by one clip) folds its
    extra clips into its last batch.  A last batch under 2 rows on any rank (train-mode BatchNorm needs >= 2) is
    merged into the step before it on every rank."""
    smin = min(shard_sizes)
    steps = max(1, -(-smin // batch))
    if steps > 1 and any(s - (steps - 1) * batch < 2 for s in shard_sizes):
        steps -= 1
    n = shard_sizes[rank]
    return [(k * batch, n if k == steps - 1 else (k + 1) * batch) for k in range(steps)]


def _all_gather_rows(t, group, bounds):
    """[hi - lo, ...] per rank -> [n, ...] in clip order (every rank).  gloo gathers host copies."""
    import torch.distributed as dist
    world = len(bounds)
    width = max(hi - lo for lo, hi in bounds)
    gloo = dist.get_backend(group) == "gloo"
    src = t if not gloo else t.cpu()
    pad = torch.zeros((width,) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
    pad[:t.shape[0]] = src
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:hi - lo] for p, (lo, hi) in zip(parts, bounds)]).to(t.device)


def run_pipeline(n_clips, batch=256, epochs=1, text_dim=768, latent_dim=128, compute_dtype="bf16", k=10,
                 n_init=10, seed=0, pcm_fn=None, lyrics=None, eps_fn=None, order_fn=None, keep_outputs=False,
                 device=None, process_group=None, grad_dtype=torch.float32):
    """Run config[4] on `n_clips` clips; returns a dict of per-stage seconds and results.

    pcm_fn(i, b) -> [b, 661500] float32 device PCM of clips i..i+b (default: synthetic_clips seeded per batch);
    lyrics: [n_clips, text_dim] lyric embeddings (default: seeded N(0, 1/text_dim), on the device);
    eps_fn(step, b) -> reparameterisation noise (default None: the engine draws it on the device from its Philox
    stream, as the reference's randn_like; under process_group each rank's stream is keyed by its rank, see
    Trainer);
    order_fn(epoch) -> clip order of that epoch over the rank's shard (local indices; default a seeded
    torch.randperm: DataLoader(shuffle=True)).

    process_group (data parallel, one process per GPU): the clips are cut into contiguous shards, one per rank
    (shard_bounds).  Each rank computes the mel-dB of its own shard only; the per-pixel StandardScaler all-reduces
    its f64 pass sums (every rank gets the global statistics, as the reference's whole-dataset fit,
    src/1_preprocessing_advanced.py:376-382); training is Trainer(distributed=True) — every step each rank takes
    `batch` clips of its shard (local_batches), gradients are SUM all-reduced (RCCL over xGMI) and rank 0's
    BatchNorm running statistics broadcast (DDP semantics); each rank encodes its shard with the (identical)
    trained model, the latents are all-gathered in clip order and KMeans(process_group) shards the n_init
    restarts, so every rank returns the same labels."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    world, rank = 1, 0
    if process_group is not None:
        import torch.distributed as dist
        world, rank = dist.get_world_size(process_group), dist.get_rank(process_group)
    bounds = shard_bounds(n_clips, world)
    lo, hi = bounds[rank]
    n_local = hi - lo
    if pcm_fn is None:
        def pcm_fn(i, b):
            return synthetic_clips(b, CLIP_SAMPLES, seed * 1000003 + i, dev)
    out = {"n_clips": n_clips, "batch": batch, "epochs": epochs, "compute_dtype": compute_dtype, "world": world,
           "shard": (lo, hi), "stages_s": {}}
    st = out["stages_s"]

    # ---- 1. mel-dB of this rank's clips (1292 frames, ref = max over all of them, 1024 kept), resident in HBM
    t0 = _sync()
    mel = torch.empty(n_local, 128, KEEP_FRAMES, device=dev)
    evs = []   # per batch: (before the clip source, after it = before the mel kernels, after them)
    for i in range(0, n_local, batch):
        b = min(batch, n_local - i)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        pcm = pcm_fn(lo + i, b)
        e[1].record()
        mel[i:i + b] = extract_mel_spectrogram(pcm, fixed_time_steps=KEEP_FRAMES)
        e[2].record()
        evs.append(e)
    t1 = _sync()
    st["pcm_and_mel"] = t1 - t0
    st["mel_only"] = sum(e[1].elapsed_time(e[2]) for e in evs) / 1e3     # GPU time of the STFT/mel/dB kernels
    st["pcm_source"] = sum(e[0].elapsed_time(e[1]) for e in evs) / 1e3   # synthetic clip generation (torch)

    # ---- 2. per-pixel StandardScaler over [N, 131072] (float64 accumulators; all-reduced over the shards)
    scaler = StandardScaler(process_group=process_group).fit(mel.view(n_local, -1))
    t2 = _sync()
    st["scaler_fit"] = t2 - t1

    # ---- 3. HybridVAE(128 x 1024) training, z-score applied per batch into the input buffer
    if lyrics is None:
        g = torch.Generator(device=dev).manual_seed(seed + 17)
        lyrics = torch.randn(n_clips, text_dim, device=dev, generator=g) / text_dim ** 0.5
    lyrics = lyrics.to(dev).float()[lo:hi].contiguous()
    torch.manual_seed(42)
    model = HybridVAE(latent_dim, text_dim, (128, KEEP_FRAMES), compute_dtype=compute_dtype).to(dev)
    trainer = Trainer(model, lr=1e-4, process_group=process_group, grad_dtype=grad_dtype)
    slices = local_batches([h - l for l, h in bounds], rank, batch)
    bmax = max(b - a for a, b in slices)
    xb = torch.empty(bmax, 1, 128, KEEP_FRAMES, device=dev)
    tb = torch.empty(bmax, text_dim, device=dev)

    def zscore_into(idx):
        b = idx.numel()
        rows = mel.index_select(0, idx).view(b, -1)
        L.check(L.lib().hlmc_zscore_apply(L.stream(), rows.data_ptr(), b, rows.shape[1], scaler.mean_d.data_ptr(),
                                          scaler.scale_d.data_ptr(), L.HLMC_F32, xb.data_ptr()), "hlmc_zscore_apply")
        tb[:b].copy_(lyrics.index_select(0, idx))
        return xb[:b], tb[:b]

    gperm = torch.Generator(device=dev).manual_seed(seed + 29 + 7919 * rank)
    step, sums = 0, None
    for ep in range(epochs):
        order = (order_fn(ep).to(dev) if order_fn is not None
                 else torch.randperm(n_local, device=dev, generator=gperm))   # DataLoader(shuffle=True)
        for a, b in slices:
            idx = order[a:b]
            x, t = zscore_into(idx)
            eps = eps_fn(step, idx.numel()) if eps_fn is not None else None
            sums = trainer.step(x, t, eps=eps)
            step += 1
    t3 = _sync()
    st["train"] = t3 - t2
    out["train_steps"] = step
    out["final_loss"] = trainer.loss_tuple(sums)[0] if sums is not None else None

    # ---- 4. eval-mode latent extraction (mu of encode) of this rank's clips, gathered in clip order
    trainer.release()
    model.eval()
    latents = torch.empty(n_local, latent_dim, device=dev)
    ar = torch.arange(n_local, device=dev)
    with torch.no_grad():
        for i in range(0, n_local, batch):
            idx = ar[i:i + batch]
            x, t = zscore_into(idx)
            latents[i:i + idx.numel()] = model.encode(x, t)[0]
    if world > 1:
        latents = _all_gather_rows(latents, process_group, bounds)
    t4 = _sync()
    st["encode"] = t4 - t3

    # ---- 5. KMeans(k, random_state=42, n_init) on the latents (sklearn semantics, bit-exact labels)
    km = KMeans(n_clusters=k, random_state=42, n_init=n_init, process_group=process_group).fit(latents)
    t5 = _sync()
    st["kmeans"] = t5 - t4
    st["total"] = t5 - t0
    out["labels"] = km.labels_
    out["inertia"] = km.inertia_
    out["kmeans_n_iter"] = km.n_iter_
    out["clips_per_s_end_to_end"] = n_clips / st["total"]
    if keep_outputs:
        out.update(mel=mel, scaler=scaler, latents=latents, model=model)
    else:
        del mel
        torch.cuda.empty_cache()
    return out
