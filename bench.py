"""Benchmark: clips/sec of the mel + VAE train step (BASELINE.json metric), 128-mel x 128-frame, bs=256/GPU.

One step = PCM [256, 65024] (synthetic, resident in HBM) -> HIP STFT + Slaney mel + power_to_db(ref=max)
-> per-pixel z-score (StandardScaler fitted once at setup) -> audio-only ConvVAE (BASELINE config[1],
HybridVAE without the text branch) forward + loss + backward + Adam, bf16 activations / MFMA operands
with fp32 accumulation and fp32 master weights; for N > 1 ranks the flat fp32 gradient is all-reduced
(RCCL over xGMI) before Adam.  Weak scaling: 256 clips per GPU per step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload audio|hybrid] [--no-cpu-baseline]
N > 1 is launched by torch.distributed.run (one process per GPU); rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import hlmc_amd  # noqa: E402
from hlmc_amd import _lib as L  # noqa: E402

SR, NFFT, HOP, NMEL = 22050, 2048, 512, 128
FRAMES = 128
N_SAMPLES = (FRAMES - 1) * HOP  # 65024 samples -> 128 centred frames
PEAK_BF16_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def synthetic_pcm(batch, n, seed, device):
    """Seeded sum of 8 sinusoids (50-8000 Hz) + noise per clip, generated on the device."""
    g = torch.Generator(device=device).manual_seed(seed)
    t = torch.arange(n, device=device, dtype=torch.float32) / SR
    f = torch.rand(batch, 8, 1, device=device, generator=g) * 7950 + 50
    a = torch.rand(batch, 8, 1, device=device, generator=g) * 0.08 + 0.02
    ph = torch.rand(batch, 8, 1, device=device, generator=g) * 6.2831853
    y = (a * torch.sin(6.2831853 * f * t + ph)).sum(1)
    y += 0.01 * torch.randn(batch, n, device=device, generator=g)
    return y.clamp_(-1, 1).contiguous()


class MelStage:
    """PCM -> mel dB [B,128,128] -> z-score -> audio tensor [B,1,128,128] (f32) for the VAE."""

    def __init__(self, batch, device, scaler):
        self.plan = hlmc_amd.features._plan(SR, NFFT, HOP, NMEL)
        self.B = batch
        self.mel = torch.empty(batch, NMEL, FRAMES, device=device)
        self.audio = torch.empty(batch, 1, NMEL, FRAMES, device=device)
        self.ws = torch.empty(int(L.lib().hlmc_mel_workspace(self.plan, batch, N_SAMPLES)), dtype=torch.uint8,
                              device=device)
        self.scaler = scaler

    def __call__(self, pcm):
        L.check(L.lib().hlmc_mel_db(self.plan, L.stream(), pcm.data_ptr(), self.B, N_SAMPLES, FRAMES, 1e-10, 80.0,
                                    self.mel.data_ptr(), self.ws.data_ptr()))
        L.check(L.lib().hlmc_zscore_apply(L.stream(), self.mel.data_ptr(), self.B, NMEL * FRAMES,
                                          self.scaler.mean_d.data_ptr(), self.scaler.scale_d.data_ptr(), L.HLMC_F32,
                                          self.audio.data_ptr()))
        return self.audio


def conv_layers(batch, hw=(128, 128)):
    """(name, M, N, K) of every MFMA implicit-GEMM launch family in one train step (encoder + decoder)."""
    enc = (1, 32, 64, 128, 256, 512, 512)
    dec = (512, 512, 256, 128, 64, 32, 1)
    H, W = hw
    out = []
    h, w = H, W
    for l in range(6):
        h, w = h // 2, w // 2
        if l > 0:
            out.append((f"enc{l}_fwd", batch * h * w, enc[l + 1], 9 * enc[l], ("conv_s2", batch, 2 * h, 2 * w,
                                                                               enc[l], enc[l + 1])))
    h, w = H // 64, W // 64
    for l in range(5):
        # 4 sub-pixel phases with 1/2/2/4 taps: K summed over phases = 9 * Ci per low-res position
        out.append((f"dec{l}_fwd", batch * h * w, dec[l + 1], 9 * dec[l], ("subpixel", batch, h, w, dec[l], dec[l + 1])))
        h, w = 2 * h, 2 * w
    return out


def time_op(spec, device, reps=20):
    """Average duration (ms) of one launch of an op-level kernel, HIP events on the launch stream."""
    kind, B, Hi, Wi, Ci, Co = spec
    ws_bytes = 512 << 20
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    x = torch.randn(B, Hi, Wi, Ci, device=device).to(torch.bfloat16)
    wp = (torch.randn(Co, 3, 3, Ci, device=device) * 0.05).to(torch.bfloat16)
    bias = torch.zeros(Co, device=device)
    if kind == "conv_s2":
        y = torch.empty(B, Hi // 2, Wi // 2, Co, device=device, dtype=torch.bfloat16)
        fn = lambda: L.lib().hlmc_op_conv_s2(L.stream(), L.HLMC_BF16, x.data_ptr(), B, Hi, Wi, Ci, wp.data_ptr(),  # noqa
                                              bias.data_ptr(), Co, y.data_ptr(), ws.data_ptr(), ws_bytes)
    else:
        y = torch.empty(B, 2 * Hi, 2 * Wi, Co, device=device, dtype=torch.bfloat16)
        fn = lambda: L.lib().hlmc_op_subpixel(L.stream(), L.HLMC_BF16, x.data_ptr(), B, Hi, Wi, Ci, wp.data_ptr(),  # noqa
                                               bias.data_ptr(), Co, y.data_ptr(), ws.data_ptr(), ws_bytes)
    for _ in range(3):
        L.check(fn())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def cpu_baseline(batch=64, steps=3):
    """Oracle (torch-CPU restatement of the reference model + numpy restatement of librosa) on host cores."""
    from multiprocessing import Pool

    from oracle import mel_oracle, models_oracle

    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    pcm = mel_oracle.synthetic_pcm(batch, N_SAMPLES, seed=0)
    torch.manual_seed(42)
    model = models_oracle.HybridVAE(128, 768, (128, 128), audio_only=True)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    with Pool(cores) as pool:
        def one_step():
            mel = np.stack(pool.map(mel_oracle.extract_mel_spectrogram, list(pcm)))
            x = torch.from_numpy((mel - mel.mean(0)) / (mel.std(0) + 1e-8)).float()[:, None]
            opt.zero_grad()
            ra, _, mu, lv = model(x)
            loss = models_oracle.loss_function(ra, x, None, None, mu, lv)[0]
            loss.backward()
            opt.step()
        one_step()
        t0 = time.perf_counter()
        for _ in range(steps):
            one_step()
        dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 2), "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"audio-only HybridVAE 128x128 torch-CPU restatement fwd+bwd+Adam + numpy librosa-mel "
                      f"restatement ({cores}-process pool), bs={batch}, {steps} timed steps after 1 warmup "
                      f"({dt:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--workload", choices=["audio", "hybrid"], default="audio")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world == 1:
        raise SystemExit("--gpus N>1: launch with python -m torch.distributed.run --nproc-per-node N bench.py ...")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    B = args.batch
    audio_only = args.workload == "audio"
    # ---- setup (untimed): model, optimizer state, scaler fit on a calibration batch
    torch.manual_seed(42)
    model = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=audio_only, compute_dtype=args.dtype).to(device)
    trainer = hlmc_amd.Trainer(model, lr=1e-4, distributed=world > 1)
    pcm = synthetic_pcm(B, N_SAMPLES, seed=1000 + rank, device=device)
    text = (torch.randn(B, 384, device=device) / 384 ** 0.5) if not audio_only else None
    calib = hlmc_amd.extract_mel_spectrogram(pcm, fixed_time_steps=FRAMES)
    scaler = hlmc_amd.StandardScaler().fit(calib.reshape(B, -1))
    mel = MelStage(B, device, scaler)

    def step():
        x = mel(pcm)
        return trainer.step(x, text)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sums = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = trainer.loss_tuple(sums)[0]
    if not np.isfinite(loss):
        raise SystemExit(f"non-finite loss {loss}")

    if rank == 0:
        value = world * B * args.steps / elapsed
        ms = 1000 * elapsed / args.steps
        flops_clip = 1.0668e9 if not audio_only else 1.0597e9   # fwd+bwd (FlopCounterMode)
        rec = {"metric": "clips/sec mel+VAE train step, 128-mel x 128-frame, bs=256, 1/2/4/8 MI355X",
               "value": round(value, 2), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded sinusoid+noise PCM; random init)",
               "config": {"workload": ("Convolutional_VAE audio-only (BASELINE config[1])" if audio_only else
                                       "Convolutional_VAE hybrid, text_dim 384 (BASELINE config[2])") +
                                      ": PCM[256,65024] -> HIP mel-dB 128x128 -> z-score -> VAE fwd+bwd+Adam",
                          "per_gpu_batch": B, "global_batch": B * world, "mel": "128x128", "params": sum(
                              p.numel() for p in model.parameters()), "parallelism": f"dp{world}",
                          "final_loss": round(loss, 3),
                          "step_mfma_frac": round(value / world * flops_clip / 1e12 / PEAK_BF16_TFLOPS, 4)}}
        if not args.no_roofline:
            # dominant MFMA kernel family: the stride-2 conv GEMM with the most FLOPs per launch
            layers = conv_layers(B)
            name, M, N, K, spec = max(layers, key=lambda t: t[1] * t[2] * t[3])
            ms_k = time_op(spec, device)
            flops = 2.0 * M * N * K
            ach = flops / (ms_k * 1e-3) / 1e12
            rec["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": None,
                               "kernel": f"gemm_nt_kernel {name} M={M} N={N} K={K} (bf16, avg {ms_k * 1e3:.1f} us/launch)"}
        if not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline()
        print(json.dumps(rec), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
