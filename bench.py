"""Benchmark: clips/sec of the mel + VAE train step (BASELINE.json metric), 128-mel x 128-frame, bs=256/GPU.

One step = PCM [256, 65024] (synthetic, resident in HBM) -> HIP STFT + Slaney mel + power_to_db(ref=max)
-> per-pixel z-score (StandardScaler fitted once at setup) -> audio-only ConvVAE (BASELINE config[1],
HybridVAE without the text branch) forward + loss + backward + Adam, bf16 activations / MFMA operands
with fp32 accumulation and fp32 master weights; for N > 1 ranks the flat fp32 gradient is all-reduced
(RCCL over xGMI) before Adam.  Weak scaling: 256 clips per GPU per step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload audio|hybrid|cvae] [--dtype bf16|fp32]
                    [--grad-dtype bf16|fp32] [--no-cpu-baseline] [--no-roofline] [--no-extras] [--graph]
N > 1 runs one process per GPU under torch.distributed.run; `python bench.py --gpus N` outside torchrun starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child process (nothing touches the GPU in the
parent), relays rank 0's JSON line and exits with the child's status.  Rank 0 prints ONE JSON line.
Besides the headline (BASELINE config[1]), the default run times three more workloads on the same mel stage and
reports them under "extras" (never as `value`): the headline in fp32 (the parity precision), the hybrid ConvVAE
with 384-d lyrics (config[2]) and the genre-conditioned ConditionalVAE (config[3]), each bs=256 per GPU; the
K-Means fit of config[3]/[4]'s clustering scale (N = 100 000 x 128, k = 10, n_init = 10) beside sklearn's on the
host cores; and config[4] end to end (run_pipeline: 30 s PCM -> mel -> scaler -> HybridVAE 128x1024 training ->
latents -> K-Means) on --e2e-clips clips.
"""
from __future__ import annotations

import argparse
import ctypes as C
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
    """PCM -> mel dB [B,128,128] -> z-score -> audio tensor [B,1,128,128] (f32) for the VAE: the STFT/mel kernel,
    then one dB pass with the fitted StandardScaler's transform fused in (hlmc_mel_db_zscore)."""

    def __init__(self, batch, device, scaler):
        self.plan = hlmc_amd.features._plan(SR, NFFT, HOP, NMEL)
        self.B = batch
        self.audio = torch.empty(batch, 1, NMEL, FRAMES, device=device)
        self.ws = torch.empty(int(L.lib().hlmc_mel_workspace(self.plan, batch, N_SAMPLES)), dtype=torch.uint8,
                              device=device)
        self.scaler = scaler

    def __call__(self, pcm):
        L.check(L.lib().hlmc_mel_db_zscore(self.plan, L.stream(), pcm.data_ptr(), self.B, N_SAMPLES, FRAMES, 1e-10,
                                           80.0, self.scaler.mean_d.data_ptr(), self.scaler.scale_d.data_ptr(),
                                           L.HLMC_F32, self.audio.data_ptr(), self.ws.data_ptr()))
        return self.audio


# Op kinds of the live kernel probe (include/hlmc.h hlmc_probe_arm) and the kernel each one launches
PROBE_KINDS = {
    1: ("conv_s2", "gemm_nt ConvS2Loader (conv fwd / convT dgrad)", "mfma"),
    2: ("subpixel", "gemm_nt SubpixelLoader (convT fwd / conv dgrad)", "mfma"),
    4: ("wgrad_s2", "gemm_tn KRowConvS2 (conv / convT weight gradient)", "mfma"),
    8: ("linear", "gemm_nt DenseLoader (Linear fwd / dgrad)", "mfma"),
    16: ("linear_wgrad", "gemm_tn KRowDense (Linear weight gradient)", "mfma"),
    32: ("stft_mel", "stft_mel0_kernel (STFT + mel)", "hbm"),
    64: ("bn", "BatchNorm / reduction streaming family (bn_act, bn_bwd_moments, bn_bwd_apply, col_moments, "
               "parts_fold, finalizers)", "hbm"),
}


WORKLOADS = {
    "audio": "Convolutional_VAE audio-only (BASELINE config[1])",
    "hybrid": "Convolutional_VAE hybrid, text_dim 384 (BASELINE config[2])",
    "cvae": "Conditional_VAE genre-conditioned, latent 64, text_dim 768, 10 classes (BASELINE config[3])",
}


def build_workload(name, dtype, B, device, world, seed=42, grad_dtype=torch.float32):
    """Model (seed-42 init), fused Trainer and the synthetic side inputs (lyrics embeddings ~ N(0, 1/td), one-hot
    genres) of one BASELINE workload at 128 x 128 mel."""
    torch.manual_seed(seed)
    g = torch.Generator(device=device).manual_seed(7)
    text = cond = None
    if name == "cvae":
        model = hlmc_amd.ConditionalVAE(64, 768, 10, (128, 128), compute_dtype=dtype).to(device)
        text = torch.randn(B, 768, device=device, generator=g) / 768 ** 0.5
        cond = torch.nn.functional.one_hot(torch.randint(0, 10, (B,), device=device, generator=g), 10).float()
    else:
        model = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=name == "audio", compute_dtype=dtype).to(device)
        if name == "hybrid":
            text = torch.randn(B, 384, device=device, generator=g) / 384 ** 0.5
    trainer = hlmc_amd.Trainer(model, lr=1e-4, distributed=world > 1, grad_dtype=grad_dtype)
    return model, trainer, text, cond


def time_workload(name, dtype, B, device, world, mel, pcms, dist, steps=10, warmup=3, grad_dtype=torch.float32):
    """Whole-job clips/s of one extra workload (same mel stage, same rotating PCM batches, same timing protocol as
    the headline)."""
    model, trainer, text, cond = build_workload(name, dtype, B, device, world, grad_dtype=grad_dtype)
    for k in range(warmup):
        trainer.step(mel(pcms[k % len(pcms)]), text, cond)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        sums = trainer.step(mel(pcms[k % len(pcms)]), text, cond)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    loss = trainer.loss_tuple(sums)[0]
    out = {"workload": WORKLOADS[name], "dtype": dtype, "value": round(world * B * steps / el, 2), "unit": "clips/s",
           "ms_per_step": round(1000 * el / steps, 4), "steps": steps, "warmup": warmup,
           "params": sum(p.numel() for p in model.parameters()), "final_loss": round(loss, 3),
           "finite": bool(np.isfinite(loss))}
    del trainer, model
    torch.cuda.empty_cache()
    return out


def _kmeans_data(n=100000, d=128, k=10, spread=0.3, seed=5):
    """Latent-like rows: N(0, 1) points around k centres drawn from N(0, spread^2) (overlapping clusters, the
    tests/golden N = 100k recipe), float32."""
    rng = np.random.default_rng(seed)
    c = rng.normal(0, spread, (k, d))
    lab = rng.integers(0, k, n)
    return (c[lab] + rng.normal(0, 1.0, (n, d))).astype(np.float32)


def time_kmeans(device, dist, world, rank, cpu_leg=True):
    """KMeans(10, random_state=42, n_init=10).fit on 100 000 x 128 latents (src/Convolutional_VAE.py:317-319 at
    BASELINE config[4]'s clustering scale): the HIP k-means++ draws / distances and Lloyd E/M-step kernels, the
    n_init restarts in lockstep (sharded over ranks), against sklearn's fit on the host cores (rank 0, N = 1)."""
    X = _kmeans_data()
    Xd = torch.from_numpy(X).to(device)
    group = dist.group.WORLD if dist else None
    hlmc_amd.KMeans(10, random_state=42, n_init=10, process_group=group).fit(Xd)      # warm-up (allocations)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    km = hlmc_amd.KMeans(10, random_state=42, n_init=10, process_group=group).fit(Xd)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    out = {"workload": "KMeans(n_clusters=10, random_state=42, n_init=10).fit, N=100000 x 128 f32 latents",
           "fit_ms": round(1e3 * el, 2), "n_iter": int(km.n_iter_), "inertia": float(km.inertia_),
           "higher_is_better": False}
    if cpu_leg and rank == 0 and world == 1:
        from sklearn.cluster import KMeans as SkKMeans
        from sklearn.metrics import adjusted_rand_score
        from threadpoolctl import threadpool_limits
        cores, _ = host_cpu_share()
        with threadpool_limits(limits=cores):
            t0 = time.perf_counter()
            sk = SkKMeans(10, random_state=42, n_init=10).fit(X)
            sk_s = time.perf_counter() - t0
        out["sklearn_cpu"] = {"fit_ms": round(1e3 * sk_s, 1), "cores": cores, "n_iter": int(sk.n_iter_),
                              "inertia": float(sk.inertia_)}
        out["speedup_vs_sklearn"] = round(sk_s / el, 1)
        # sklearn at `cores` threads sums centres in a thread-dependent order; the bit-exact label contract is pinned
        # against single-thread sklearn in tests/test_kmeans_gpu.py — here the agreement is reported as ARI
        out["ari_vs_sklearn"] = round(float(adjusted_rand_score(sk.labels_, km.labels_)), 6)
    return out


def time_e2e(device, dist, world, n_clips, grad_dtype):
    """BASELINE config[4] end to end (hlmc_amd.pipeline.run_pipeline): synthetic 30 s PCM -> HIP mel-dB (1024 kept
    frames) -> per-pixel StandardScaler -> HybridVAE 128x1024 (768-d lyrics) bf16 training, one epoch, bs 256 per
    GPU -> eval latents -> KMeans(10, n_init=10).  Strong scaling: n_clips in total, sharded over the ranks."""
    group = dist.group.WORLD if dist else None
    hlmc_amd.pipeline.run_pipeline(512 * world, batch=256, epochs=1, process_group=group, grad_dtype=grad_dtype)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    r = hlmc_amd.pipeline.run_pipeline(n_clips, batch=256, epochs=1, process_group=group, grad_dtype=grad_dtype)
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    src = r["stages_s"].get("pcm_source", 0.0)
    return {"workload": "config[4] end to end: 30 s PCM -> mel-dB -> scaler -> HybridVAE 128x1024 bf16 train (1 epoch) "
                        "-> eval latents -> KMeans(10, n_init=10)",
            "n_clips": n_clips, "value": round(n_clips / el, 2), "unit": "clips/s", "seconds": round(el, 3),
            # the synthetic PCM generation (torch, stands in for WAV decoding, which is out of scope) excluded
            "value_excl_pcm_source": round(n_clips / max(1e-9, el - src), 2),
            "stages_s_rank0": {k: round(v, 4) for k, v in r["stages_s"].items()}, "train_steps": r["train_steps"],
            "final_loss": r["final_loss"], "kmeans_n_iter": int(r["kmeans_n_iter"])}


def probe_read(cap=4096):
    n = L.c_int()
    tot, fl, by = L.c_f64(), L.c_f64(), L.c_f64()
    each = (L.c_f32 * cap)()
    L.check(L.lib().hlmc_probe_read(C.byref(n), C.byref(tot), C.byref(fl), C.byref(by), each, cap), "hlmc_probe_read")
    return {"launches": n.value, "ms": tot.value, "flops": fl.value, "bytes": by.value,
            "each_ms": list(each)[: min(n.value, cap)]}


def kind_roofline(kind, st):
    """Achieved rate of one probed kernel kind: algorithmic work per launch / its average launch duration."""
    name, kernel, bound = PROBE_KINDS[kind]
    n = max(1, st["launches"])
    avg_s = st["ms"] / n * 1e-3
    if bound == "mfma":
        ach = st["flops"] / n / avg_s / 1e12
        peak, unit = PEAK_BF16_TFLOPS, "TFLOP/s"
    else:
        ach = st["bytes"] / n / avg_s / 1e9
        peak, unit = PEAK_HBM_GBS, "GB/s"
    return {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
            "kernel": kernel, "op": name, "launches": st["launches"], "avg_us_per_launch": round(avg_s * 1e6, 2),
            "flops_per_launch": st["flops"] / n, "bytes_per_launch": st["bytes"] / n}


def pmc_traffic(kind):
    """The committed rocprofv3 summary of this kind (profiles/pmc_traffic.json, scripts/pmc_traffic.py): HBM bytes
    per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB -> bytes, per the gfx950 correction of MI355X_MICROARCH.md), the
    counter-based MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the dispatch's SIMD-cycles) and the kernel-trace
    average launch duration in us; {} when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = dict(d["kinds"][PROBE_KINDS[kind][0]])
        e["source"] = d.get("source")
        e["file"] = d.get("file", "profiles/pmc_traffic.json")
        return e
    except (OSError, KeyError, ValueError):
        return {}


def host_cpu_share():
    """Host cores the CPU baseline may use: every core in this process's affinity mask, unless a cgroup CPU
    quota (cgroup v2 cpu.max) grants fewer, in which case the quota's CPU count.  Returns (cores, quota)."""
    cores = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(period), 2)
            cores = max(1, min(cores, int(quota)))
    except (OSError, ValueError):
        pass
    return cores, quota


def cpu_baseline(batch=256, steps=5, warmup=2):
    """Oracle (torch-CPU restatement of the reference model + numpy restatement of librosa) on host cores:
    SURVEY §8(d) protocol (2 warm-up steps, >= 5 timed), the mel stage and the VAE step timed separately so the
    VAE-only rate (the reference's Convolutional_VAE.py train step alone) is reported beside the whole step."""
    from multiprocessing import Pool

    from oracle import mel_oracle, models_oracle

    cores, quota = host_cpu_share()
    torch.set_num_threads(cores)
    pcm = mel_oracle.synthetic_pcm(batch, N_SAMPLES, seed=0)
    torch.manual_seed(42)
    model = models_oracle.HybridVAE(128, 768, (128, 128), audio_only=True)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    with Pool(cores) as pool:
        def mel_stage():
            mel = np.stack(pool.map(mel_oracle.extract_mel_spectrogram, list(pcm)))
            return torch.from_numpy((mel - mel.mean(0)) / (mel.std(0) + 1e-8)).float()[:, None]

        def vae_step(x):
            opt.zero_grad()
            ra, _, mu, lv = model(x)
            loss = models_oracle.loss_function(ra, x, None, None, mu, lv)[0]
            loss.backward()
            opt.step()

        for _ in range(warmup):
            vae_step(mel_stage())
        t_mel = t_vae = 0.0
        for _ in range(steps):
            t0 = time.perf_counter()
            x = mel_stage()
            t1 = time.perf_counter()
            vae_step(x)
            t2 = time.perf_counter()
            t_mel += t1 - t0
            t_vae += t2 - t1
    dt = t_mel + t_vae
    return {"value": round(batch * steps / dt, 2), "unit": "clips/s", "cores": cores, "kind": "port",
            "vae_only_value": round(batch * steps / t_vae, 2), "mel_only_value": round(batch * steps / t_mel, 2),
            "affinity_cores": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota,
            "sample": f"audio-only HybridVAE 128x128 torch-CPU restatement fwd+bwd+Adam ({cores} torch threads) + "
                      f"numpy librosa-mel restatement ({cores}-process pool), bs={batch}, {steps} timed steps after "
                      f"{warmup} warm-up steps ({dt:.1f} s: mel {t_mel:.1f} s, VAE {t_vae:.1f} s)"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def relaunch_under_torchrun(n, timeout=1800.0):
    """`--gpus N > 1` outside torch.distributed.run: run this same command line as N ranks in a child
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1).  Called before any GPU or libhlmc use,
    so the parent never initialises the device; the child is a subprocess, never an exec.  Rank 0's JSON line is
    relayed to stdout, everything else the ranks print goes to stderr.  Returns the child's exit status, or 124 when
    the child's process group had to be ended after `timeout` seconds (a hung rank would otherwise block forever)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    import signal
    import threading
    env = dict(os.environ, HLMC_BENCH_SELF_LAUNCHED="1")
    # own process group, so a hung rank (e.g. stuck in a rendezvous) can be ended as a whole after the timeout
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1, start_new_session=True)
    expired = threading.Event()

    def _expire():
        expired.set()
        sys.stderr.write(f"bench: the {n}-rank child exceeded {timeout:.0f} s; terminating its process group\n")
        for sig in (signal.SIGTERM, signal.SIGKILL):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                return
            try:
                proc.wait(timeout=10)
                return
            except subprocess.TimeoutExpired:
                pass

    timer = threading.Timer(timeout, _expire)
    timer.daemon = True
    timer.start()
    try:
        for line in proc.stdout:
            if line.startswith("{") and '"metric"' in line:
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.write(line)
        rc = proc.wait()
    finally:
        timer.cancel()
    return 124 if expired.is_set() else rc


PROBE_STEPS = int(os.environ.get("HLMC_PROBE_STEPS", "3"))  # timed steps whose dominant-kernel launches are timed
PCM_BATCHES = 5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--workload", choices=["audio", "hybrid", "cvae"], default="audio")
    ap.add_argument("--no-extras", action="store_true", help="skip the fp32 / hybrid / CVAE extra lines")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--grad-dtype", choices=["bf16", "fp32"], default="fp32",
                    help="gradient all-reduce wire for N > 1 (default fp32, the reference's numerics; bf16 halves the "
                         "xGMI bytes and is reported as the labelled `headline_bf16_wire` extra, DESIGN.md §7)")
    ap.add_argument("--e2e-clips", type=int, default=100000,
                    help="clips of the config[4] end-to-end extra line (BASELINE configs[4]: 100k synthetic clips)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one HIP graph (N = 1 only; measured 12%% slower on ROCm 7: the graph "
                         "executor serialises the weight-gradient stream's branch, see DESIGN.md)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_under_torchrun(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; HLMC_DIST_BACKEND=gloo (with ranks sharing a device) rehearses the N > 1 control flow
    # (barriers, max-over-ranks timing, bucketed all-reduce) on a one-GPU box
    backend = os.environ.get("HLMC_DIST_BACKEND", "nccl")
    local_dev = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local_dev)
    device = torch.device("cuda", local_dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    B = args.batch
    audio_only = args.workload == "audio"
    # ---- setup (untimed): model, optimizer state, scaler fit on a calibration batch
    # PCM_BATCHES distinct batches (5 x 66.6 MB = 333 MB at B = 256, more than the 256 MiB Infinity Cache), one per
    # step in rotation: every step's STFT streams its PCM from HBM, not from a cache that held the last step's
    pcms = [synthetic_pcm(B, N_SAMPLES, seed=1000 + 17 * j + rank, device=device) for j in range(PCM_BATCHES)]
    pcm = pcms[0]
    calib = hlmc_amd.extract_mel_spectrogram(pcm, fixed_time_steps=FRAMES)
    scaler = hlmc_amd.StandardScaler().fit(calib.reshape(B, -1))
    mel = MelStage(B, device, scaler)
    gd = args.grad_dtype
    grad_dtype = torch.bfloat16 if gd == "bf16" else torch.float32
    model, trainer, text, cond = build_workload(args.workload, args.dtype, B, device, world, grad_dtype=grad_dtype)
    nstep = [0]

    def step():
        p = pcms[nstep[0] % PCM_BATCHES]
        nstep[0] += 1
        x = mel(p)
        return trainer.step(x, text, cond)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    breakdown, dominant = {}, None
    if not args.no_roofline:
        # untimed calibration: kernel time per step of every probed kind (one extra step each); the kind with
        # the most time is the dominant kernel whose launches are then timed live inside the timed region
        for kind in PROBE_KINDS:
            # capacity for the timed probe too: every timing event is created here, outside the timed region
            L.check(L.lib().hlmc_probe_arm(kind, max(256, 64 * min(args.steps, PROBE_STEPS))), "hlmc_probe_arm")
            step()
            st = probe_read()
            if st["launches"]:
                r = kind_roofline(kind, st)
                e = {"us_per_step": round(st["ms"] * 1e3, 1), "launches_per_step": st["launches"],
                     "achieved": r["achieved"], "unit": r["unit"], "frac": r["frac"],
                     "bytes_per_launch": round(r["bytes_per_launch"]), "flops_per_launch": round(r["flops_per_launch"])}
                # HBM traffic of the kind from the committed PMC summary against its algorithmic bytes
                pm = pmc_traffic(kind)
                if pm.get("hbm_bytes_per_launch") and r["bytes_per_launch"] > 0:
                    e["traffic_per_launch"] = round(pm["hbm_bytes_per_launch"])
                    e["traffic_ratio"] = round(pm["hbm_bytes_per_launch"] / r["bytes_per_launch"], 3)
                breakdown[r["op"]] = e
        # the dominant single kernel (the BatchNorm family is 7 kernel types over ~96 launches per step: reported
        # from this untimed calibration only — event pairs around all its launches would cost the timed steps ~2.5 %)
        dominant = max((k for k in PROBE_KINDS if k != 64),
                       key=lambda k: breakdown.get(PROBE_KINDS[k][0], {}).get("us_per_step", 0.0))
        # rehearse the timed probe once (untimed) so every event it records has been used before the clock starts
        L.check(L.lib().hlmc_probe_arm(dominant, 64 * min(args.steps, PROBE_STEPS)), "hlmc_probe_arm")
        for _ in range(min(args.steps, PROBE_STEPS)):
            step()
        probe_read()
        torch.cuda.synchronize()
    graphed = None
    if world == 1 and args.graph:
        # the whole step (mel stage + train step) as one HIP graph; the probe's event pair around each launch of
        # the dominant kernel is captured with it and re-recorded by every replay
        arm = (lambda: L.check(L.lib().hlmc_probe_arm(dominant, 64), "hlmc_probe_arm")) if dominant else None
        graphed = hlmc_amd.GraphedStep(trainer, step, warmup=1, before_capture=arm)
        run_step = graphed
    else:
        run_step = step
    # live timing of the dominant kind over the LAST `probe_steps` timed steps (the event pairs cost a little;
    # arming them for every step measurably lowered the headline on the two-stream backward)
    probe_steps = min(args.steps, PROBE_STEPS)
    probe_from = args.steps - probe_steps if (dominant and not graphed) else -1
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if k == probe_from:
            L.check(L.lib().hlmc_probe_arm(dominant, 64 * probe_steps), "hlmc_probe_arm")
        sums = run_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    live, probe_note = None, None
    if dominant:
        try:
            live = probe_read()
        except L.HLMCError as e:  # event nodes not readable after replay: time the kind on eager steps instead
            probe_note = f"graph event timing unavailable ({e}); eager steps after the timed region"
            if graphed:
                graphed.release()
            L.check(L.lib().hlmc_probe_arm(dominant, 64 * 4), "hlmc_probe_arm")
            for _ in range(4):
                step()
            live = probe_read()
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = trainer.loss_tuple(sums)[0]
    if not np.isfinite(loss):
        raise SystemExit(f"non-finite loss {loss}")
    params_of_headline = sum(p.numel() for p in model.parameters())
    extras = {}
    if not args.no_extras and args.workload == "audio" and args.dtype == "bf16" and args.batch == 256:
        del trainer, model
        torch.cuda.empty_cache()
        for key, (wl, dt) in {"audio_fp32": ("audio", "fp32"), "hybrid_td384_bf16": ("hybrid", "bf16"),
                              "cvae_bf16": ("cvae", "bf16")}.items():
            extras[key] = time_workload(wl, dt, B, device, world, mel, pcms, dist, grad_dtype=grad_dtype)
        if world > 1:  # the headline on the half-width gradient wire (convert + all-reduce + copy back on the comm stream)
            extras["headline_bf16_wire"] = dict(time_workload("audio", "bf16", B, device, world, mel, pcms, dist,
                                                              steps=args.steps, warmup=args.warmup,
                                                              grad_dtype=torch.bfloat16), grad_wire="bf16")
        extras["kmeans_n100k_k10"] = time_kmeans(device, dist, world, rank)
        extras[f"config4_e2e_n{args.e2e_clips // 1000}k"] = time_e2e(device, dist, world, args.e2e_clips, grad_dtype)

    if rank == 0:
        n_params = params_of_headline
        value = world * B * args.steps / elapsed
        ms = 1000 * elapsed / args.steps
        # fwd+bwd FLOPs per clip (FlopCounterMode on the reference classes); CVAE not measured there
        flops_clip = {"audio": 1.0597e9, "hybrid": 1.0668e9}.get(args.workload)
        rec = {"metric": "clips/sec mel+VAE train step, 128-mel x 128-frame, bs=256, 1/2/4/8 MI355X",
               "value": round(value, 2), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded sinusoid+noise PCM; random init)",
               "config": {"workload": WORKLOADS[args.workload] +
                                      ": PCM[256,65024] -> HIP mel-dB 128x128 -> z-score -> VAE fwd+bwd+Adam",
                          "per_gpu_batch": B, "global_batch": B * world, "mel": "128x128", "params": n_params,
                          "parallelism": f"dp{world}",
                          "world_size": dist.get_world_size() if dist else 1,
                          "backend": backend if dist else None, "grad_wire": gd if dist else None,
                          "launch": ("self-launched torch.distributed.run child" if
                                     os.environ.get("HLMC_BENCH_SELF_LAUNCHED") == "1" else
                                     "torch.distributed.run" if dist else "single process"),
                          "pcm_batches": f"{PCM_BATCHES} distinct batches in rotation "
                                         f"({PCM_BATCHES * B * N_SAMPLES * 4 / 1e6:.0f} MB)",
                          "final_loss": round(loss, 3),
                          "execution": "HIP graph replay of the whole step" if graphed else "eager launches",
                          "step_mfma_frac": (round(value / world * flops_clip / 1e12 / PEAK_BF16_TFLOPS, 4)
                                             if flops_clip else None)}}
        if live is not None:
            roof = kind_roofline(dominant, live)
            pmc = pmc_traffic(dominant)
            roof["traffic"] = pmc.get("hbm_bytes_per_launch")
            roof["mfma_busy"] = pmc.get("mfma_busy")
            roof["traffic_source"] = pmc.get("source")
            # the same rate from the committed rocprofv3 kernel-trace average (no event pairs, no live probe):
            # reproducible from profiles/ alone.  The live figure above includes the other stream's contention.
            tavg = pmc.get("trace_avg_us")
            if tavg:
                work = roof["flops_per_launch"] if roof["bound"] == "mfma" else roof["bytes_per_launch"]
                ach_t = work / (tavg * 1e-6) / (1e12 if roof["bound"] == "mfma" else 1e9)
                roof["trace"] = {"avg_us_per_launch": tavg, "launches": pmc.get("trace_dispatches"),
                                 "achieved": round(ach_t, 2), "frac": round(ach_t / roof["peak"], 4),
                                 "file": pmc.get("file")}
            roof["timing"] = (f"HIP events around each launch on its stream, inside the timed region "
                              + (f"(event nodes of the step graph; the {live['launches']} launches of the last "
                                 f"of {args.steps} replays)" if graphed else
                                 f"({live['launches']} launches in the last {probe_steps} of the {args.steps} "
                                 f"timed steps)"))
            if probe_note:
                roof["timing"] = probe_note
            roof["per_kind_untimed"] = breakdown  # concurrent streams: kernel times overlap
            rec["roofline"] = roof
        if extras:
            rec["extras"] = extras
        if not args.no_cpu_baseline and world == 1:  # the host cores' baseline: rank 0 at N = 1 only
            rec["cpu_baseline"] = cpu_baseline()
        print(json.dumps(rec), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
