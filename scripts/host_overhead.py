"""Host enqueue time of the bench step vs its GPU time: is the training step launch-bound?"""
import sys, time
import torch
sys.path.insert(0, ".")
import hlmc_amd
from bench import MelStage, synthetic_pcm, N_SAMPLES, FRAMES  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(42)
model = hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True, compute_dtype="bf16").to(dev)
tr = hlmc_amd.Trainer(model, lr=1e-4)
B = 256
pcm = synthetic_pcm(B, N_SAMPLES, seed=1000, device=dev)
calib = hlmc_amd.extract_mel_spectrogram(pcm, fixed_time_steps=FRAMES)
sc = hlmc_amd.StandardScaler().fit(calib.reshape(B, -1))
mel = MelStage(B, dev, sc)
step = lambda: tr.step(mel(pcm), None)
for _ in range(5):
    step()
torch.cuda.synchronize()
for n in (1, 5, 20):
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"steps={n}: host enqueue {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step")
