"""Vendor yardstick for the dense middle: torch.nn.functional.linear (hipBLASLt) on the audio HybridVAE's linear
shapes at B = 256, bf16, forward / data-gradient / weight-gradient, HIP-event timed (min of 5 x 200 calls)."""
import torch

dev = torch.device("cuda")
B = 256
layers = {"audio_fc": (1024, 8192), "fc_fusion": (512, 1024), "fc_mu": (128, 512), "fc_logvar": (128, 512),
          "decoder_input": (512, 128), "decoder_split": (1024, 512), "audio_decoder_fc": (8192, 1024)}


def t(fn, n=200):
    best = 1e9
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / n * 1e3)
    return best


tot = [0.0, 0.0, 0.0]
for name, (N, K) in layers.items():
    x = torch.randn(B, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(B, N, device=dev, dtype=torch.bfloat16)
    for _ in range(10):
        torch.nn.functional.linear(x, w, b)
    f = t(lambda: torch.nn.functional.linear(x, w, b))
    d = t(lambda: dy @ w)
    g = t(lambda: dy.t() @ x)
    tot[0] += f; tot[1] += d; tot[2] += g
    print(f"{name:18s} N={N:5d} K={K:5d}  fwd {f:6.1f} us  dgrad {d:6.1f} us  wgrad {g:6.1f} us")
print(f"total fwd {tot[0]:.1f} us, dgrad {tot[1]:.1f} us, wgrad {tot[2]:.1f} us")
