"""BASELINE config[4] end to end on ONE MI355X (hlmc_amd.pipeline.run_pipeline): N synthetic 30 s clips ->
HIP mel-dB (1024 frames) -> GPU StandardScaler -> HybridVAE(128 x 1024, lyrics 768) training -> eval encode ->
KMeans(10, random_state=42, n_init=10).  Prints one JSON line with the per-stage seconds.

    python scripts/e2e.py [--clips 100000] [--batch 256] [--epochs 1] [--dtype bf16]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hlmc_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=100000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-init", type=int, default=10)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    # warm the kernels / allocator on a small run first (first-launch costs stay out of the stage timings)
    hlmc_amd.pipeline.run_pipeline(512, batch=args.batch, epochs=1, compute_dtype=args.dtype, k=args.k, n_init=1)
    r = hlmc_amd.pipeline.run_pipeline(args.clips, batch=args.batch, epochs=args.epochs, compute_dtype=args.dtype,
                                       k=args.k, n_init=args.n_init)
    counts = np.bincount(r.pop("labels"), minlength=args.k).tolist()
    st = r["stages_s"]
    r["stages_s"] = {k: round(v, 4) for k, v in st.items()}
    r["stage_clips_per_s"] = {k: round(args.clips * (args.epochs if k == "train" else 1) / v, 1)
                              for k, v in st.items() if k not in ("total", "pcm_source") and v > 0}
    r["cluster_sizes"] = counts
    r["config"] = "BASELINE config[4] on 1 GPU: 30 s synthetic PCM -> mel 128x1024 -> z-score -> HybridVAE(128, " \
                  "text 768) train -> eval encode -> KMeans(k, random_state=42, n_init)"
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
