"""Debug aid: one HybridVAE train step (B=4, seeded; bf16, or fp32 with DBG_DTYPE=fp32) under the current HLMC_*
environment; saves recon, mu, BatchNorm running statistics and every gradient to gpurun_out/<tag>.pt, then (with
two tags) compares them.
  python scripts/debug_bn_in.py run TAG ;  python scripts/debug_bn_in.py cmp TAG_A TAG_B"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(tag):
    import hlmc_amd
    torch.manual_seed(42)
    m = hlmc_amd.HybridVAE(128, 768, (128, 128), compute_dtype=os.environ.get("DBG_DTYPE", "bf16")).cuda()
    g = torch.Generator().manual_seed(3)
    audio = torch.randn(4, 1, 128, 128, generator=g).cuda()
    text = (torch.randn(4, 768, generator=g) / 768 ** 0.5).cuda()
    eps = torch.randn(4, 128, generator=g).cuda()
    out = m(audio, text, eps=eps)
    loss = hlmc_amd.loss_function(out[0], audio, out[1], text, out[2], out[3])
    loss[0].backward()
    torch.cuda.synchronize()
    res = {"recon": out[0].detach().cpu(), "mu": out[2].detach().cpu(),
           "buffers": {n: b.detach().cpu().clone() for n, b in m.named_buffers()},
           "grads": {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}}
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(res, f"gpurun_out/{tag}.pt")


def cmp(a, b):
    A = torch.load(f"gpurun_out/{a}.pt", weights_only=True)
    B = torch.load(f"gpurun_out/{b}.pt", weights_only=True)

    def rel(x, y):
        return float((x.double() - y.double()).norm() / max(float(y.double().norm()), 1e-30))
    print("recon", rel(A["recon"], B["recon"]), "mu", rel(A["mu"], B["mu"]))
    thr = float(os.environ.get("DBG_THR", "1e-2"))
    for n in A["buffers"]:
        e = rel(A["buffers"][n].float(), B["buffers"][n].float())
        if e > thr / 10:
            print("buffer", n, e)
    for n in A["grads"]:
        e = rel(A["grads"][n], B["grads"][n])
        if e > thr:
            print("grad", n, e)


if __name__ == "__main__":
    run(sys.argv[2]) if sys.argv[1] == "run" else cmp(sys.argv[2], sys.argv[3])
