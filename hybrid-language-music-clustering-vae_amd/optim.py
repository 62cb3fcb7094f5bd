"""Adam on the HIP path: one multi-tensor launch per param group (src/Convolutional_VAE.py:208,235).

Same constructor, defaults, update rule and state layout ('step', 'exp_avg', 'exp_avg_sq') as
torch.optim.Adam (non-amsgrad, non-maximize), so optimizer state_dicts interchange with the
reference's.  Parameters must be float32 CUDA tensors.
"""
from __future__ import annotations

import torch

from . import _lib as L


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0 or eps < 0 or not 0 <= betas[0] < 1 or not 0 <= betas[1] < 1 or weight_decay < 0:
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps, gs, ms, vs, ns, ks = [], [], [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32 or not p.is_cuda:
                    raise L.HLMCError("hlmc Adam needs dense float32 CUDA parameters")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                # 'step' is a host (CPU) tensor as in torch.optim.Adam (non-capturable): no device sync
                st["step"] += 1
                ks.append(int(st["step"]))
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                ps.append(p)
                gs.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
                ns.append(p.numel())
            if not ps:
                continue
            b1, b2 = group["betas"]
            for step in sorted(set(ks)):
                idx = [i for i, k in enumerate(ks) if k == step]
                L.check(L.lib().hlmc_adam_step(
                    L.stream(), len(idx), L.vp_array([ps[i].data_ptr() for i in idx]),
                    L.vp_array([gs[i].data_ptr() for i in idx]), L.vp_array([ms[i].data_ptr() for i in idx]),
                    L.vp_array([vs[i].data_ptr() for i in idx]), L.i64_array([ns[i] for i in idx]),
                    float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                    step, None), "hlmc_adam_step")
        return loss
