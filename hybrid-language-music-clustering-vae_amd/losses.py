"""VAE losses on the HIP path (deterministic float64 reductions, no host sync).

  loss_function       — src/Convolutional_VAE.py:187-194   sum-MSE(audio) + 350 sum-MSE(text) + beta KLD
  cvae_loss_function  — src/Conditional_VAE.py:233-246     sum-MSE(audio) + 200 sum-MSE(text) + beta KLD
  vae_loss            — src/Simple_VAE.py:108-114          mean-MSE + beta mean-KL

Each returns the reference's tuple of 0-dim float32 tensors; gradients flow to the reconstructions,
mu and logvar (the targets are constants, as in the reference's training loops).
"""
from __future__ import annotations

import torch

from . import _lib as L


class _LossFn(torch.autograd.Function):
    """sums = (sum (ra-a)^2, sum (rt-t)^2, sum (1 + lv - mu^2 - e^lv)) on device; tuple formed from them."""

    @staticmethod
    def forward(ctx, ra, a, rt, t, mu, lv, w_text, beta, mean_mode):
        L.require_cuda(ra, a, rt, t, mu, lv)
        na, nt, nl = ra.numel(), (rt.numel() if rt is not None else 0), mu.numel()
        dev = ra.device
        sums = torch.empty(3, dtype=torch.float64, device=dev)
        ws = torch.empty(max(8, int(L.lib().hlmc_loss_workspace(na, nt, nl))), dtype=torch.uint8, device=dev)
        L.check(L.lib().hlmc_loss_sums(L.stream(), L.ptr(ra), L.ptr(a), na, L.ptr(rt), L.ptr(t), nt, L.ptr(mu),
                                       L.ptr(lv), nl, sums.data_ptr(), ws.data_ptr()), "hlmc_loss_sums")
        if mean_mode:
            la = sums[0] / na
            kld = -0.5 * sums[2] / nl
            lt = torch.zeros((), dtype=torch.float64, device=dev)
        else:
            la, lt, kld = sums[0], sums[1], -0.5 * sums[2]
        total = la + w_text * lt + beta * kld
        ctx.save_for_backward(ra, a, rt if rt is not None else torch.empty(0, device=dev),
                              t if t is not None else torch.empty(0, device=dev), mu, lv)
        ctx.cfg = (w_text, beta, mean_mode, na, nt, nl)
        return total.float(), la.float(), lt.float(), kld.float()

    @staticmethod
    def backward(ctx, g_total, g_la, g_lt, g_kld):
        ra, a, rt, t, mu, lv = ctx.saved_tensors
        w_text, beta, mean_mode, na, nt, nl = ctx.cfg
        dev = ra.device
        z = torch.zeros((), device=dev)
        gT = g_total if g_total is not None else z
        gA = g_la if g_la is not None else z
        gX = g_lt if g_lt is not None else z
        gK = g_kld if g_kld is not None else z
        if mean_mode:  # d mean-MSE = 2 (r - x) / n ; d mean-KL = (mu, -0.5 (1 - e^lv)) / nl
            coef = torch.stack([2.0 * (gT + gA) / na, 0.0 * gT, (beta * gT + gK) / nl]).float().contiguous()
        else:
            coef = torch.stack([2.0 * (gT + gA), 2.0 * (w_text * gT + gX), beta * gT + gK]).float().contiguous()
        dra = torch.empty_like(ra)
        drt = torch.empty_like(rt) if nt else None
        dmu = torch.empty_like(mu)
        dlv = torch.empty_like(lv)
        L.check(L.lib().hlmc_loss_backward(L.stream(), L.ptr(ra), L.ptr(a), na, L.ptr(dra), L.ptr(rt) if nt else None,
                                           L.ptr(t) if nt else None, nt, L.ptr(drt), L.ptr(mu), L.ptr(lv), nl,
                                           coef.data_ptr(), L.ptr(dmu), L.ptr(dlv)), "hlmc_loss_backward")
        return dra, None, drt, None, dmu, dlv, None, None, None


def _c(x):
    return None if x is None else x.float().contiguous()


def loss_function(recon_audio, audio, recon_text, text, mu, logvar, alpha=1.0, beta=1.0):
    """(total, recon_loss_audio, recon_loss_text, kld); text term omitted when recon_text is None (audio-only)."""
    return _LossFn.apply(_c(recon_audio), _c(audio), _c(recon_text), _c(text) if recon_text is not None else None,
                         _c(mu), _c(logvar), 350.0, float(beta), False)


def cvae_loss_function(recon_audio, x_audio, recon_text, x_text, mu, logvar, beta=1.0):
    """(total, mse_audio, mse_text, kld) with the reference's text weight 200."""
    return _LossFn.apply(_c(recon_audio), _c(x_audio), _c(recon_text), _c(x_text), _c(mu), _c(logvar), 200.0,
                         float(beta), False)


def vae_loss(reconstruction, x, mu, logvar, beta=1.0):
    """(total, recon_loss, kl_loss) with mean reductions."""
    total, la, _, kl = _LossFn.apply(_c(reconstruction), _c(x), None, None, _c(mu), _c(logvar), 0.0, float(beta), True)
    return total, la, kl
