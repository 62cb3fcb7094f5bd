"""Drop-in VAE classes: the reference's nn.Module surface, computed by the native HIP engine.

  HybridVAE       — src/Convolutional_VAE.py:75-185
  ConditionalVAE  — src/Conditional_VAE.py:109-231
  VAE             — src/Simple_VAE.py:47-105

Each class registers exactly the reference's submodules (same names, shapes, construction order),
so ``torch.manual_seed(s); Model(...)`` initialises bit-identical weights and ``state_dict`` files
are interchangeable with the reference.  The submodules only hold parameters and BatchNorm
buffers: ``forward`` runs one native call (``hlmc_net_forward``) and autograd's backward one
``hlmc_net_backward``; there is no eager-PyTorch fallback.

Generalisation: ``input_hw`` sets the mel grid (default (128, 1024) = the reference); the flatten
width is F = 512*(H/64)*(W/64).  ``compute_dtype`` chooses the activation / MFMA
operand type: "fp32" (exact-fp32 MFMA, the parity mode) or "bf16" (throughput mode, fp32 accumulate,
fp32 master weights and grads).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn

from . import _lib as L

ENC_CHANNELS = (1, 32, 64, 128, 256, 512, 512)
DEC_CHANNELS = (512, 512, 256, 128, 64, 32, 1)
_DTYPES = {"fp32": L.HLMC_F32, "float32": L.HLMC_F32, "bf16": L.HLMC_BF16, "bfloat16": L.HLMC_BF16}


def flat_dims(input_hw):
    h, w = input_hw
    if h % 64 or w % 64 or h < 64 or w < 64:
        raise ValueError("input_hw must be multiples of 64 (six stride-2 convolutions)")
    return 512 * (h // 64) * (w // 64), (512, h // 64, w // 64)


def _conv_encoder():
    mods = []
    for ci, co in zip(ENC_CHANNELS[:-1], ENC_CHANNELS[1:]):
        mods += [nn.Conv2d(ci, co, kernel_size=3, stride=2, padding=1), nn.BatchNorm2d(co), nn.LeakyReLU()]
    return nn.Sequential(*mods, nn.Flatten())


def _convT_decoder(unflatten=None):
    mods = [] if unflatten is None else [nn.Unflatten(1, unflatten)]
    pairs = list(zip(DEC_CHANNELS[:-1], DEC_CHANNELS[1:]))
    for i, (ci, co) in enumerate(pairs):
        mods.append(nn.ConvTranspose2d(ci, co, kernel_size=3, stride=2, padding=1, output_padding=1))
        if i + 1 < len(pairs):
            mods += [nn.BatchNorm2d(co), nn.LeakyReLU()]
    return nn.Sequential(*mods)


def _lin_bn_lrelu(dims):
    mods = []
    for a, b in zip(dims[:-1], dims[1:]):
        mods += [nn.Linear(a, b), nn.BatchNorm1d(b), nn.LeakyReLU()]
    return nn.Sequential(*mods)


# ----------------------------------------------------------------------------------------- native net
class NativeNet:
    """An ``hlmc_net`` handle bound to a module's parameters, grads and BatchNorm buffers."""

    def __init__(self, kind: int, cfg, dtype: int):
        self.kind, self.cfg, self.dtype = kind, list(cfg), dtype
        h = C.c_void_p()
        L.check(L.lib().hlmc_net_create(kind, L.i64_array(cfg), len(cfg), dtype, C.byref(h)), "hlmc_net_create")
        self.h = h
        self.n_params = L.lib().hlmc_net_num_params(h)
        self.n_bn = L.lib().hlmc_net_num_bn(h)
        self.param_specs = []
        for i in range(self.n_params):
            name = C.create_string_buffer(256)
            nd = C.c_int()
            shape = (C.c_int64 * 4)()
            L.check(L.lib().hlmc_net_param_info(h, i, name, 256, C.byref(nd), shape))
            self.param_specs.append((name.value.decode(), tuple(shape[k] for k in range(nd.value))))
        # reparameterisation noise drawn on the device when no eps is passed (hlmc_net_set_rng): the stream is
        # keyed by torch's current seed, so torch.manual_seed(s) before building a model fixes its noise as it
        # fixes torch.randn_like's in the reference (src/Convolutional_VAE.py:162-165)
        L.check(L.lib().hlmc_net_set_rng(h, torch.initial_seed() & 0xFFFFFFFFFFFFFFFF, 0), "hlmc_net_set_rng")
        self.state = None
        self._bound = None
        self._ws = {}

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and L._lib is not None:
                L.lib().hlmc_net_destroy(self.h)
        except Exception:
            pass

    def check_module(self, module: nn.Module):
        got = [(n, tuple(p.shape)) for n, p in module.named_parameters()]
        if got != self.param_specs:
            raise L.HLMCError(f"module parameters do not match the native layout:\n{got}\nvs\n{self.param_specs}")

    def workspace_bytes(self, batch: int) -> int:
        return int(L.lib().hlmc_net_workspace_bytes(self.h, batch))

    def bind(self, module: nn.Module, grads):
        params = list(module.parameters())
        bns = [m for m in module.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
        if len(bns) != self.n_bn:
            raise L.HLMCError("BatchNorm count mismatch")
        key = tuple(p.data_ptr() for p in params) + tuple(g.data_ptr() for g in grads) + tuple(
            b.running_mean.data_ptr() for b in bns)
        if key == self._bound:
            return
        dev = params[0].device
        if self.state is None or self.state.device != dev:
            self.state = torch.empty(max(1, int(L.lib().hlmc_net_state_bytes(self.h))), dtype=torch.uint8, device=dev)
        running = []
        for b in bns:
            running += [b.running_mean.data_ptr(), b.running_var.data_ptr()]
        nbt = [b.num_batches_tracked.data_ptr() for b in bns]
        L.check(L.lib().hlmc_net_bind(self.h, L.vp_array([p.data_ptr() for p in params]),
                                      L.vp_array([g.data_ptr() for g in grads]), L.vp_array(running),
                                      L.vp_array(nbt), self.state.data_ptr()), "hlmc_net_bind")
        self._bound = key

    def new_workspace(self, batch: int, device):
        return torch.empty(self.workspace_bytes(batch), dtype=torch.uint8, device=device)


class _NetFn(torch.autograd.Function):
    """forward = hlmc_net_forward, backward = hlmc_net_backward (grads of every parameter)."""

    @staticmethod
    def forward(ctx, owner, train, audio, text, cond, eps, dropout, *params):
        net = owner._native_net()
        B = audio.shape[0]
        dev = audio.device
        ws = net.new_workspace(B, dev)
        out = owner._alloc_outputs(B, dev)
        L.check(L.lib().hlmc_net_forward(net.h, L.stream(), B, int(train), L.ptr(audio), L.ptr(text), L.ptr(cond),
                                         L.ptr(eps), L.ptr(dropout), L.ptr(out["recon"]), L.ptr(out.get("recon_text")),
                                         L.ptr(out["mu"]), L.ptr(out["logvar"]), L.ptr(out.get("z")), ws.data_ptr()),
                "hlmc_net_forward")
        # the engine's backward re-reads audio (the first conv's weight gradient): keep it alive until then
        ctx.owner, ctx.ws, ctx.B, ctx.audio = owner, ws, B, audio
        ctx.has_text = "recon_text" in out
        ctx.shapes = {k: v.shape for k, v in out.items()}
        outs = [out["recon"], out.get("recon_text"), out["mu"], out["logvar"], out.get("z")]
        for o in outs:
            if o is None:
                continue
        ctx.mark_non_differentiable(*[o for o in [out.get("z")] if o is not None])
        return tuple(o if o is not None else torch.empty(0, device=dev) for o in outs)

    @staticmethod
    def backward(ctx, d_recon, d_rt, d_mu, d_lv, d_z):
        owner = ctx.owner
        net = owner._native_net()
        dev = ctx.ws.device

        def g(t, key):
            if t is None or t.numel() == 0:
                return torch.zeros(ctx.shapes[key], device=dev, dtype=torch.float32)
            return t.contiguous().float()

        d_recon = g(d_recon, "recon")
        d_mu = g(d_mu, "mu")
        d_lv = g(d_lv, "logvar")
        d_rt = g(d_rt, "recon_text") if ctx.has_text else None
        L.check(L.lib().hlmc_net_backward(net.h, L.stream(), ctx.B, L.ptr(d_recon), L.ptr(d_rt), L.ptr(d_mu),
                                          L.ptr(d_lv), ctx.ws.data_ptr()), "hlmc_net_backward")
        # autograd reads every gradient right away: no Adam-overlapped tail on this path
        L.check(L.lib().hlmc_net_settle(net.h, L.stream()), "hlmc_net_settle")
        ctx.ws = ctx.audio = None
        return (None, None, None, None, None, None, None, *owner._grad_views)


class _NativeModule(nn.Module):
    """Shared plumbing: lazily created native net, flat grad buffer, dtype selection."""

    _kind = -1

    def _native_cfg(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def _init_native(self, compute_dtype):
        if compute_dtype not in _DTYPES:
            raise ValueError(f"compute_dtype must be one of {sorted(_DTYPES)}")
        self.compute_dtype = compute_dtype
        self._net = None
        self._gflat = None
        self._grad_views = None

    def _native_net(self) -> NativeNet:
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise L.HLMCError(f"{type(self).__name__} runs on the MI355X engine: move it to a cuda device first")
        if self._net is None:
            self._net = NativeNet(self._kind, self._native_cfg(), _DTYPES[self.compute_dtype])
            self._net.check_module(self)
        if self._gflat is None or self._gflat.device != dev:
            n = sum(p.numel() for p in self.parameters())
            self._gflat = torch.zeros(n, dtype=torch.float32, device=dev)
            views, off = [], 0
            for p in self.parameters():
                views.append(self._gflat[off:off + p.numel()].view_as(p))
                off += p.numel()
            self._grad_views = views
        self._net.bind(self, self._grad_views)
        return self._net

    def _params(self):
        return list(self.parameters())

    def _flatten_bn_buffers(self):
        """Re-point every BatchNorm's running_mean / running_var at views of ONE flat fp32 tensor (values kept;
        state_dict keys and shapes unchanged), so the data-parallel Trainer broadcasts them in one collective.
        Returns the flat tensor."""
        bns = [m for m in self.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
        if not bns:
            return torch.zeros(0, device=next(self.parameters()).device)
        first = bns[0].running_mean
        flat = getattr(self, "_bn_flat", None)
        if flat is not None and first.data_ptr() == flat.data_ptr() and first.device == flat.device:
            return flat
        n = sum(2 * b.running_mean.numel() for b in bns)
        flat = torch.empty(n, dtype=torch.float32, device=first.device)
        off = 0
        for b in bns:
            for name in ("running_mean", "running_var"):
                t = getattr(b, name)
                v = flat[off:off + t.numel()]
                v.copy_(t)
                setattr(b, name, v)
                off += t.numel()
        self._bn_flat = flat
        return flat

    def get_rng_state(self):
        """(seed, offset) of the engine's Philox reparameterisation-noise stream (drawn when forward gets no eps).
        Not part of state_dict (whose keys stay the reference's); Trainer.state_dict carries it for resume."""
        seed, off = C.c_uint64(), C.c_uint64()
        L.check(L.lib().hlmc_net_get_rng(self._native_net().h, C.byref(seed), C.byref(off)), "hlmc_net_get_rng")
        return int(seed.value), int(off.value)

    def set_rng_state(self, state):
        seed, off = state
        L.check(L.lib().hlmc_net_set_rng(self._native_net().h, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                         int(off) & 0xFFFFFFFFFFFFFFFF), "hlmc_net_set_rng")

    def _run(self, audio, text=None, cond=None, eps=None, dropout=None):
        L.require_cuda(audio, text, cond, eps, dropout)
        if eps is None and audio.is_cuda and torch.cuda.is_current_stream_capturing():
            # under torch.cuda.graph capture the engine's host-side Philox offset would freeze into the graph (every
            # replay the same noise): draw it with torch's graph-safe generator instead, as Trainer does
            eps = torch.randn(audio.shape[0], self.latent_dim, device=audio.device)
        train = self.training
        return _NetFn.apply(self, train, audio, text, cond, eps, dropout, *self._params())

    def _encode_native(self, in0, in1=None, in2=None):
        net = self._native_net()
        L.require_cuda(in0, in1, in2)
        B = in0.shape[0]
        mu = torch.empty(B, self.latent_dim, device=in0.device)
        lv = torch.empty_like(mu)
        ws = net.new_workspace(B, in0.device)
        L.check(L.lib().hlmc_net_encode(net.h, L.stream(), B, int(self.training), L.ptr(in0), L.ptr(in1), L.ptr(in2),
                                        L.ptr(mu), L.ptr(lv), ws.data_ptr()), "hlmc_net_encode")
        return mu, lv

    def _decode_native(self, z, cond=None, dropout=None):
        """Decoder-only native call (hlmc_net_decode): inference entry, no autograd graph is recorded."""
        net = self._native_net()
        L.require_cuda(z, cond, dropout)
        z = z.detach().float().contiguous()
        B = z.shape[0]
        if z.dim() != 2 or z.shape[1] != self.latent_dim:
            raise ValueError(f"z must be [batch, {self.latent_dim}], got {tuple(z.shape)}")
        if self.training and B < 2:
            raise ValueError("BatchNorm in train mode needs batch >= 2 (call .eval() to decode one latent)")
        out = self._alloc_outputs(B, z.device)
        ws = net.new_workspace(B, z.device)
        c = None if cond is None else cond.detach().float().contiguous()
        L.check(L.lib().hlmc_net_decode(net.h, L.stream(), B, int(self.training), L.ptr(z), L.ptr(c), L.ptr(dropout),
                                        L.ptr(out["recon"]), L.ptr(out.get("recon_text")), ws.data_ptr()),
                "hlmc_net_decode")
        return out

    @staticmethod
    def reparameterize(mu, logvar, eps=None):
        """z = mu + eps * exp(0.5 logvar) (reference reparameterize; eps ~ N(0,1) when not given)."""
        std = torch.exp(0.5 * logvar)
        if eps is None:
            eps = torch.randn_like(std)
        return mu + eps * std


# ----------------------------------------------------------------------------------------- models
class HybridVAE(_NativeModule):
    """src/Convolutional_VAE.py:75-185.  audio_only=True: BASELINE config[1]'s audio-only ConvVAE
    (text branch, its fusion slice and its loss term removed)."""

    _kind = L.NET_HYBRID

    def __init__(self, latent_dim=128, text_dim=768, input_hw=(128, 1024), audio_only=False, compute_dtype="fp32"):
        super().__init__()
        self.latent_dim, self.text_dim, self.input_hw = latent_dim, text_dim, tuple(input_hw)
        self.audio_only = audio_only
        self.flat, self.unflat = flat_dims(input_hw)
        tl = 0 if audio_only else 128
        self.audio_encoder = _conv_encoder()
        self.audio_fc = nn.Linear(self.flat, 1024)
        if not audio_only:
            self.text_encoder = _lin_bn_lrelu((text_dim, 256, 128))
        self.fc_fusion = nn.Linear(1024 + tl, 512)
        self.fc_mu = nn.Linear(512, latent_dim)
        self.fc_logvar = nn.Linear(512, latent_dim)
        self.decoder_input = nn.Linear(latent_dim, 512)
        self.decoder_split = nn.Linear(512, 1024 + tl)
        self.audio_decoder_fc = nn.Linear(1024, self.flat)
        self.audio_decoder = _convT_decoder(self.unflat)
        if not audio_only:
            self.text_decoder = nn.Sequential(nn.Linear(128, 256), nn.BatchNorm1d(256), nn.LeakyReLU(),
                                              nn.Linear(256, text_dim))
        self._init_native(compute_dtype)

    def _native_cfg(self):
        return [self.latent_dim, 0 if self.audio_only else self.text_dim, self.input_hw[0], self.input_hw[1]]

    def _alloc_outputs(self, B, dev):
        H, W = self.input_hw
        out = {"recon": torch.empty(B, 1, H, W, device=dev), "mu": torch.empty(B, self.latent_dim, device=dev),
               "logvar": torch.empty(B, self.latent_dim, device=dev)}
        if not self.audio_only:
            out["recon_text"] = torch.empty(B, self.text_dim, device=dev)
        return out

    def encode(self, audio, text=None):
        """(mu, logvar) of the encoder (latent extraction, src/Convolutional_VAE.py:286-303)."""
        return self._encode_native(audio.contiguous(), None if self.audio_only else text.contiguous())

    def decode(self, z):
        """(recon_audio [B,1,H,W], recon_text [B,text_dim] or None when audio_only) — src/Convolutional_VAE.py:167-179.
        Inference entry: computed by the native decoder without recording an autograd graph."""
        out = self._decode_native(z)
        return out["recon"], out.get("recon_text")

    def forward(self, audio, text=None, eps=None):
        # eps None: drawn on the device by the engine (its Philox stream), as torch.randn_like(std) in the reference
        ra, rt, mu, lv, _ = self._run(audio.contiguous(), None if self.audio_only else text.contiguous(), None,
                                      None if eps is None else eps.contiguous())
        return ra, (None if self.audio_only else rt), mu, lv


class ConditionalVAE(_NativeModule):
    """src/Conditional_VAE.py:109-231."""

    _kind = L.NET_CVAE

    def __init__(self, latent_dim=64, text_dim=768, num_classes=10, input_hw=(128, 1024), compute_dtype="fp32"):
        super().__init__()
        self.latent_dim, self.text_dim, self.num_classes, self.input_hw = latent_dim, text_dim, num_classes, tuple(input_hw)
        self.flat, self.unflat = flat_dims(input_hw)
        self.audio_encoder = _conv_encoder()
        self.text_encoder = _lin_bn_lrelu((text_dim, 256))
        fusion = self.flat + 256 + num_classes
        self.fc_mu = nn.Linear(fusion, latent_dim)
        self.fc_logvar = nn.Linear(fusion, latent_dim)
        self.decoder_fc = nn.Linear(latent_dim + num_classes, self.flat + 256)
        self.text_decoder = nn.Sequential(nn.Linear(256, 512), nn.BatchNorm1d(512), nn.LeakyReLU(),
                                          nn.Linear(512, text_dim))
        self.audio_unflatten = nn.Unflatten(1, self.unflat)
        self.audio_decoder = _convT_decoder()
        self._init_native(compute_dtype)

    def _native_cfg(self):
        return [self.latent_dim, self.text_dim, self.num_classes, self.input_hw[0], self.input_hw[1]]

    def _alloc_outputs(self, B, dev):
        H, W = self.input_hw
        return {"recon": torch.empty(B, 1, H, W, device=dev), "recon_text": torch.empty(B, self.text_dim, device=dev),
                "mu": torch.empty(B, self.latent_dim, device=dev), "logvar": torch.empty(B, self.latent_dim, device=dev)}

    def encode(self, audio, text, condition):
        return self._encode_native(audio.contiguous(), text.contiguous(), condition.float().contiguous())

    def decode(self, z, condition):
        """(recon_audio, recon_text) from z and the one-hot condition — src/Conditional_VAE.py:206-225.
        Inference entry: computed by the native decoder without recording an autograd graph."""
        if condition.shape != (z.shape[0], self.num_classes):
            raise ValueError(f"condition must be [batch, {self.num_classes}], got {tuple(condition.shape)}")
        out = self._decode_native(z, condition)
        return out["recon"], out["recon_text"]

    def forward(self, audio, text, condition, eps=None):
        ra, rt, mu, lv, _ = self._run(audio.contiguous(), text.contiguous(), condition.float().contiguous(),
                                      None if eps is None else eps.contiguous())
        return ra, rt, mu, lv


class VAE(_NativeModule):
    """src/Simple_VAE.py:47-105: MLP VAE with Linear-BN1d-ReLU-Dropout(0.2) blocks."""

    _kind = L.NET_SIMPLE
    dropout_p = 0.2

    def __init__(self, input_dim, hidden_dims=(512, 256, 128), latent_dim=64, compute_dtype="fp32"):
        super().__init__()
        hidden_dims = list(hidden_dims)
        self.input_dim, self.hidden_dims, self.latent_dim = input_dim, hidden_dims, latent_dim

        def blocks(dims):
            mods = []
            for a, b in zip(dims[:-1], dims[1:]):
                mods += [nn.Linear(a, b), nn.BatchNorm1d(b), nn.ReLU(), nn.Dropout(self.dropout_p)]
            return mods

        self.encoder = nn.Sequential(*blocks([input_dim] + hidden_dims))
        self.fc_mu = nn.Linear(hidden_dims[-1], latent_dim)
        self.fc_logvar = nn.Linear(hidden_dims[-1], latent_dim)
        rev = hidden_dims[::-1]
        self.decoder = nn.Sequential(*blocks([latent_dim] + rev), nn.Linear(rev[-1], input_dim))
        self._init_native(compute_dtype)

    def _native_cfg(self):
        return [self.input_dim, self.latent_dim, len(self.hidden_dims), *self.hidden_dims]

    def _alloc_outputs(self, B, dev):
        return {"recon": torch.empty(B, self.input_dim, device=dev), "mu": torch.empty(B, self.latent_dim, device=dev),
                "logvar": torch.empty(B, self.latent_dim, device=dev), "z": torch.empty(B, self.latent_dim, device=dev)}

    def mask_widths(self):
        """Dropout keep-mask layout: encoder blocks then decoder blocks, [B, width] each (uint8)."""
        return self.hidden_dims + self.hidden_dims[::-1]

    def make_dropout_mask(self, batch, device, generator=None):
        n = batch * sum(self.mask_widths())
        return (torch.rand(n, device=device, generator=generator) >= self.dropout_p).to(torch.uint8)

    def encode(self, x):
        return self._encode_native(x.float().contiguous())

    def decode(self, z, dropout_mask=None):
        """self.decoder(z) — src/Simple_VAE.py:95-96.  In train mode the decoder's Dropout(0.2) layers apply
        `dropout_mask` (the forward's keep-mask layout, make_dropout_mask; drawn when None).  Inference entry:
        no autograd graph is recorded."""
        if self.training and dropout_mask is None:
            dropout_mask = self.make_dropout_mask(z.shape[0], z.device)
        return self._decode_native(z, None, dropout_mask if self.training else None)["recon"]

    def forward(self, x, eps=None, dropout_mask=None):
        B = x.shape[0]
        if self.training and dropout_mask is None:
            dropout_mask = self.make_dropout_mask(B, x.device)
        recon, _, mu, lv, z = self._run(x.float().contiguous(), None, None, None if eps is None else eps.contiguous(),
                                        dropout_mask if self.training else None)
        return recon, mu, lv, z

    def get_latent_features(self, x):
        return self.encode(x)[0]
