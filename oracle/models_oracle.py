"""CPU oracle (TEST INFRASTRUCTURE ONLY) — torch-CPU restatement of the reference VAE classes.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use this.

Restates (same parameter registration order => same ``torch.manual_seed`` init and identical
``state_dict`` keys):
  * ``HybridVAE``  — src/Convolutional_VAE.py:75-185; ``loss_function`` — :187-194
  * ``ConditionalVAE`` — src/Conditional_VAE.py:109-231; ``cvae_loss_function`` — :233-246
  * ``SimpleAutoencoder`` — src/Conditional_VAE.py:252-273
  * ``VAE`` — src/Simple_VAE.py:47-105; ``vae_loss`` — :108-114
The only generalisation is the flatten width: F = 512*(H/64)*(W/64); at the
reference's 128x1024 input F = 16384 and the classes reduce exactly to the reference.
``audio_only=True`` defines BASELINE config[1]'s audio-only ConvVAE: the HybridVAE with the text
branch, its fusion slice and its loss term removed.
Pinned by tests/golden/*.npz produced from the AST-loaded reference classes (make_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn

ENC_CHANNELS = (1, 32, 64, 128, 256, 512, 512)
DEC_CHANNELS = (512, 512, 256, 128, 64, 32, 1)


def flat_dims(input_hw=(128, 1024)):
    h, w = input_hw
    assert h % 64 == 0 and w % 64 == 0, "six stride-2 convs need H, W divisible by 64"
    return 512 * (h // 64) * (w // 64), (512, h // 64, w // 64)


def _conv_encoder() -> nn.Sequential:
    mods = []
    for cin, cout in zip(ENC_CHANNELS[:-1], ENC_CHANNELS[1:]):
        mods += [nn.Conv2d(cin, cout, kernel_size=3, stride=2, padding=1), nn.BatchNorm2d(cout), nn.LeakyReLU()]
    mods.append(nn.Flatten())
    return nn.Sequential(*mods)


def _convT_stack(with_unflatten=None) -> nn.Sequential:
    mods = [] if with_unflatten is None else [nn.Unflatten(1, with_unflatten)]
    pairs = list(zip(DEC_CHANNELS[:-1], DEC_CHANNELS[1:]))
    for i, (cin, cout) in enumerate(pairs):
        mods.append(nn.ConvTranspose2d(cin, cout, kernel_size=3, stride=2, padding=1, output_padding=1))
        if i + 1 < len(pairs):
            mods += [nn.BatchNorm2d(cout), nn.LeakyReLU()]
    return nn.Sequential(*mods)


def _mlp_bn_lrelu(dims) -> nn.Sequential:
    mods = []
    for a, b in zip(dims[:-1], dims[1:]):
        mods += [nn.Linear(a, b), nn.BatchNorm1d(b), nn.LeakyReLU()]
    return nn.Sequential(*mods)


class HybridVAE(nn.Module):
    def __init__(self, latent_dim=128, text_dim=768, input_hw=(128, 1024), audio_only=False):
        super().__init__()
        self.latent_dim = latent_dim
        self.audio_only = audio_only
        self.flat, self.unflat = flat_dims(input_hw)
        t_lat = 0 if audio_only else 128
        self.audio_encoder = _conv_encoder()
        self.audio_fc = nn.Linear(self.flat, 1024)
        if not audio_only:
            self.text_encoder = _mlp_bn_lrelu((text_dim, 256, 128))
        self.fc_fusion = nn.Linear(1024 + t_lat, 512)
        self.fc_mu = nn.Linear(512, latent_dim)
        self.fc_logvar = nn.Linear(512, latent_dim)
        self.decoder_input = nn.Linear(latent_dim, 512)
        self.decoder_split = nn.Linear(512, 1024 + t_lat)
        self.audio_decoder_fc = nn.Linear(1024, self.flat)
        self.audio_decoder = _convT_stack(with_unflatten=self.unflat)
        if not audio_only:
            self.text_decoder = nn.Sequential(nn.Linear(128, 256), nn.BatchNorm1d(256), nn.LeakyReLU(),
                                              nn.Linear(256, text_dim))

    def encode(self, audio, text=None):
        a = self.audio_fc(self.audio_encoder(audio))
        if not self.audio_only:
            a = torch.cat((a, self.text_encoder(text)), dim=1)
        h = torch.relu(self.fc_fusion(a))
        return self.fc_mu(h), self.fc_logvar(h)

    def reparameterize(self, mu, logvar, eps=None):
        std = torch.exp(0.5 * logvar)
        if eps is None:
            eps = torch.randn_like(std)
        return mu + eps * std

    def decode(self, z):
        s = torch.relu(self.decoder_split(torch.relu(self.decoder_input(z))))
        recon_audio = self.audio_decoder(torch.relu(self.audio_decoder_fc(s[:, :1024])))
        recon_text = None if self.audio_only else self.text_decoder(s[:, 1024:])
        return recon_audio, recon_text

    def forward(self, audio, text=None, eps=None):
        mu, logvar = self.encode(audio, text)
        ra, rt = self.decode(self.reparameterize(mu, logvar, eps))
        return ra, rt, mu, logvar


def kld_sum(mu, logvar):
    return -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())


def loss_function(recon_audio, audio, recon_text, text, mu, logvar, alpha=1.0, beta=1.0):
    """src/Convolutional_VAE.py:187-194 (alpha unused there too). Text term dropped when recon_text is None."""
    la = nn.functional.mse_loss(recon_audio, audio, reduction="sum")
    kld = kld_sum(mu, logvar)
    if recon_text is None:
        lt = torch.zeros((), dtype=la.dtype)
        return la + kld * beta, la, lt, kld
    lt = nn.functional.mse_loss(recon_text, text, reduction="sum")
    return la + lt * 350 + kld * beta, la, lt, kld


class ConditionalVAE(nn.Module):
    def __init__(self, latent_dim=64, text_dim=768, num_classes=10, input_hw=(128, 1024)):
        super().__init__()
        self.latent_dim = latent_dim
        self.flat, self.unflat = flat_dims(input_hw)
        self.audio_encoder = _conv_encoder()
        self.text_encoder = _mlp_bn_lrelu((text_dim, 256))
        fusion = self.flat + 256 + num_classes
        self.fc_mu = nn.Linear(fusion, latent_dim)
        self.fc_logvar = nn.Linear(fusion, latent_dim)
        self.decoder_fc = nn.Linear(latent_dim + num_classes, self.flat + 256)
        self.text_decoder = nn.Sequential(nn.Linear(256, 512), nn.BatchNorm1d(512), nn.LeakyReLU(),
                                          nn.Linear(512, text_dim))
        self.audio_unflatten = nn.Unflatten(1, self.unflat)
        self.audio_decoder = _convT_stack()

    def encode(self, audio, text, condition):
        c = torch.cat([self.audio_encoder(audio), self.text_encoder(text), condition], dim=1)
        return self.fc_mu(c), self.fc_logvar(c)

    def reparameterize(self, mu, logvar, eps=None):
        std = torch.exp(0.5 * logvar)
        if eps is None:
            eps = torch.randn_like(std)
        return mu + eps * std

    def decode(self, z, condition):
        s = self.decoder_fc(torch.cat([z, condition], dim=1))
        ra = self.audio_decoder(self.audio_unflatten(s[:, :self.flat]))
        return ra, self.text_decoder(s[:, self.flat:])

    def forward(self, audio, text, condition, eps=None):
        mu, logvar = self.encode(audio, text, condition)
        ra, rt = self.decode(self.reparameterize(mu, logvar, eps), condition)
        return ra, rt, mu, logvar


def cvae_loss_function(recon_audio, x_audio, recon_text, x_text, mu, logvar, beta=1.0):
    """src/Conditional_VAE.py:233-246."""
    ma = nn.functional.mse_loss(recon_audio, x_audio, reduction="sum")
    mt = nn.functional.mse_loss(recon_text, x_text, reduction="sum")
    kld = kld_sum(mu, logvar)
    return ma + mt * 200 + beta * kld, ma, mt, kld


class SimpleAutoencoder(nn.Module):
    """src/Conditional_VAE.py:252-273."""

    def __init__(self, input_dim, latent_dim=64):
        super().__init__()
        enc = [input_dim, 1024, 256, latent_dim]
        dec = enc[::-1]

        def chain(d):
            mods = []
            for i, (a, b) in enumerate(zip(d[:-1], d[1:])):
                mods.append(nn.Linear(a, b))
                if i + 2 < len(d):
                    mods.append(nn.ReLU())
            return nn.Sequential(*mods)

        self.encoder = chain(enc)
        self.decoder = chain(dec)

    def forward(self, x):
        z = self.encoder(x)
        return self.decoder(z), z


class VAE(nn.Module):
    """src/Simple_VAE.py:47-105 (MLP VAE with Linear-BN1d-ReLU-Dropout(0.2) blocks)."""

    def __init__(self, input_dim, hidden_dims=(512, 256, 128), latent_dim=64):
        super().__init__()
        hidden_dims = list(hidden_dims)
        self.input_dim, self.latent_dim = input_dim, latent_dim

        def blocks(dims):
            mods = []
            for a, b in zip(dims[:-1], dims[1:]):
                mods += [nn.Linear(a, b), nn.BatchNorm1d(b), nn.ReLU(), nn.Dropout(0.2)]
            return mods

        self.encoder = nn.Sequential(*blocks([input_dim] + hidden_dims))
        self.fc_mu = nn.Linear(hidden_dims[-1], latent_dim)
        self.fc_logvar = nn.Linear(hidden_dims[-1], latent_dim)
        rev = hidden_dims[::-1]
        self.decoder = nn.Sequential(*blocks([latent_dim] + rev), nn.Linear(rev[-1], input_dim))

    def encode(self, x):
        h = self.encoder(x)
        return self.fc_mu(h), self.fc_logvar(h)

    def reparameterize(self, mu, logvar, eps=None):
        std = torch.exp(0.5 * logvar)
        if eps is None:
            eps = torch.randn_like(std)
        return mu + eps * std

    def decode(self, z):
        return self.decoder(z)

    def forward(self, x, eps=None):
        mu, logvar = self.encode(x)
        z = self.reparameterize(mu, logvar, eps)
        return self.decode(z), mu, logvar, z

    def get_latent_features(self, x):
        return self.encode(x)[0]


def vae_loss(reconstruction, x, mu, logvar, beta=1.0):
    """src/Simple_VAE.py:108-114 (mean reductions)."""
    r = nn.functional.mse_loss(reconstruction, x, reduction="mean")
    kl = -0.5 * torch.mean(1 + logvar - mu.pow(2) - logvar.exp())
    return r + beta * kl, r, kl
