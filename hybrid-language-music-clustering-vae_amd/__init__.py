"""hlmc_amd — MI355X-native hot path of Shahriar1638/Hybrid-Language-Music-Clustering-VAE.

Drop-in surface (reference names):
  HybridVAE, loss_function                     (src/Convolutional_VAE.py)
  ConditionalVAE, cvae_loss_function           (src/Conditional_VAE.py)
  VAE, vae_loss                                (src/Simple_VAE.py)
  melspectrogram, power_to_db, mfcc, extract_mel_spectrogram, mean_std_pool, StandardScaler
                                               (librosa / sklearn calls of src/1_preprocessing*.py)
  KMeans                                       (sklearn KMeans calls of the three model scripts)
  metrics.silhouette_score / davies_bouldin_score / calinski_harabasz_score / adjusted_rand_score /
  normalized_mutual_info_score / calculate_purity   (the sklearn.metrics evaluation calls)
  Adam                                         (torch.optim.Adam of the train loops)
  Trainer                                      (fused train step + RCCL data parallel)
  pipeline.run_pipeline                        (BASELINE config[4]: 30 s clips -> mel -> scaler -> ConvVAE train ->
                                                latents -> KMeans, resident in HBM)
All compute runs in libhlmc.so (hand-written HIP for gfx950); see include/hlmc.h.
"""
from . import _lib
from .cluster import KMeans
from .features import (SPECTRAL_FEATURES, StandardScaler, chroma_stft, extract_mel_spectrogram, extract_spectral_features,
                       mean_std_pool, mel_filterbank, melspectrogram, mfcc, power_to_db, rms, spectral_bandwidth,
                       spectral_centroid, spectral_rolloff, spectral_stats, zero_crossing_rate)
from . import metrics
from . import preprocess
from .losses import cvae_loss_function, loss_function, vae_loss
from .models import VAE, ConditionalVAE, HybridVAE
from .optim import Adam
from .train import GraphedStep, Trainer
from . import pipeline

__all__ = ["HybridVAE", "ConditionalVAE", "VAE", "loss_function", "cvae_loss_function", "vae_loss", "melspectrogram",
           "power_to_db", "mfcc", "extract_mel_spectrogram", "mean_std_pool", "mel_filterbank", "StandardScaler",
           "KMeans", "Adam", "Trainer", "GraphedStep", "metrics"]
