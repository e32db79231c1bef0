"""Hyper-parameters of the latent-diffusion path: the reference's `config` dict (models/config.py:2-19),
same keys and values, so code written against `from config import config` runs unchanged.

Notes on keys this implementation reads:
  forward_diffusion_num_timesteps  T of the DDPM schedule (ForwardDiffusion default)
  latent_dim_encoder               VAE latent channels (32)
  unet_num_filters                 UNet width (64; the cross-attention dims 256/512 assume it)
  compression_feature_extractor    'lpips' -> LPIPS-alex perceptual term (needs user-supplied weights,
                                   see loss.set_perceptual_backend), 'vggish' -> VGGishFeatureLoss
  training_iteration_noise         multiplier applied to epoch-average losses (reporting only,
                                   reference train.py:240-243)
"""

_optimizer = dict(
    learning_rate=5e-4,
    learning_rate_factor=0.5,
    learning_rate_patience=5,
    learning_rate_min=1e-6,
)

_schedule = dict(
    num_epochs=202,
    batch_size=128,
)

_model = dict(
    style_loss_weight=3.0,
    latent_dim_encoder=32,
    unet_num_filters=64,
    forward_diffusion_num_timesteps=200,
    compression_feature_extractor="lpips",
    training_iteration_noise=50,
)

_paths = dict(
    data_dir="downloads/",
    processed_spectograms_dataset_folderpath="processed_images",
    pairing_file_path="spectrogram_pair_dataset_pairings.csv",
)

config = {**_optimizer, **_schedule, **_model, **_paths}
