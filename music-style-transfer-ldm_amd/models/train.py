"""Drop-in for the reference's models/train.py: LDMTrainer (train_step / train_epoch / train),
train_autoencoder, train_ldm, main — same signatures, defaults, loss composition, optimiser and
GradScaler semantics, with forward, backward and optimiser step on libldm_amd.

Differences from the reference, all deliberate:
  * The "GPU or raise" check runs when an entry point is used, not at import (train.py:21-26), so the
    API can be imported and inspected on a host without a GPU.
  * torch.optim.Adam / AdamW are ldm_amd.optim.Adam / AdamW (same update, one fused multi-tensor HIP
    launch per group); torch.amp.GradScaler is ldm_amd.optim.GradScaler (same scale / skip / growth
    rules).  Both are torch.optim-compatible (ReduceLROnPlateau and state_dicts work unchanged).
  * The forward runs inside torch.autocast like the reference (train.py:176); inside it the HIP
    convolutions round their operands to the region's dtype (fp16 by default on a GPU, bf16 with
    autocast_dtype) and accumulate in fp32.  autocast_enabled = False runs the step in fp32.
  * Data-parallel: when torch.distributed is initialised with world_size > 1, each rank trains on its
    own batch shard and the gradients are all-reduced (bucketed, overlapped with backward) before the
    optimiser step (ldm_amd.dist.GradAllReduce); over RCCL the graphed step captures those collectives.
    Single-process behaviour is unchanged.
  * The datasets (dataset.py) are not part of this package (torchvision-based image folders, out of
    scope for the hot path); train_autoencoder / train_ldm accept ready loaders, else they import the
    reference-style `dataset` module from sys.path.
"""
import argparse
import os
from collections.abc import Mapping

import torch

try:
    from .config import config
    from . import _pathfix  # noqa: F401
    from .model import LDM, SpectrogramDecoder, SpectrogramEncoder
    from .loss import VGGishFeatureLoss, compression_loss, diffusion_loss, is_const_zero, style_loss
except ImportError:   # reference-style flat imports (models/ on sys.path)
    from config import config
    import _pathfix  # noqa: F401
    from model import LDM, SpectrogramDecoder, SpectrogramEncoder
    from loss import VGGishFeatureLoss, compression_loss, diffusion_loss, is_const_zero, style_loss

from ldm_amd import dist as hdist
from ldm_amd import functional as hF
from ldm_amd import graphs as hgraphs
from ldm_amd import ops
from ldm_amd import optim as hoptim


def _require_gpu():
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if device.type == "cuda":
        print("Using GPU")
    else:
        raise RuntimeError("GPU not available, please check your setup.")
    return device


def _prepare_loaders(cfg):
    try:
        import dataset  # reference-style module on sys.path
    except ImportError as e:
        raise RuntimeError("train: no data loader given and no `dataset` module importable "
                           f"({e}); pass train_loader= explicitly") from e
    return dataset


# ------------------------------------------------------------------------------------------------
def autoencoder_step(encoder, decoder, optimizer, spectrogram, feature_extractor, reducer=None):
    """One inner iteration of train_autoencoder (reference train.py:69-82): encode -> decode ->
    compression_loss -> zero_grad -> backward (-> data-parallel gradient all-reduce) -> AdamW step.
    Returns the loss tensor (the caller's .item() is the reference's host sync)."""
    latent = encoder(spectrogram)
    reconstructed = decoder(latent)
    loss = compression_loss(spectrogram, reconstructed, latent, feature_extractor)
    optimizer.zero_grad()
    loss.backward()
    if reducer is not None:
        reducer.finish()
    optimizer.step()
    return loss


def train_autoencoder(config, train_loader=None, test_loader=None, device=None):
    """VAE pre-training (reference train.py:28-138): encoder+decoder, AdamW, ReduceLROnPlateau,
    compression_loss with the configured feature extractor, best-val checkpointing."""
    device = device or _require_gpu()
    encoder = SpectrogramEncoder(config["latent_dim_encoder"]).to(device)
    decoder = SpectrogramDecoder(config["latent_dim_encoder"]).to(device)
    feature_extractor = VGGishFeatureLoss().to(device)
    optimizer = hoptim.AdamW(list(encoder.parameters()) + list(decoder.parameters()), lr=config["learning_rate"])
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(
        optimizer, mode="min", factor=config["learning_rate_factor"], patience=config["learning_rate_patience"],
        min_lr=config["learning_rate_min"])
    if train_loader is None:
        train_loader, test_loader = _prepare_loaders(config).prepare_dataset(config)
    reducer = None
    if hdist.world_size() > 1:
        hdist.broadcast_parameters(encoder)
        hdist.broadcast_parameters(decoder)
        reducer = hdist.GradAllReduce(list(encoder.parameters()) + list(decoder.parameters()), average=True)

    num_epochs = config["num_epochs"]
    train_losses, val_losses = [], []
    best_val_loss = float("inf")
    os.makedirs("models/pretrained", exist_ok=True)
    for epoch in range(num_epochs):
        running = 0.0
        encoder.train()
        decoder.train()
        for spectrogram in train_loader:
            spectrogram = spectrogram[0].to(device)
            loss = autoencoder_step(encoder, decoder, optimizer, spectrogram, feature_extractor, reducer)
            running += loss.item()
        avg_train = running / max(1, len(train_loader))
        train_losses.append(avg_train)

        encoder.eval()
        decoder.eval()
        running_val = 0.0
        n_val = 0
        with torch.no_grad():
            for spectrogram in (test_loader or []):
                spectrogram = spectrogram[0].to(device)
                latent = encoder(spectrogram)
                reconstructed = decoder(latent)
                running_val += compression_loss(spectrogram, reconstructed, latent, feature_extractor).item()
                n_val += 1
        avg_val = running_val / max(1, n_val)
        val_losses.append(avg_val)
        scheduler.step(avg_val)
        if avg_val < best_val_loss and hdist.rank() == 0:
            best_val_loss = avg_val
            torch.save(encoder.state_dict(), "models/pretrained/encoder.pth")
            torch.save(decoder.state_dict(), "models/pretrained/decoder.pth")
        print(f"Epoch: {epoch}")
        print(f"Average Train Loss: {avg_train:.6f}")
        print(f"Average Val Loss: {avg_val:.6f}")
        print(f"Learning Rate: {optimizer.param_groups[0]['lr']:.6f}")
    if hdist.rank() == 0:
        torch.save(encoder.state_dict(), "models/pretrained/encoder.pth")
        torch.save(decoder.state_dict(), "models/pretrained/decoder.pth")
    return train_losses, val_losses


# ------------------------------------------------------------------------------------------------
class StepLosses(Mapping):
    """{"compression_loss", "denoisinsg_loss", "style_loss", "total_loss"} -> float, the fp32 values .item() would
    return, read from a pinned copy issued when the step was queued; the first access waits for that copy."""
    KEYS = ("compression_loss", "denoisinsg_loss", "style_loss", "total_loss")

    def __init__(self, vec):
        self._host = torch.empty(vec.shape, dtype=vec.dtype, pin_memory=True)
        self._host.copy_(vec, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()
        self._vals = None

    def _values(self):
        if self._vals is None:
            self._event.synchronize()
            self._vals = dict(zip(self.KEYS, self._host.tolist()))
        return self._vals

    def __getitem__(self, k):
        return self._values()[k]

    def __iter__(self):
        return iter(self.KEYS)

    def __len__(self):
        return len(self.KEYS)

    def __repr__(self):
        return repr(self._values())


class LDMTrainer:
    """Reference train.py:140-293."""

    def __init__(self, model, train_loader, device, lr=1e-4, style_loss_weight=0.1):
        self.model = model.to(device)
        self.train_loader = train_loader
        self.device = torch.device(device) if not isinstance(device, torch.device) else device
        self.style_loss_weight = style_loss_weight
        trainable_params = [p for p in model.parameters() if p.requires_grad]
        self._trainable = trainable_params
        self.optimizer = hoptim.Adam(trainable_params, lr=lr)
        self.scaler = hoptim.GradScaler("cuda")
        # dtype of the train step's autocast region (train.py:174 uses the device default: fp16 on a GPU;
        # bfloat16 = BASELINE config 3); the HIP convs then round their operands to it (ldm_capi.h LDM_DT_*)
        self.autocast_dtype = None
        self.autocast_enabled = True
        # graph_step = True: after graph_warmup eager steps, the whole step (forward, backward, unscale,
        # optimizer, scaler update) is captured once into a hipGraph and replayed; the loss values are read
        # after each replay.  Data-parallel over RCCL the capture holds the bucketed gradient all-reduces
        # (launched from the backward's hooks, joined before the optimizer) and SyncBN's statistic
        # all-reduces too; over gloo (host-staged collectives) the step stays eager.
        self.graph_step = False
        self.graph_warmup = 2
        # batched_repack: the packed (MFMA fragment-order) copies of the trainable conv weights are refreshed
        # by one launch right after the optimizer step (ops.PackSet, recorded on the first eager step) instead
        # of one launch per weight at its first use in the next step; LDM_AMD_BATCHED_REPACK=0 turns it off
        self.batched_repack = os.environ.get("LDM_AMD_BATCHED_REPACK", "1") != "0"
        self._packset = None
        self._packset_tried = False
        self._graph = None
        self._graph_calls = 0
        self.scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, mode="min", factor=0.5,
                                                                    patience=10)
        self.reducer = None
        if hdist.world_size() > 1:
            hdist.broadcast_parameters(self.model)
            hdist.convert_sync_batchnorm(self.model)      # global-batch BN statistics
            self.reducer = hdist.GradAllReduce(trainable_params)
            self.scaler.set_grad_divisor(hdist.world_size())

    def _sample_t(self, batch_size):
        return torch.randint(0, self.model.num_timesteps, (batch_size,), device=self.device)

    def train_step(self, content_spec, style_spec, t=None, noise=None):
        """One step (reference train.py:163-208).  t / noise may be injected (parity tests); by default
        they are drawn like the reference (randint on the device; randn_like inside the scheduler)."""
        if self.graph_step and self.device.type == "cuda" and (self.reducer is None or self.reducer.capturable):
            return self._graphed_step(content_spec, style_spec, t, noise)
        return self._losses(self._loss_vec(self._step(content_spec, style_spec, t, noise)))

    def _step(self, content_spec, style_spec, t, noise):
        """The step's device work; returns the four loss tensors (no host synchronisation)."""
        self.optimizer.zero_grad()
        content_spec = content_spec.float()
        style_spec = style_spec.float()
        batch_size = content_spec.shape[0]
        if t is None:
            t = self._sample_t(batch_size)
        ac = {} if self.autocast_dtype is None else {"dtype": self.autocast_dtype}
        record = rec = None
        if self.batched_repack and not self._packset_tried and self.device.type == "cuda" and \
                not torch.cuda.is_current_stream_capturing():
            record = ops.record_packs()
            rec = record.__enter__()
        try:
            return self._step_body(content_spec, style_spec, t, noise, ac, rec)
        finally:
            if record is not None:
                record.__exit__(None, None, None)

    def _step_body(self, content_spec, style_spec, t, noise, ac, rec):
        with torch.autocast(device_type=self.device.type, enabled=self.autocast_enabled, **ac):
            with hF.bn_counts_deferred():   # the BN layers' num_batches_tracked: one add launch, not five
                outputs = self.model(content_spec, style_spec, t, noise=noise)
            noise_pred = outputs["noise_pred"]
            noise = outputs["noise"]
            z_0 = outputs["z_0"]
            reconstructed = outputs["reconstructed"]
            denoisinsg_loss = diffusion_loss(noise_pred, noise)
            compression_loss_ = compression_loss(content_spec, reconstructed, z_0, self.model.feature_loss_net)
            style_loss_ = style_loss(reconstructed, style_spec, self.model.feature_loss_net)
            if is_const_zero(style_loss_):   # no VGGish weights offline: + w * 0 adds nothing
                total_loss = compression_loss_ + denoisinsg_loss
            else:
                total_loss = compression_loss_ + denoisinsg_loss + self.style_loss_weight * style_loss_
        # the step's reconstruction (a static buffer of the graph when the step is replayed): for callers that
        # inspect the step's output, e.g. the parity tests; nothing in the step reads it
        self.last_outputs = {"reconstructed": reconstructed.detach()}
        # the convs' bias-gradient finalizes as one launch after the backward (no all-reduce hook reads them early)
        with ops.bias_grads_deferred(enabled=self.reducer is None and os.environ.get("LDM_AMD_DEFER_BIAS", "1") != "0"):
            self.scaler.scale(total_loss).backward()
        if self.reducer is not None:
            self.reducer.finish()
        self.scaler.step(self.optimizer)
        self.scaler.update()
        if rec is not None:
            self._packset_tried = True
            self._packset = ops.PackSet(rec, self.device) if rec.entries else None
        if self._packset is not None:
            self._packset.repack()
        return compression_loss_, denoisinsg_loss, style_loss_, total_loss

    @staticmethod
    def _loss_vec(t4):
        """The four 0-d losses stacked on the device (inside the graph when the step is replayed), so the host
        reads them with one device-to-host copy and one synchronisation per step instead of four .item()s."""
        return torch.stack([t.detach().reshape(()).float() for t in t4])

    @staticmethod
    def _losses(vec):
        """The step's four losses as the reference's dict of Python floats (train.py:203-208).  On the GPU the values
        come back through an asynchronous copy (StepLosses): the host waits for it only when a value is read, so a
        loop of steps that reads them later (or not at all) queues its steps on the device back to back."""
        if vec.device.type != "cuda":
            return dict(zip(StepLosses.KEYS, vec.tolist()))
        return StepLosses(vec)

    def _graphed_step(self, content_spec, style_spec, t, noise):
        """train_step as one hipGraph replay.  The optimizer runs its capturable form (device step count,
        device-side inf/nan skip: ldm_adam_step_dev), so nothing in the step reads the device from the host;
        t / noise are drawn inside the graph (torch's graph-safe Philox offsets) unless injected, in which
        case every later call must inject them too (they are copied into the captured input buffers)."""
        self.optimizer.capturable = True
        args = (content_spec, style_spec, t, noise)
        # host scalars the capture bakes into the graph (the optimizer's hyper-parameters: ReduceLROnPlateau
        # moves lr between epochs; the style-loss weight): a change re-captures
        hyper = tuple((g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]) for g in self.optimizer.param_groups)
        sig = tuple(None if a is None else (tuple(a.shape), a.dtype) for a in args) + (
            hyper, self.style_loss_weight, self.autocast_enabled, self.autocast_dtype,
            getattr(self.optimizer, "state_epoch", 0))
        if self._graph is None or self._graph_sig != sig:
            if self._graph_calls < self.graph_warmup:
                self._graph_calls += 1
                return self._losses(self._loss_vec(self._step(*args)))
            static = [None if a is None else a.detach().clone() for a in args]
            if self._graph is not None:
                hoptim.release_captured(self._graph_tables)
                self._graph = None
            tables = hoptim.reserve_capture_buffers(device=self.device)
            # new versions for the capture: every weight pack of the step misses the version-keyed caches and
            # is recorded into the graph (a cache hit would bake a pack made outside it into every replay)
            for p in self._trainable:
                torch.autograd.graph.increment_version(p)
            if self._packset is not None:
                # ...except the batched re-pack's buffers: packed here, outside the graph, for the captured
                # forward to read; the graph re-packs them at its end (after the optimizer) for the next replay
                self._packset.repack()
            hgraphs.prepare_streams(self.device)    # the branch streams exist before the capture starts
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with hgraphs.capture(g):
                outs = self._loss_vec(self._step(*static))
            hoptim.fill_captured(tables)   # the optimizer's slot tables: filled once, outside the graph
            self._graph, self._graph_in, self._graph_out, self._graph_sig = g, static, outs, sig
            self._graph_tables = tables
        for dst, src in zip(self._graph_in, args):
            if dst is not None and (src.data_ptr() != dst.data_ptr() or src.shape != dst.shape):
                dst.copy_(src)      # (a caller that fills graph_inputs() in place passes them back: no copy)
        if self._packset is not None and not self._packset.current():
            self._packset.repack()     # the weights changed outside the graph since its last re-pack
        self._graph.replay()
        # the replay rewrote the parameters on the device, but their autograd versions moved only once, at
        # capture: move them again so that version-keyed caches (packed conv weights, the UNet engine's bound
        # weights) never serve pre-replay values to a later eager forward or to a re-capture
        for p in self._trainable:
            torch.autograd.graph.increment_version(p)
        if self._packset is not None:
            self._packset.rekey()      # the replay ended by re-packing them from the updated weights
        return self._losses(self._graph_out)

    def graph_inputs(self):
        """The captured step's static input buffers (content, style, t, noise; None until the graph exists or
        for an input drawn inside it).  A caller may fill them in place and pass them to train_step, which
        then skips the copy into them."""
        return None if self._graph is None else tuple(self._graph_in)

    def train_epoch(self, epoch):
        self.model.train()
        total_loss = total_compression = total_denoise = total_style = 0
        num_batches = len(self.train_loader)
        for batch_idx, element in enumerate(self.train_loader):
            (content_spec, content_label), (style_spec, style_label) = element
            content_spec = content_spec.to(self.device)
            style_spec = style_spec.to(self.device)
            losses = self.train_step(content_spec, style_spec)
            total_loss += losses["total_loss"]
            total_compression += losses["compression_loss"]
            total_denoise += losses["denoisinsg_loss"]
            total_style += losses["style_loss"]
        k = config["training_iteration_noise"]     # the reference's reporting multiplier (train.py:240-243)
        n = max(1, num_batches)
        return total_loss / n * k, total_compression / n * k, total_denoise / n * k, total_style / n * k

    def train(self, num_epochs):
        best_loss = float("inf")  # noqa: F841  (kept from the reference)
        train_losses, compression_losses, denoise_losses, style_losses = [], [], [], []
        for epoch in range(num_epochs):
            train_loss, comp, den, sty = self.train_epoch(epoch)
            print(f"Epoch {epoch}: Train Loss = {train_loss:.4f}")
            self.scheduler.step(train_loss)
            train_losses.append(train_loss)
            compression_losses.append(comp)
            denoise_losses.append(den)
            style_losses.append(sty)
            print(f"Compression Loss: {comp:.4f}")
            print(f"Denoisinsg Loss: {den:.4f}")
            print(f"Style Loss: {sty:.4f}")
            if epoch % 100 == 0 and hdist.rank() == 0:
                os.makedirs("models/pretrained", exist_ok=True)
                torch.save(self.model.state_dict(), f"models/pretrained/ldm_{epoch}.pth")
        return train_losses, compression_losses, denoise_losses, style_losses


def train_ldm(config, train_loader=None, device=None):
    """Reference train.py:296-316."""
    device = device or _require_gpu()
    model = LDM(latent_dim=config["latent_dim_encoder"], load_full_model=False).to(device)
    if train_loader is None:
        ds = _prepare_loaders(config)
        style_dataset = ds.SpectrogramPairDataset(config["processed_spectograms_dataset_folderpath"],
                                                  config["pairing_file_path"])
        train_dataset, _test = torch.utils.data.random_split(style_dataset, [0.8, 0.2])
        train_loader = torch.utils.data.DataLoader(train_dataset, batch_size=config["batch_size"], shuffle=True,
                                                   num_workers=0)
    trainer = LDMTrainer(model, train_loader, device, lr=config["learning_rate"],
                         style_loss_weight=config["style_loss_weight"])
    return trainer.train(config["num_epochs"])


def main():
    parser = argparse.ArgumentParser(description="Train models")
    parser.add_argument("--model", type=str, required=True, choices=["autoencoder", "ldm"],
                        help="Which model to train (autoencoder or ldm)")
    args = parser.parse_args()
    if args.model == "autoencoder":
        train_autoencoder(config)
    elif args.model == "ldm":
        train_ldm(config)


if __name__ == "__main__":
    main()
