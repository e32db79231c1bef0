"""The reference's AudioPreprocessor (data/audio_processor.py): the 8-bit mel PNG format either side of
the path.

The quantisation (log-mel dB -> uint8 pixel, :55-73) and its inverse (:91-93) are kept bit-exact with
the reference's numpy float32 arithmetic; given a CUDA tensor they run as HIP kernels (dataio.hip),
given a numpy array they run the reference's numpy code.  Audio decoding, the mel filterbank and
Griffin-Lim are librosa calls in the reference; librosa is not installed here, so those methods raise
ImportError naming it (out of scope: off-path audio I/O).
"""
import os
import sys
from io import BytesIO

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _librosa():
    try:
        import librosa
    except ImportError as e:
        raise ImportError("AudioPreprocessor: this method needs librosa (audio decoding / mel filterbank / "
                          "Griffin-Lim), which is not installed") from e
    return librosa


def _is_cuda_tensor(x):
    try:
        import torch
    except ImportError:   # pragma: no cover
        return False
    return isinstance(x, torch.Tensor) and x.is_cuda


class AudioPreprocessor:
    def __init__(self, target_sr=22050):
        self.target_sr = target_sr

    def load_audio(self, filepath):
        return _librosa().load(filepath, sr=self.target_sr, mono=True)

    def trim_silence(self, audio, top_db=20):
        trimmed, _ = _librosa().effects.trim(audio, top_db=top_db)
        return trimmed

    def normalize_audio(self, audio):   # a TODO stub in the reference
        pass

    def get_mel_spectogram(self, audio, sr, n_mels=256):
        lr = _librosa()
        return lr.power_to_db(lr.feature.melspectrogram(y=audio, sr=sr, n_mels=n_mels), ref=np.max)

    @staticmethod
    def quantize(spectogram, max_db=80):
        """uint8 pixels of a log-mel dB array: clip((db + max_db) * 255/max_db, 0, 255) + 0.5, truncated.
        numpy in -> numpy out (the reference's arithmetic); CUDA tensor in -> CUDA uint8 tensor (HIP)."""
        if _is_cuda_tensor(spectogram):
            from ldm_amd import ops
            return ops.mel_quantize(spectogram, max_db)
        spectogram = np.asarray(spectogram, dtype=np.float32)
        spectogram = spectogram + max_db
        spectogram = spectogram * (255.0 / max_db)
        spectogram = np.clip(spectogram, 0, 255)
        return (spectogram + 0.5).astype(np.uint8)

    @staticmethod
    def dequantize(pixels, max_db=80):
        """log-mel dB of uint8 pixels: u8 * max_db/255 - max_db (the first half of :81-100)."""
        if _is_cuda_tensor(pixels):
            from ldm_amd import ops
            return ops.mel_dequantize(pixels, max_db)
        return np.asarray(pixels, dtype=np.uint8).astype(np.float32) * (max_db / 255.0) - max_db

    def mel_spectogram_to_grayscale_image(self, spectogram, max_db=80):
        from PIL import Image
        px = self.quantize(spectogram, max_db)
        if _is_cuda_tensor(px):
            px = px.cpu().numpy()
        return Image.fromarray(px)

    def get_raw_image_bytes(self, image):
        with BytesIO() as output:
            image.save(output, format="PNG")
            return output.getvalue()

    def grayscale_mel_spectogram_image_to_audio(self, image, sr, im_height, im_width, max_db=80):
        px = np.frombuffer(image.tobytes(), dtype=np.uint8).reshape(im_height, im_width)
        lr = _librosa()
        return lr.feature.inverse.mel_to_audio(lr.db_to_power(self.dequantize(px, max_db)), sr=sr)

    def get_spectogram(self, audio):
        lr = _librosa()
        return lr.amplitude_to_db(np.abs(lr.stft(audio)), ref=np.max)

    def spectogram_to_grayscale_image(self, spectogram, max_db=80):
        return self.mel_spectogram_to_grayscale_image(spectogram, max_db)
