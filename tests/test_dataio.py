"""Mel PNG quantisation and the spectrogram folder / pair datasets.

CPU: the numpy quantisation equals an independent float32 restatement of audio_processor.py:55-73
(bit-exact, boundaries included); the folder listing, transform and pairing CSV on a synthetic PNG tree
(the RandomState(42) sequence of dataset.py:262-299 restated); the pair item structure.  GPU: the HIP
kernels (dataio.hip) bit-exact against the numpy forms, and the device batch path equal to the
ToTensor items.  (torchvision / librosa are absent here: parity is pinned by these restatements,
not by running the reference's dataset module.)
"""
import csv
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "music-style-transfer-ldm_amd")


def _db_values():
    g = np.random.Generator(np.random.PCG64(3))
    v = g.uniform(-100, 20, 4097).astype(np.float32)
    edges = np.array([-80, -79.99, -80.2, 0, 0.1, -0.0, 1e-7, -40.0, -40.078431, 80, 1e6, -1e6], dtype=np.float32)
    return np.concatenate([v, edges])


def _ref_quant(s, max_db=80):
    s = s.astype(np.float32)
    out = np.empty(s.shape, dtype=np.uint8)
    for i, x in enumerate(s):
        y = np.float32(x) + np.float32(max_db)
        y = np.float32(y * np.float32(255.0 / max_db))
        y = min(max(y, np.float32(0)), np.float32(255))
        out[i] = int(np.float32(y + np.float32(0.5)))
    return out


def test_quantize_numpy_matches_restatement():
    sys.path.insert(0, PKG)
    from data.audio_processor import AudioPreprocessor
    v = _db_values()
    q = AudioPreprocessor.quantize(v)
    assert q.dtype == np.uint8
    assert np.array_equal(q, _ref_quant(v))
    d = AudioPreprocessor.dequantize(q)
    assert d.dtype == np.float32
    assert np.array_equal(d, q.astype(np.float32) * np.float32(80 / 255.0) - np.float32(80))


def _make_tree(tmp_path, n_per=(3, 2, 4)):
    from PIL import Image
    g = np.random.Generator(np.random.PCG64(9))
    root = tmp_path / "spectrograms"
    for k, n in enumerate(n_per):
        d = root / f"label{k}"
        d.mkdir(parents=True)
        for i in range(n):
            Image.fromarray(g.integers(0, 256, (130, 140), dtype=np.uint8)).save(d / f"s{i:02d}.png")
        (d / "notes.txt").write_text("ignored")
    return root


def test_folder_listing_transform_and_pairs(tmp_path):
    sys.path.insert(0, PKG)
    from PIL import Image
    from models.dataset import ImageFolderNoSubdirs, SpectrogramPairDataset, SpectrogramTransform
    root = _make_tree(tmp_path)
    ds = ImageFolderNoSubdirs(str(root / "label1"), transform=SpectrogramTransform())
    assert ds.classes == ["label1"] and len(ds) == 2
    x, y = ds[1]
    px = np.array(Image.open(root / "label1" / "s01.png"))[:128, :128]
    assert x.shape == (1, 128, 128) and x.dtype == torch.float32 and y == 0
    assert torch.equal(x[0], torch.from_numpy(px).float().div(255))
    top = ImageFolderNoSubdirs(str(root))
    assert top.classes == ["label0", "label1", "label2"] and len(top) == 9
    # the reference's pairing sequence, restated
    out = tmp_path / "pairs.csv"
    SpectrogramPairDataset.generate_pairings(str(root), str(out), num_pairs=25)
    rng = np.random.RandomState(42)
    labels, sizes = ["label0", "label1", "label2"], {"label0": 3, "label1": 2, "label2": 4}
    want = []
    for _ in range(25):
        a, b = rng.choice(labels, size=2, replace=False)
        want.append([str(a), str(rng.randint(0, sizes[a])), str(b), str(rng.randint(0, sizes[b]))])
    assert list(csv.reader(open(out))) == want
    pds = SpectrogramPairDataset(str(root), str(out))
    (i1, l1), (i2, l2) = pds[3]
    assert (l1, l2) == (want[3][0], want[3][2]) and i1.shape == i2.shape == (1, 128, 128)


@pytest.mark.gpu
def test_dataio_kernels_bitexact(cuda):
    from ldm_amd import ops
    v = _db_values()
    for n in (v.size, 7, 1):
        q = ops.mel_quantize(torch.from_numpy(v[:n]).to(cuda))
        assert np.array_equal(q.cpu().numpy(), _ref_quant(v[:n]))
    q = ops.mel_quantize(torch.from_numpy(v[1:]).to(cuda))          # unaligned start
    assert np.array_equal(q.cpu().numpy(), _ref_quant(v[1:]))
    px = torch.from_numpy(_ref_quant(v)).to(cuda)
    d = ops.mel_dequantize(px)
    assert np.array_equal(d.cpu().numpy(), px.cpu().numpy().astype(np.float32) * np.float32(80 / 255.0) - np.float32(80))
    u = ops.u8_to_unit(px)
    assert torch.equal(u.cpu(), px.cpu().float().div(255))


@pytest.mark.gpu
def test_device_batches_equal_items(cuda, tmp_path):
    sys.path.insert(0, PKG)
    from models.dataset import ImageFolderNoSubdirs, SpectrogramTransform, to_device
    root = _make_tree(tmp_path)
    ref = ImageFolderNoSubdirs(str(root), transform=SpectrogramTransform())
    raw = ImageFolderNoSubdirs(str(root), transform=SpectrogramTransform(raw=True))
    batch = torch.stack([raw[i][0] for i in range(len(raw))])
    dev = to_device(batch, cuda)
    assert torch.equal(dev.cpu(), torch.stack([ref[i][0] for i in range(len(ref))]))
