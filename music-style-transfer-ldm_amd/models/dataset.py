"""Spectrogram datasets of the reference (models/dataset.py): the 8-bit mel PNG folders and the
content/style pair loader, with the same class names, constructor arguments,
sample order, pairing CSV and item structure.

torchvision is not a dependency here: its three transform steps (dataset.py:250-260) are restated --
crop to (0, 0, 128, 128), PIL convert("L") (the ITU-R 601 luma of the RGB image ImageFolder's loader
makes, exact for grayscale PNGs), and ToTensor (uint8 / 255 in fp32).  Items are CPU tensors like the
reference's; `to_device` turns a uint8 batch into the model's [0,1] fp32 input on the GPU in one HIP
launch (dataio.hip ldm_u8_to_unit), which is what `raw=True` datasets feed.
"""
import csv
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

try:
    from .config import config  # noqa: F401
    from . import _pathfix  # noqa: F401
except ImportError:   # reference-style flat imports (models/ on sys.path)
    from config import config  # noqa: F401
    import _pathfix  # noqa: F401

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")   # torchvision's


def _pil():
    try:
        from PIL import Image
    except ImportError as e:   # pragma: no cover - PIL ships with this image
        raise ImportError("models.dataset needs PIL to read spectrogram PNGs") from e
    return Image


def pil_loader(path):
    """torchvision's default loader: the image converted to RGB."""
    Image = _pil()
    with open(path, "rb") as f:
        img = Image.open(f)
        return img.convert("RGB")


class SpectrogramTransform:
    """crop((0, 0, 128, 128)) -> Grayscale -> ToTensor (dataset.py:252-260).  raw=True stops before
    ToTensor and returns the uint8 pixels [1, 128, 128] (for `to_device`)."""

    def __init__(self, size=128, raw=False):
        self.size = size
        self.raw = raw

    def __call__(self, img):
        img = img.crop((0, 0, self.size, self.size)).convert("L")
        px = torch.from_numpy(np.array(img, dtype=np.uint8, copy=True))[None]
        if self.raw:
            return px
        return px.to(torch.float32).div(255)   # ToTensor: uint8 / 255, fp32


def to_device(u8_batch, device):
    """[B,1,H,W] uint8 pixels -> the model's [0,1] fp32 input on `device` (one HIP launch)."""
    from ldm_amd import ops
    return ops.u8_to_unit(u8_batch.to(device, non_blocking=True))


class ImageFolderNoSubdirs(Dataset):
    """ImageFolder whose root may itself be the single class folder (dataset.py:119-203): classes are
    the sorted sub-folders, or the folder's own name when it has none; samples are (path, class index)
    in sorted walk order, files filtered by extension."""

    def __init__(self, root, transform=None, loader=pil_loader, extensions=IMG_EXTENSIONS):
        self.root = os.path.expanduser(root)
        self.transform = transform
        self.loader = loader
        self.classes, self.class_to_idx = self.find_classes(self.root)
        self.samples = self.make_dataset(self.root, self.class_to_idx, extensions)
        self.targets = [s[1] for s in self.samples]

    @staticmethod
    def find_classes(directory):
        subdirs = sorted(d for d in os.listdir(directory) if os.path.isdir(os.path.join(directory, d)))
        if not subdirs:
            name = os.path.basename(os.path.normpath(directory))
            return [name], {name: 0}
        return subdirs, {c: i for i, c in enumerate(subdirs)}

    @staticmethod
    def make_dataset(directory, class_to_idx, extensions=IMG_EXTENSIONS):
        instances = []
        for target_class in sorted(class_to_idx):
            idx = class_to_idx[target_class]
            target_dir = directory if os.path.basename(os.path.normpath(directory)) == target_class \
                else os.path.join(directory, target_class)
            if not os.path.isdir(target_dir):
                continue
            for root, _, fnames in sorted(os.walk(target_dir, followlinks=True)):
                for fname in sorted(fnames):
                    if fname.lower().endswith(tuple(extensions)):
                        instances.append((os.path.join(root, fname), idx))
        if not instances:
            raise FileNotFoundError(f"Found no valid file in {directory} (extensions {', '.join(extensions)})")
        return instances

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        path, target = self.samples[index]
        img = self.loader(path)
        if self.transform is not None:
            img = self.transform(img)
        return img, target


class SpectrogramDataset(Dataset):
    """The labelled spectrogram folder of config["processed_spectograms_dataset_folderpath"]
    (dataset.py:28-56)."""

    def __init__(self, config, raw=False):
        super().__init__()
        self.image_dir_path = config["processed_spectograms_dataset_folderpath"]
        self.data = ImageFolderNoSubdirs(root=self.image_dir_path, transform=SpectrogramTransform(raw=raw))

    def __getitem__(self, idx):
        return self.data[idx]

    def __len__(self):
        return len(self.data)

    def _get_transform(self):
        return SpectrogramTransform()


class SpectrogramPairDataset(Dataset):
    """Predetermined (content, style) pairs across label folders (dataset.py:206-303): the CSV rows are
    (label1, idx1, label2, idx2); an item is ((img1, label1), (img2, label2))."""

    def __init__(self, root_folder, pairing_file, transform=None):
        self.root_folder = root_folder
        self.pairing_file = pairing_file
        self.transform = transform if transform is not None else self._get_transform()
        self.pairs = []
        with open(self.pairing_file, "r") as f:
            for row in csv.reader(f):
                self.pairs.append((row[0], int(row[1]), row[2], int(row[3])))
        self.datasets = {}
        for folder in sorted(os.listdir(root_folder)):
            folder_path = os.path.join(root_folder, folder)
            if os.path.isdir(folder_path):
                self.datasets[folder] = ImageFolderNoSubdirs(root=folder_path, transform=self.transform)

    def __len__(self):
        return len(self.pairs)

    def __getitem__(self, index):
        label1, idx1, label2, idx2 = self.pairs[index]
        img1, _ = self.datasets[label1][idx1]
        img2, _ = self.datasets[label2][idx2]
        return (img1, label1), (img2, label2)

    @classmethod
    def _get_transform(cls):
        return SpectrogramTransform()

    @classmethod
    def generate_pairings(cls, root_folder, output_file_path="spectrogram_pair_dataset_pairings.csv",
                          num_pairs=15000):
        """The reference's deterministic pairing file: RandomState(42), two distinct sorted labels per pair
        (rng.choice without replacement), then one index in each (rng.randint), num_pairs rows."""
        labels = sorted(f for f in os.listdir(root_folder) if os.path.isdir(os.path.join(root_folder, f)))
        if len(labels) < 2:
            raise ValueError("Need at least two classes to form pairs.")
        sizes = {label: len(ImageFolderNoSubdirs(os.path.join(root_folder, label)).samples) for label in labels}
        rng = np.random.RandomState(42)
        pairs = []
        for _ in range(num_pairs):
            label1, label2 = rng.choice(labels, size=2, replace=False)
            idx1 = rng.randint(0, sizes[label1])
            idx2 = rng.randint(0, sizes[label2])
            pairs.append((label1, idx1, label2, idx2))
        with open(output_file_path, "w", newline="") as f:
            writer = csv.writer(f)
            for pair in pairs:
                writer.writerow(pair)
        print(f"Pairings saved to {output_file_path}")


def prepare_dataset(config):
    """80/20 random split of SpectrogramDataset into shuffled train / ordered test loaders (dataset.py:306-316)."""
    dataset = SpectrogramDataset(config)
    train_size = int(0.8 * len(dataset))
    test_size = len(dataset) - train_size
    train_dataset, test_dataset = torch.utils.data.random_split(dataset, [train_size, test_size])
    train_loader = DataLoader(train_dataset, batch_size=config["batch_size"], shuffle=True, num_workers=0)
    test_loader = DataLoader(test_dataset, batch_size=config["batch_size"], shuffle=False, num_workers=0)
    return train_loader, test_loader
