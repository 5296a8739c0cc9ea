"""Data entry points (``dataset_creation/data_loader.py:7-79``,
``dataset_creation/custom_dataset.py:10-100``, ``dataset_creation/SIDD_dataset.py:10-168``).

* ``load_data(image_folder, batch_size, num_workers, validation_split, augment,
  dataset_percentage, only_validation, include_noise_level, train_noise_levels,
  val_noise_levels, use_rgb)`` -> ``(train_loader, val_loader)`` yielding
  ``(noisy, clean)`` in [-1, 1] NCHW fp32, as the reference.  ``CustomDataset``
  cuts non-overlapping 256x256 patches, adds N(0, sigma) noise in uint8 space,
  clips, and applies the reference's transform: with ``augment``,
  RandomHorizontalFlip + RandomRotation(10) (PIL, NEAREST, fill 0) drawn once per
  item for both images, then ToTensor + Normalize(0.5, 0.5) (restated in
  numpy/torch: torchvision is not a dependency).
* ``load_sidd_data`` / ``CustomSIDD_Dataset``: the SIDD-Medium real-noise pairs
  (``Scene_Instances.txt`` + ``Data/<scene>/{NOISY,GT}*``).
* The GPU pipeline (decode once, synthesis on the device) is
  ``vub_image_denoising_amd.synth.load_data_gpu`` / ``load_sidd_data_gpu``.
* ``SyntheticNoiseDataset`` / ``synthetic_batch``: the benchmark's seeded
  synthetic stream (uniform clean images, sigma in {15, 25, 50}).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, random_split


def _to_tensor_normalized(arr: np.ndarray) -> torch.Tensor:
    """ToTensor (HWC uint8 -> CHW float/255) + Normalize(0.5, 0.5) -> [-1, 1]."""
    if arr.ndim == 2:
        arr = arr[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1))).float().div_(255.0)
    return t.sub_(0.5).div_(0.5)


def add_gaussian_noise_u8(patch_u8: np.ndarray, sigma: float, rng=np.random) -> np.ndarray:
    """custom_dataset.py:84-86: float32 + N(0, sigma) -> clip [0, 255] -> uint8."""
    noisy = patch_u8.astype(np.float32)
    noisy += rng.normal(scale=sigma, size=noisy.shape)
    return np.clip(noisy, 0, 255).astype(np.uint8)


def _augment_pair(a: np.ndarray, b: np.ndarray):
    """The reference's augmentation transform on both images of an item with one
    parameter draw (custom_dataset.py:89-95: the same torch seed before each):
    RandomHorizontalFlip (torch.rand(1) < 0.5 -> Image.transpose(FLIP_LEFT_RIGHT)),
    RandomRotation(10) (angle ~ U(-10, 10) -> Image.rotate(angle, NEAREST, fill 0))."""
    from PIL import Image
    flip = bool(torch.rand(1) < 0.5)
    angle = float(torch.empty(1).uniform_(-10.0, 10.0).item())
    out = []
    for arr in (a, b):
        im = Image.fromarray(arr if arr.shape[2] == 3 else arr[:, :, 0])
        if flip:
            im = im.transpose(Image.FLIP_LEFT_RIGHT)
        im = im.rotate(angle, Image.NEAREST, False, None, fillcolor=0)
        r = np.array(im)
        out.append(r if r.ndim == 3 else r[:, :, None])
    return out


def _read(path, use_rgb, allow_rgba=True):
    from PIL import Image
    with Image.open(path) as im:
        if allow_rgba and im.mode == 'RGBA':
            im = im.convert('RGB')
        if not use_rgb:
            im = im.convert('L')
        a = np.array(im)
    return a if a.ndim == 3 else a[:, :, None]


class CustomDataset(Dataset):
    """custom_dataset.py:10-100 (PIL decode; same patch grid, noise, length, transform)."""

    def __init__(self, image_folder, transform=None, include_noise_level=False, noise_levels=None, use_rgb=False,
                 augment=False, patch_size=256):
        exts = ('png', 'jpg', 'jpeg')
        self.image_paths = sorted(os.path.join(image_folder, f) for f in os.listdir(image_folder)
                                  if f.lower().endswith(exts))
        self.noise_levels = noise_levels if noise_levels is not None else [15, 25, 50]
        self.include_noise_level = include_noise_level
        self.use_rgb = use_rgb
        self.augment = augment
        self.patch_size = patch_size
        self.patch_pairs = self._extract_patches()

    def _extract_patches(self):
        from PIL import Image
        pairs = []
        ps = self.patch_size
        for path in self.image_paths:
            with Image.open(path) as im:
                w, h = im.size
            for top in range(0, h, ps):
                for left in range(0, w, ps):
                    if top + ps <= h and left + ps <= w:
                        pairs.append((path, top, left))
        return pairs

    def __len__(self):
        return len(self.patch_pairs) * len(self.noise_levels)

    def __getitem__(self, idx):
        noise_idx = idx % len(self.noise_levels)
        path, top, left = self.patch_pairs[idx // len(self.noise_levels)]
        ps = self.patch_size
        gt = np.ascontiguousarray(_read(path, self.use_rgb)[top:top + ps, left:left + ps])
        sigma = self.noise_levels[noise_idx]
        noisy = add_gaussian_noise_u8(gt, sigma)
        if self.augment:
            seed = random.randint(0, 2 ** 32)
            torch.manual_seed(seed)
            gt, noisy = _augment_pair(gt, noisy)
        gt_t, noisy_t = _to_tensor_normalized(gt), _to_tensor_normalized(noisy)
        if self.include_noise_level:
            return noisy_t, gt_t, sigma
        return noisy_t, gt_t


def load_data(image_folder, batch_size=4, num_workers=4, validation_split=0.2, augment=False, dataset_percentage=1.0,
              only_validation=False, include_noise_level=False, train_noise_levels=None, val_noise_levels=None,
              use_rgb=False):
    """data_loader.py:7-79."""
    if only_validation:
        val = CustomDataset(image_folder, include_noise_level=include_noise_level, noise_levels=val_noise_levels,
                            use_rgb=use_rgb, augment=augment)
        return None, DataLoader(val, batch_size=batch_size, shuffle=False, num_workers=num_workers)
    train_dataset = CustomDataset(image_folder, include_noise_level=include_noise_level,
                                  noise_levels=train_noise_levels, use_rgb=use_rgb, augment=augment)
    total = len(train_dataset)
    subset = int(total * dataset_percentage)
    if subset < total:
        train_dataset, _ = random_split(train_dataset, [subset, total - subset])
    train_size = int((1 - validation_split) * len(train_dataset))
    train_dataset, val_dataset = random_split(train_dataset, [train_size, len(train_dataset) - train_size])
    return (DataLoader(train_dataset, batch_size=batch_size, shuffle=True, num_workers=num_workers),
            DataLoader(val_dataset, batch_size=batch_size, shuffle=False, num_workers=num_workers))


class CustomSIDD_Dataset(Dataset):
    """SIDD_dataset.py:10-97: noisy/gt pairs of every scene in Scene_Instances.txt,
    all full non-overlapping 256x256 patches."""

    def __init__(self, root_folder, transform=None, use_rgb=False, augment=False, patch_size=256):
        from .synth import sidd_pairs
        from PIL import Image
        self.image_pairs = sidd_pairs(root_folder)
        self.use_rgb = use_rgb
        self.augment = augment
        self.patch_size = ps = patch_size
        self.patch_pairs = []
        for noisy_path, gt_path in self.image_pairs:
            with Image.open(noisy_path) as im:
                w, h = im.size
            for top in range(0, h, ps):
                for left in range(0, w, ps):
                    if top + ps <= h and left + ps <= w:
                        self.patch_pairs.append((noisy_path, gt_path, top, left))

    def __len__(self):
        return len(self.patch_pairs)

    def __getitem__(self, idx):
        noisy_path, gt_path, top, left = self.patch_pairs[idx]
        ps = self.patch_size
        noisy = np.ascontiguousarray(_read(noisy_path, self.use_rgb, False)[top:top + ps, left:left + ps])
        gt = np.ascontiguousarray(_read(gt_path, self.use_rgb, False)[top:top + ps, left:left + ps])
        if self.augment:
            seed = random.randint(0, 2 ** 32)
            torch.manual_seed(seed)
            gt, noisy = _augment_pair(gt, noisy)
        return _to_tensor_normalized(noisy), _to_tensor_normalized(gt)


def load_sidd_data(root_folder, batch_size=4, num_workers=2, validation_split=0.2, augment=False,
                   dataset_percentage=1.0, only_validation=False, use_rgb=False):
    """SIDD_dataset.py:99-168."""
    dataset = CustomSIDD_Dataset(root_folder, use_rgb=use_rgb, augment=augment)
    if only_validation:
        return None, DataLoader(dataset, batch_size=batch_size, shuffle=False, num_workers=num_workers)
    total = len(dataset)
    subset = int(total * dataset_percentage)
    if subset < total:
        dataset, _ = random_split(dataset, [subset, total - subset])
    train_size = int((1 - validation_split) * len(dataset))
    train_dataset, val_dataset = random_split(dataset, [train_size, len(dataset) - train_size])
    return (DataLoader(train_dataset, batch_size=batch_size, shuffle=True, num_workers=num_workers),
            DataLoader(val_dataset, batch_size=batch_size, shuffle=False, num_workers=num_workers))


# ----------------------------------------------------------------- synthetic
def synthetic_batch(batch, h=256, w=256, sigma=25.0, seed=1234, device="cuda", generator=None):
    """Seeded synthetic (noisy, clean) pair in [-1, 1]: clean ~ U(-1, 1),
    noisy = clean + (sigma/255*2) * N(0, 1)."""
    g = generator or torch.Generator(device=device).manual_seed(seed)
    clean = torch.rand(batch, 3, h, w, generator=g, device=device) * 2 - 1
    noisy = clean + (sigma / 255.0 * 2.0) * torch.randn(batch, 3, h, w, generator=g, device=device)
    return noisy, clean


class SyntheticNoiseDataset(Dataset):
    """Deterministic synthetic dataset: item i has sigma = levels[i % 3]."""

    def __init__(self, n, h=256, w=256, noise_levels=(15, 25, 50), seed=0):
        self.n, self.h, self.w, self.levels, self.seed = n, h, w, list(noise_levels), seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        clean = torch.rand(3, self.h, self.w, generator=g) * 2 - 1
        sigma = self.levels[i % len(self.levels)]
        noisy = clean + (sigma / 255.0 * 2.0) * torch.randn(3, self.h, self.w, generator=g)
        return noisy, clean
