"""Data entry points (``dataset_creation/data_loader.py:7-79``,
``dataset_creation/custom_dataset.py:10-100``, ``dataset_creation/SIDD_dataset.py:99-168``).

* ``load_data(image_folder, batch_size, num_workers, validation_split, augment,
  dataset_percentage, only_validation, include_noise_level, train_noise_levels,
  val_noise_levels, use_rgb)`` -> ``(train_loader, val_loader)`` yielding
  ``(noisy, clean)`` in [-1, 1] NCHW fp32, as the reference.  ``CustomDataset``
  cuts non-overlapping 256x256 patches, adds N(0, sigma) noise in uint8 space,
  clips, and normalises with mean = std = 0.5 (ToTensor + Normalize restated
  in numpy: torchvision is not a dependency).
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


class CustomDataset(Dataset):
    """custom_dataset.py:10-100 (PIL decode; same patch grid, noise and length)."""

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
        from PIL import Image
        noise_idx = idx % len(self.noise_levels)
        path, top, left = self.patch_pairs[idx // len(self.noise_levels)]
        with Image.open(path) as im:
            if im.mode == 'RGBA':
                im = im.convert('RGB')
            if not self.use_rgb:
                im = im.convert('L')
            gt = np.array(im.crop((left, top, left + self.patch_size, top + self.patch_size)))
        sigma = self.noise_levels[noise_idx]
        noisy = add_gaussian_noise_u8(gt, sigma)
        if self.augment and random.random() < 0.5:  # RandomHorizontalFlip, same draw for both
            gt, noisy = gt[:, ::-1], noisy[:, ::-1]
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


def load_sidd_data(image_folder, batch_size=4, num_workers=4, validation_split=0.2, augment=False,
                   dataset_percentage=1.0, use_rgb=True):
    """SIDD_dataset.py:99-168 entry point.  The SIDD-Medium pairs are not in this
    environment; the loader is the next row of the build plan."""
    raise NotImplementedError("SIDD real-noise loader: dataset not available in this environment "
                              "(SURVEY.md §8f row 4)")


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
