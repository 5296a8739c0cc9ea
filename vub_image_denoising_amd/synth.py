"""GPU data pipeline: the reference's per-item host loaders
(``dataset_creation/custom_dataset.py:10-100``, ``SIDD_dataset.py:10-97`` behind
``data_loader.py:7-79`` / ``SIDD_dataset.py:99-168``) re-designed for an
MI355X fed at thousands of images/s.

* ``PatchPool`` decodes the image folder ONCE (PIL) and keeps every image as
  uint8 HWC in one HBM buffer (DIV2K-train is ~6.6 GB; 288 GB per GPU), with the
  reference's non-overlapping patch grid (custom_dataset.py:44-58).
* ``GpuLoader`` iterates dataset indices like a DataLoader; per batch the host
  only draws the item parameters (patch, sigma = levels[i % L]
  (custom_dataset.py:68-71), flip, rotation angle, noise seed) and
  ``rdn_synth_batch`` builds the whole (noisy, clean) batch on the device in
  one launch: noise -> clip -> uint8 -> flip -> rotate -> ToTensor/Normalize.
* ``load_data_gpu`` / ``load_sidd_data_gpu`` mirror ``load_data``'s signature and
  split semantics and return (train_loader, val_loader) yielding device tensors.

Noise is drawn on the device from a counter-based stream (distributionally the
reference's ``np.random.normal``; pass ``noise=`` to ``synth_batch`` to reproduce
given float64 draws bit for bit).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _hip as H

ITEM_DTYPE = np.dtype([("clean_off", "<i8"), ("noisy_off", "<i8"), ("seed", "<u8"), ("row_stride", "<i4"),
                       ("sigma", "<f4"), ("flip", "<i4"), ("rotate", "<i4"), ("affine", "<i4", (6,))])


def rotate_coeffs(angle: float, w: int, h: int):
    """Pillow ``Image.rotate(angle, NEAREST)`` as the 16.16 fixed-point output->input
    coefficients of its nearest-neighbour affine (PIL/Image.py rotate; Geometry.c
    affine_fixed).  None = Pillow's copy fast path (angle % 360 == 0)."""
    angle = angle % 360.0
    if angle == 0:
        return None
    if angle in (90.0, 180.0, 270.0):
        raise ValueError("right-angle rotations take Pillow's transpose path; RandomRotation(10) never draws them")
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    m[2], m[5] = m[0] * -cx + m[1] * -cy + m[2], m[3] * -cx + m[4] * -cy + m[5]
    m[2] += cx
    m[5] += cy
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))
    return [fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
            fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5)]


def _read_image(path, use_rgb):
    from PIL import Image
    with Image.open(path) as im:
        if im.mode == "RGBA":
            im = im.convert("RGB")
        im = im.convert("RGB") if use_rgb else im.convert("L")
        a = np.array(im, dtype=np.uint8)
    return a if a.ndim == 3 else a[:, :, None]


class PatchPool:
    """uint8 HWC images resident in device memory + the non-overlapping patch grid.
    ``noisy_images`` (same shapes) makes it a paired (real-noise) pool."""

    def __init__(self, images, patch_size=256, device="cuda", noisy_images=None):
        if not images:
            raise ValueError("PatchPool: no images")
        self.channels = images[0].shape[2]
        self.patch_size = ps = patch_size
        offs, o = [], 0
        for im in images:
            if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != self.channels:
                raise ValueError("PatchPool: images must be uint8 HxWxC with one channel count")
            offs.append(o)
            o += im.size
        self.shapes = [im.shape for im in images]
        self.offsets = offs
        self.clean = torch.from_numpy(np.concatenate([im.reshape(-1) for im in images])).to(device)
        self.noisy = None
        if noisy_images is not None:
            if [im.shape for im in noisy_images] != self.shapes:
                raise ValueError("PatchPool: noisy/gt shape mismatch")
            self.noisy = torch.from_numpy(np.concatenate([im.reshape(-1) for im in noisy_images])).to(device)
        # custom_dataset.py:44-58 / SIDD_dataset.py:51-68: every full non-overlapping patch
        self.patches = [(k, top, left) for k, (h, w, _) in enumerate(self.shapes)
                        for top in range(0, h, ps) for left in range(0, w, ps) if top + ps <= h and left + ps <= w]
        self.device = self.clean.device

    @classmethod
    def from_folder(cls, image_folder, use_rgb=False, patch_size=256, device="cuda"):
        """custom_dataset.py:34-42: sorted *.png/*.jpg/*.jpeg (RGBA -> RGB, 'L' unless use_rgb)."""
        exts = ("png", "jpg", "jpeg")
        paths = sorted(os.path.join(image_folder, f) for f in os.listdir(image_folder) if f.lower().endswith(exts))
        return cls([_read_image(p, use_rgb) for p in paths], patch_size, device)

    @classmethod
    def from_sidd(cls, root_folder, use_rgb=False, patch_size=256, device="cuda"):
        """SIDD_dataset.py:31-49: scenes of Scene_Instances.txt, sorted NOISY/GT files paired."""
        pairs = sidd_pairs(root_folder)
        gts = [_read_image(g, use_rgb) for _, g in pairs]
        noisy = [_read_image(n, use_rgb) for n, _ in pairs]
        return cls(gts, patch_size, device, noisy_images=noisy)

    def __len__(self):
        return len(self.patches)

    def encode(self, patch_idx, sigma, flip, angle, seed, item):
        k, top, left = self.patches[patch_idx]
        h, w, c = self.shapes[k]
        off = self.offsets[k] + (top * w + left) * c
        item["clean_off"] = off
        item["noisy_off"] = off
        item["row_stride"] = w * c
        item["sigma"] = sigma
        item["flip"] = int(bool(flip))
        co = None if angle is None else rotate_coeffs(angle, self.patch_size, self.patch_size)
        item["rotate"] = int(co is not None)
        item["affine"] = co if co is not None else [0] * 6
        item["seed"] = seed


def sidd_pairs(root_folder):
    data = os.path.join(root_folder, "Data")
    with open(os.path.join(root_folder, "Scene_Instances.txt")) as f:
        scenes = f.read().splitlines()
    pairs = []
    for scene in scenes:
        d = os.path.join(data, scene)
        if os.path.isdir(d):
            noisy = sorted(os.path.join(d, f) for f in os.listdir(d) if "NOISY" in f)
            gt = sorted(os.path.join(d, f) for f in os.listdir(d) if "GT" in f)
            pairs.extend(zip(noisy, gt))
    return pairs


def synth_batch(pool: PatchPool, items: np.ndarray, noise: torch.Tensor | None = None):
    """One rdn_synth_batch launch: ``items`` (ITEM_DTYPE array) -> (noisy, clean) fp32
    NCHW device tensors.  ``noise``: optional float64 [n, P, P, C] device draws."""
    n, P, C = len(items), pool.patch_size, pool.channels
    dev = pool.device
    items_dev = torch.from_numpy(np.ascontiguousarray(items).view(np.uint8)).to(dev, non_blocking=True)
    noisy = torch.empty(n, C, P, P, dtype=torch.float32, device=dev)
    clean = torch.empty_like(noisy)
    if noise is not None:
        if noise.dtype != torch.float64 or tuple(noise.shape) != (n, P, P, C) or not noise.is_contiguous():
            raise RuntimeError("synth_batch: noise must be contiguous float64 [n, P, P, C] on the device")
        H.require_device(noise)
    H.check(H.lib().rdn_synth_batch(items_dev.data_ptr(), n, C, P, pool.clean.data_ptr(),
                                    None if pool.noisy is None else pool.noisy.data_ptr(),
                                    None if noise is None else noise.data_ptr(), noisy.data_ptr(),
                                    clean.data_ptr(), H.stream_ptr()), "synth_batch")
    return noisy, clean


class GpuLoader:
    """DataLoader-like iterable over dataset indices of a PatchPool.  Synthetic-noise
    pools: index i -> patch i // L, sigma levels[i % L] (custom_dataset.py:60-71);
    paired pools: index = patch (SIDD_dataset.py:70-72).  Yields (noisy, clean)
    [, sigma] on the device."""

    def __init__(self, pool, indices, batch_size, noise_levels=None, shuffle=False, augment=False, seed=0,
                 include_noise_level=False, drop_last=False):
        self.pool = pool
        self.indices = list(indices)
        self.batch_size = batch_size
        self.levels = list(noise_levels) if noise_levels is not None else [15, 25, 50]
        self.shuffle, self.augment = shuffle, augment
        self.include_noise_level = include_noise_level
        self.drop_last = drop_last
        self.rng = np.random.default_rng(seed)
        self.dataset = self.indices   # len(loader.dataset) as with torch's DataLoader

    def __len__(self):
        n = len(self.indices)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _decode(self, idx):
        if self.pool.noisy is not None:
            return idx, 0.0
        return idx // len(self.levels), float(self.levels[idx % len(self.levels)])

    def __iter__(self):
        order = self.rng.permutation(len(self.indices)) if self.shuffle else np.arange(len(self.indices))
        for b in range(len(self)):
            sel = [self.indices[j] for j in order[b * self.batch_size:(b + 1) * self.batch_size]]
            items = np.zeros(len(sel), ITEM_DTYPE)
            sig = []
            for k, idx in enumerate(sel):
                p, sigma = self._decode(idx)
                flip = bool(self.augment and self.rng.random() < 0.5)         # RandomHorizontalFlip()
                angle = float(self.rng.uniform(-10.0, 10.0)) if self.augment else None   # RandomRotation(10)
                self.pool.encode(p, sigma, flip, angle, int(self.rng.integers(0, 2 ** 63)), items[k])
                sig.append(sigma)
            noisy, clean = synth_batch(self.pool, items)
            if self.include_noise_level:
                yield noisy, clean, torch.tensor(sig)
            else:
                yield noisy, clean


class MixedPatchLoader:
    """Config 5's mixed patch stream (BASELINE.json: SIDD at 128 and 256; the
    reference hard-codes 256, SIDD_dataset.py:56,63-66): one loader per patch size
    (each over its own PatchPool of the same images), batches taken from them in
    turn -- loader 0, 1, 0, 1, ... -- until every loader is exhausted.  The network
    takes any H, W divisible by 8; each shape gets its own engine (and, under
    train_graph.TrainStepGraphs, its own captured step)."""

    def __init__(self, loaders):
        if not loaders:
            raise ValueError("MixedPatchLoader: no loaders")
        self.loaders = list(loaders)
        self.dataset = [i for ld in self.loaders for i in ld.dataset]
        self.batch_size = self.loaders[0].batch_size

    def __len__(self):
        return sum(len(ld) for ld in self.loaders)

    def __iter__(self):
        its = [iter(ld) for ld in self.loaders]
        live = list(range(len(its)))
        while live:
            for k in list(live):
                try:
                    yield next(its[k])
                except StopIteration:
                    live.remove(k)


def _sizes(patch_size):
    return [int(patch_size)] if isinstance(patch_size, (int, np.integer)) else [int(p) for p in patch_size]


def _mixed(make, patch_size):
    """(train, val) loaders of one patch size, or MixedPatchLoaders over several."""
    pairs = [make(ps) for ps in _sizes(patch_size)]
    if len(pairs) == 1:
        return pairs[0]
    tr = [a for a, _ in pairs]
    va = [b for _, b in pairs]
    return (None if tr[0] is None else MixedPatchLoader(tr)), MixedPatchLoader(va)


def _cell_split(pools, n_levels, dataset_percentage, validation_split, generator):
    """Train / validation split of several patch grids over the SAME images (config
    5's mixed sizes): the unit is a cell of the largest grid -- (image, top // P,
    left // P), P the largest patch size; every patch lies in exactly one cell, since
    the grids all start at 0 with strides dividing P -- and a cell goes wholly to one
    side, with all its patches of every size and every noise level.  So no validation
    patch of one size shares a pixel with a training patch of another (the per-size
    index splits of round 4 let ~80 % of the 128-pixel validation patches lie inside
    256-pixel training patches).  The cells themselves are split as data_loader.py:
    63-74 splits items (optional random subset, then random_split).  Returns one
    (train, val) index-list pair per pool (index = patch * n_levels + level)."""
    P = max(pl.patch_size for pl in pools)
    if any(P % pl.patch_size for pl in pools):
        raise ValueError("mixed patch sizes must divide the largest one")
    cell_of = [[(k, top // P, left // P) for k, top, left in pl.patches] for pl in pools]
    cells = sorted({c for cs in cell_of for c in cs})
    tr_c, va_c = _split(len(cells), dataset_percentage, validation_split, generator)
    side = {cells[i]: 0 for i in tr_c}
    side.update({cells[i]: 1 for i in va_c})
    out = []
    for cs in cell_of:
        tr, va = [], []
        for j, c in enumerate(cs):
            s_ = side.get(c)
            if s_ is not None:
                (tr if s_ == 0 else va).extend(j * n_levels + lv for lv in range(n_levels))
        out.append((tr, va))
    return out


def _split(total, dataset_percentage, validation_split, generator):
    """data_loader.py:63-74: optional random subset, then the train/val random_split."""
    idx = list(range(total))
    subset = int(total * dataset_percentage)
    if subset < total:
        perm = torch.randperm(total, generator=generator).tolist()
        idx = perm[:subset]
    train_size = int((1 - validation_split) * len(idx))
    perm = torch.randperm(len(idx), generator=generator).tolist()
    return [idx[j] for j in perm[:train_size]], [idx[j] for j in perm[train_size:]]


def load_data_gpu(image_folder, batch_size=4, validation_split=0.2, augment=False, dataset_percentage=1.0,
                  only_validation=False, include_noise_level=False, train_noise_levels=None, val_noise_levels=None,
                  use_rgb=False, patch_size=256, seed=0, device="cuda", pool=None, images=None):
    """``data_loader.load_data`` (data_loader.py:7-79) with device-side synthesis.
    ``patch_size`` may be a sequence (e.g. (128, 256)): one pool per size over the
    same images, batches alternating between them (MixedPatchLoader).  ``images``:
    uint8 HWC arrays instead of reading ``image_folder``."""
    if pool is None and (images is not None or not isinstance(patch_size, (int, np.integer))):
        if images is None:
            exts = ("png", "jpg", "jpeg")
            images = [_read_image(os.path.join(image_folder, f), use_rgb) for f in sorted(os.listdir(image_folder))
                      if f.lower().endswith(exts)]
        sizes = _sizes(patch_size)
        if len(sizes) > 1 and not only_validation:   # one split over cells of the largest grid
            pools = [PatchPool(images, ps, device) for ps in sizes]
            levels = train_noise_levels if train_noise_levels is not None else [15, 25, 50]
            g = torch.Generator().manual_seed(seed)
            splits = _cell_split(pools, len(levels), dataset_percentage, validation_split, g)
            tr = [GpuLoader(pl, a, batch_size, levels, True, augment, seed + 1, include_noise_level)
                  for pl, (a, _) in zip(pools, splits)]
            va = [GpuLoader(pl, b, batch_size, levels, False, augment, seed + 2, include_noise_level)
                  for pl, (_, b) in zip(pools, splits)]
            return MixedPatchLoader(tr), MixedPatchLoader(va)
        return _mixed(lambda ps: load_data_gpu(image_folder, batch_size, validation_split, augment, dataset_percentage,
                                               only_validation, include_noise_level, train_noise_levels,
                                               val_noise_levels, use_rgb, ps, seed, device,
                                               pool=PatchPool(images, ps, device)), patch_size)
    pool = pool or PatchPool.from_folder(image_folder, use_rgb, patch_size, device)
    if only_validation:
        levels = val_noise_levels if val_noise_levels is not None else [15, 25, 50]
        return None, GpuLoader(pool, range(len(pool) * len(levels)), batch_size, levels, False, augment, seed,
                               include_noise_level)
    levels = train_noise_levels if train_noise_levels is not None else [15, 25, 50]
    g = torch.Generator().manual_seed(seed)
    tr, va = _split(len(pool) * len(levels), dataset_percentage, validation_split, g)
    # as in the reference, the validation split comes out of the TRAIN dataset (same
    # noise levels and transform); val_noise_levels only matter with only_validation
    return (GpuLoader(pool, tr, batch_size, levels, True, augment, seed + 1, include_noise_level),
            GpuLoader(pool, va, batch_size, levels, False, augment, seed + 2, include_noise_level))


def load_sidd_data_gpu(root_folder, batch_size=4, validation_split=0.2, augment=False, dataset_percentage=1.0,
                       only_validation=False, use_rgb=False, patch_size=256, seed=0, device="cuda", pool=None):
    """``SIDD_dataset.load_data`` (SIDD_dataset.py:99-168) with device-side batches.
    ``patch_size=(128, 256)``: config 5's mixed patch stream (MixedPatchLoader)."""
    if pool is None and not isinstance(patch_size, (int, np.integer)):
        pairs = sidd_pairs(root_folder)
        gts = [_read_image(g, use_rgb) for _, g in pairs]
        noisy = [_read_image(n, use_rgb) for n, _ in pairs]
        sizes = _sizes(patch_size)
        if len(sizes) > 1 and not only_validation:   # one split over cells of the largest grid
            pools = [PatchPool(gts, ps, device, noisy_images=noisy) for ps in sizes]
            g = torch.Generator().manual_seed(seed)
            splits = _cell_split(pools, 1, dataset_percentage, validation_split, g)
            return (MixedPatchLoader([GpuLoader(pl, a, batch_size, None, True, augment, seed + 1)
                                      for pl, (a, _) in zip(pools, splits)]),
                    MixedPatchLoader([GpuLoader(pl, b, batch_size, None, False, augment, seed + 2)
                                      for pl, (_, b) in zip(pools, splits)]))
        return _mixed(lambda ps: load_sidd_data_gpu(root_folder, batch_size, validation_split, augment,
                                                    dataset_percentage, only_validation, use_rgb, ps, seed, device,
                                                    pool=PatchPool(gts, ps, device, noisy_images=noisy)),
                      patch_size)
    pool = pool or PatchPool.from_sidd(root_folder, use_rgb, patch_size, device)
    if only_validation:
        return None, GpuLoader(pool, range(len(pool)), batch_size, None, False, augment, seed)
    g = torch.Generator().manual_seed(seed)
    tr, va = _split(len(pool), dataset_percentage, validation_split, g)
    return (GpuLoader(pool, tr, batch_size, None, True, augment, seed + 1),
            GpuLoader(pool, va, batch_size, None, False, augment, seed + 2))
