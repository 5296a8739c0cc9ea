"""CPU restatement of the data-synthesis path — TEST INFRASTRUCTURE ONLY.

Restates in numpy, per item, what the reference's loaders do on the host and
what ``rdn_synth_batch`` (csrc/synth.hip) does on the GPU:

* ``dataset_creation/custom_dataset.py:83-86``: ``noisy = np.array(gt, float32);
  noisy += np.random.normal(scale=sigma)`` (float64 draws), ``np.clip(0, 255)``,
  ``astype(uint8)``;
* the transforms of ``dataset_creation/data_loader.py:35-46`` (and
  ``SIDD_dataset.py:125-136``), applied with one parameter draw to both images
  (``custom_dataset.py:89-95``): ``RandomHorizontalFlip`` -> ``RandomRotation(10)``
  -> ``ToTensor`` -> ``Normalize(0.5, 0.5)``.  torchvision is not installed here;
  its PIL path is ``F.hflip`` = ``Image.transpose(FLIP_LEFT_RIGHT)`` and
  ``F.rotate`` = ``Image.rotate(angle, NEAREST, expand=False, center=None,
  fillcolor=0)`` (torchvision 0.18, requirements.txt:116).  The rotation is
  restated from Pillow: the inverse matrix of ``Image.rotate`` (PIL/Image.py) and
  the 16.16 fixed-point nearest-neighbour affine of ``Geometry.c``
  (``affine_fixed``); ``tests/test_synth_cpu.py`` pins it against Pillow itself.
* the device noise stream of ``rdn_synth_batch``: splitmix64 counter hash ->
  Box-Muller in float64 (same generator as ``oracle/weights.py``).
"""
from __future__ import annotations

import math

import numpy as np


def pil_rotate_matrix(angle: float, w: int, h: int):
    """Image.rotate's output->input affine (PIL/Image.py, expand=False, center=None,
    translate=None).  None when Pillow takes its copy fast path (angle % 360 == 0)."""
    angle = angle % 360.0
    if angle == 0:
        return None
    if angle in (90.0, 180.0, 270.0):
        raise NotImplementedError("Pillow transposes for right angles; RandomRotation(10) never draws them")
    center = (w / 2, h / 2)
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    x, y = -center[0] - 0, -center[1] - 0
    m[2], m[5] = m[0] * x + m[1] * y + m[2], m[3] * x + m[4] * y + m[5]
    m[2] += center[0]
    m[5] += center[1]
    return m


def fixed_coeffs(m):
    """Geometry.c affine_fixed: a0..a5 in 16.16 (FIX(v) = FLOOR(v*65536 + 0.5)), the
    pixel-centre offset folded into a2/a5."""
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))
    return [fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
            fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5)]


def rotate_coeffs(angle: float, w: int, h: int):
    m = pil_rotate_matrix(angle, w, h)
    return None if m is None else fixed_coeffs(m)


def source_map(coeffs, P: int):
    """(xin, yin, valid) for every output pixel of a P x P image."""
    y, x = np.meshgrid(np.arange(P, dtype=np.int64), np.arange(P, dtype=np.int64), indexing="ij")
    if coeffs is None:
        return x, y, np.ones((P, P), bool)
    a0, a1, a2, a3, a4, a5 = (np.int64(c) for c in coeffs)
    xx = (a2 + y * a1 + x * a0).astype(np.int32)       # int32 arithmetic, as in C
    yy = (a5 + y * a4 + x * a3).astype(np.int32)
    xin, yin = (xx >> 16).astype(np.int64), (yy >> 16).astype(np.int64)
    ok = (xin >= 0) & (xin < P) & (yin >= 0) & (yin < P)
    return xin, yin, ok


def rotate_nearest(img: np.ndarray, angle: float) -> np.ndarray:
    """Image.rotate(angle, NEAREST, fillcolor=0) of a square uint8 HWC image."""
    P = img.shape[0]
    xin, yin, ok = source_map(rotate_coeffs(angle, img.shape[1], P), P)
    out = np.zeros_like(img)
    out[ok] = img[yin[ok], xin[ok]]
    return out


def add_noise_u8(patch_u8: np.ndarray, noise_f64: np.ndarray) -> np.ndarray:
    """custom_dataset.py:84-86, literally."""
    noisy = np.array(patch_u8, dtype=np.float32)
    noisy += noise_f64
    return np.clip(noisy, 0, 255).astype(np.uint8)


def to_unit(img_u8: np.ndarray) -> np.ndarray:
    """ToTensor + Normalize(0.5, 0.5) in fp32: HWC uint8 -> CHW float32 in [-1, 1]."""
    t = img_u8.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    return (t - np.float32(0.5)) / np.float32(0.5)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def device_normal(seed: int, n: int) -> np.ndarray:
    """The device stream of rdn_synth_batch: N(0, 1) for elements 0..n-1."""
    key = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    e = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        u = []
        for s in (0, 1):
            ctr = e * np.uint64(2) + np.uint64(s)
            h = _splitmix64(_splitmix64(ctr ^ key) + key)
            u.append(((h >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0))
    return np.sqrt(-2.0 * np.log(u[0])) * np.cos(6.283185307179586 * u[1])


def synth_item(patch_u8: np.ndarray, flip: bool, angle: float | None, noise_f64: np.ndarray | None = None,
               noisy_u8: np.ndarray | None = None):
    """One (noisy, clean) item: noise on the source patch, then flip -> rotate ->
    ToTensor/Normalize on both images.  ``noisy_u8`` given: paired data (SIDD)."""
    if noisy_u8 is None:
        noisy_u8 = add_noise_u8(patch_u8, noise_f64 if noise_f64 is not None else np.zeros(patch_u8.shape))
    imgs = [patch_u8, noisy_u8]
    if flip:
        imgs = [im[:, ::-1] for im in imgs]
    if angle is not None:
        imgs = [rotate_nearest(np.ascontiguousarray(im), angle) for im in imgs]
    return to_unit(imgs[1]), to_unit(imgs[0])
