"""Portable, order-independent parameter generator for fixtures (test infra).

Every tensor is a pure function of ``(seed, parameter name, element index)``:
a splitmix64 counter hash feeds a Box-Muller transform (weights) or a uniform
(biases, PReLU slopes).  The same ``seed`` therefore gives bit-identical
parameters in the build container and on the GPU box without shipping weight
files, and regardless of module construction order.

Scales follow the reference initialisation in spirit:
* ``*.weight`` of Conv2d / ConvTranspose2d (4-D): xavier-normal std
  ``sqrt(2 / (fan_in + fan_out))`` with torch's fan convention
  (``diffusion_denoising/Unet/Unet_model.py:4-21`` applies xavier_normal_ to
  every module whose class name contains "Conv2d", ConvTranspose2d included);
* ``*.bias``: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (PyTorch default kept by the
  reference);
* PReLU ``*.weight`` (1-D): 0.25 + U(-0.05, 0.05) — the reference starts every
  slope at 0.25; the per-channel jitter makes channel-mapping bugs visible.
"""
from __future__ import annotations

import zlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform01(seed: int, name: str, n: int, stream: int = 0) -> np.ndarray:
    key = (np.uint64(seed & 0xFFFFFFFF) << np.uint64(32)) | np.uint64(zlib.crc32(name.encode()))
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) * np.uint64(2) + np.uint64(stream)
        h = _splitmix64(_splitmix64(ctr ^ key) + key)
    # 53 random mantissa bits -> (0, 1)
    return ((h >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def hash_normal(seed: int, name: str, n: int) -> np.ndarray:
    u1 = _uniform01(seed, name, n, 0)
    u2 = _uniform01(seed, name, n, 1)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def hash_uniform(seed: int, name: str, n: int, lo: float, hi: float) -> np.ndarray:
    return lo + (hi - lo) * _uniform01(seed, name, n, 0)


def _fans(shape):
    receptive = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    return shape[1] * receptive, shape[0] * receptive


def make_params(shapes: dict, seed: int = 0) -> dict:
    """``shapes``: ordered ``{name: shape}`` (a state_dict's keys/shapes).

    Returns ``{name: np.float32 array}``.  A ``.bias`` uses the fan-in of the
    sibling ``.weight``.
    """
    out = {}
    for name, shape in shapes.items():
        shape = tuple(int(s) for s in shape)
        n = int(np.prod(shape))
        if name.endswith(".weight") and len(shape) == 4:
            fan_in, fan_out = _fans(shape)
            std = np.sqrt(2.0 / float(fan_in + fan_out))
            v = std * hash_normal(seed, name, n)
        elif name.endswith(".bias"):
            wshape = tuple(shapes[name[: -len(".bias")] + ".weight"])
            fan_in, _ = _fans(wshape)
            b = 1.0 / np.sqrt(fan_in)
            v = hash_uniform(seed, name, n, -b, b)
        elif name.endswith(".weight") and len(shape) == 1:
            v = 0.25 + hash_uniform(seed, name, n, -0.05, 0.05)
        else:
            raise ValueError(f"unknown parameter kind: {name} {shape}")
        out[name] = v.astype(np.float32).reshape(shape)
    return out


def hash_images(seed: int, name: str, shape, lo=-1.0, hi=1.0) -> np.ndarray:
    n = int(np.prod(shape))
    return hash_uniform(seed, name, n, lo, hi).astype(np.float32).reshape(shape)


def hash_gauss_images(seed: int, name: str, shape) -> np.ndarray:
    n = int(np.prod(shape))
    return hash_normal(seed, name, n).astype(np.float32).reshape(shape)
