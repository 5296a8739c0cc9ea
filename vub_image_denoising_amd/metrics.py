"""Image-quality metrics of the SIDD evaluation on the GPU (``rdn_image_metrics``,
csrc/metrics.hip): scikit-image 0.22's ``peak_signal_noise_ratio`` and
``structural_similarity`` as the reference calls them
(evaluate_SIDD/evaluate_SIDD.py:63-64: data_range=2, channel_axis=-1, default
7x7 uniform window, sample covariance), for whole batches resident in HBM
instead of one block at a time on the host.

``image_metrics(gt, x, data_range)`` is the batched form (NCHW fp32 device
tensors -> per-image float64 PSNR and SSIM); the two skimage-named functions take
one image (HW, or HWC with ``channel_axis=-1`` / CHW with ``channel_axis=0``) on
the device and return Python floats.
"""
from __future__ import annotations

import torch

from . import _hip as H


def image_metrics(gt: torch.Tensor, x: torch.Tensor, data_range: float):
    """Per-image PSNR and SSIM of two [N, C, H, W] batches (float64 device tensors)."""
    H.require_device(gt, x)
    if gt.shape != x.shape or gt.dim() != 4:
        raise ValueError(f"image_metrics: expected two equal [N,C,H,W] batches, got {tuple(gt.shape)} and "
                         f"{tuple(x.shape)}")
    n, c, h, w = gt.shape
    if h < 7 or w < 7:
        raise ValueError("win_size exceeds image extent (images must be at least 7x7)")
    gt = gt.contiguous().float()
    x = x.contiguous().float()
    lib = H.lib()
    ws = torch.empty(max(lib.rdn_image_metrics_workspace_size(n, c, h, w) // 8, 1), dtype=torch.float64,
                     device=gt.device)
    psnr = torch.empty(n, dtype=torch.float64, device=gt.device)
    ssim = torch.empty(n, dtype=torch.float64, device=gt.device)
    H.check(lib.rdn_image_metrics(gt.data_ptr(), x.data_ptr(), n, c, h, w, float(data_range), ws.data_ptr(),
                                  psnr.data_ptr(), ssim.data_ptr(), H.stream_ptr()), "image_metrics")
    return psnr, ssim


def _as_nchw(img: torch.Tensor, channel_axis):
    if img.dim() == 2:
        if channel_axis is not None:
            raise ValueError("channel_axis given for a 2-D image")
        return img[None, None]
    if img.dim() != 3 or channel_axis is None:
        raise ValueError("3-D images need channel_axis (0 or -1)")
    ax = channel_axis % 3
    if ax == 2:
        return img.permute(2, 0, 1)[None]
    if ax == 0:
        return img[None]
    raise ValueError("channel_axis must be the first or last axis")


def peak_signal_noise_ratio(image_true: torch.Tensor, image_test: torch.Tensor, *, data_range: float) -> float:
    """skimage.metrics.peak_signal_noise_ratio for one device image (HW, HWC or
    CHW: the MSE does not depend on the layout, so the image is read as one
    [rows, rest] plane; both extents must be >= 7)."""
    if image_true.shape != image_test.shape:
        raise ValueError("Input images must have the same dimensions.")
    a = image_true.reshape(1, 1, image_true.shape[0], -1)
    b = image_test.reshape(1, 1, image_test.shape[0], -1)
    return float(image_metrics(a, b, data_range)[0][0].item())


def structural_similarity(im1: torch.Tensor, im2: torch.Tensor, *, data_range: float, channel_axis=None,
                          multichannel=None) -> float:
    """skimage.metrics.structural_similarity (win_size 7, uniform window, sample
    covariance) for one device image; ``multichannel`` is accepted and ignored as
    skimage 0.22 does when ``channel_axis`` is given."""
    if im1.shape != im2.shape:
        raise ValueError("Input images must have the same dimensions.")
    return float(image_metrics(_as_nchw(im1, channel_axis), _as_nchw(im2, channel_axis), data_range)[1][0].item())
