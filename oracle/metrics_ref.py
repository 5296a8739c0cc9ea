"""CPU restatement of the SIDD evaluation metrics — TEST INFRASTRUCTURE ONLY.

The reference scores denoised SIDD blocks with scikit-image 0.22
(requirements.txt:98) on the host:

* ``peak_signal_noise_ratio(gt, output, data_range=2)``
  (evaluate_SIDD/evaluate_SIDD.py:63);
* ``structural_similarity(gt, output, data_range=2, multichannel=True,
  channel_axis=-1)`` (evaluate_SIDD/evaluate_SIDD.py:64).

scikit-image is not installed here, so this module restates its published
algorithm (skimage/metrics/simple_metrics.py and _structural_similarity.py,
v0.22) with numpy + scipy (scipy.ndimage.uniform_filter is what skimage calls):
fp32 images stay fp32 (``_supported_float_type``), the MSE sum is float64, the
SSIM map is cropped by (win_size - 1) // 2 and averaged in float64, channels are
averaged.  ``ssim_bruteforce`` is an independent loop restatement (float64, one
window at a time) that the tests use to pin ``ssim`` together with closed forms
(identical images -> 1; constant images -> (2ab + C1) / (a^2 + b^2 + C1)).
Parity against skimage itself is therefore pinned by restatement, not by the
library (absent from this image).
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import uniform_filter

K1, K2, WIN = 0.01, 0.03, 7


def psnr(image_true: np.ndarray, image_test: np.ndarray, data_range: float) -> float:
    """skimage.metrics.peak_signal_noise_ratio (fp32 difference, float64 mean)."""
    a = np.asarray(image_true, dtype=np.float32)
    b = np.asarray(image_test, dtype=np.float32)
    err = np.mean((a - b) ** 2, dtype=np.float64)
    with np.errstate(divide="ignore"):
        return float(10 * np.log10((data_range ** 2) / err))


def _ssim_plane(x: np.ndarray, y: np.ndarray, data_range: float) -> float:
    x = x.astype(np.float32)
    y = y.astype(np.float32)
    ndim = x.ndim
    NP = WIN ** ndim
    cov_norm = NP / (NP - 1)
    ux = uniform_filter(x, size=WIN)
    uy = uniform_filter(y, size=WIN)
    uxx = uniform_filter(x * x, size=WIN)
    uyy = uniform_filter(y * y, size=WIN)
    uxy = uniform_filter(x * y, size=WIN)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    R = data_range
    C1 = (K1 * R) ** 2
    C2 = (K2 * R) ** 2
    A1, A2, B1, B2 = (2 * ux * uy + C1, 2 * vxy + C2, ux ** 2 + uy ** 2 + C1, vx + vy + C2)
    S = (A1 * A2) / (B1 * B2)
    pad = (WIN - 1) // 2
    return float(S[pad:-pad, pad:-pad].mean(dtype=np.float64))


def ssim(im1: np.ndarray, im2: np.ndarray, data_range: float, channel_axis: int | None = None) -> float:
    """skimage.metrics.structural_similarity, uniform 7x7 window, sample covariance."""
    if channel_axis is None:
        return _ssim_plane(im1, im2, data_range)
    a = np.moveaxis(np.asarray(im1), channel_axis, -1)
    b = np.moveaxis(np.asarray(im2), channel_axis, -1)
    return float(np.mean([_ssim_plane(a[..., c], b[..., c], data_range) for c in range(a.shape[-1])]))


def ssim_bruteforce(im1: np.ndarray, im2: np.ndarray, data_range: float) -> float:
    """Independent float64 loop over every interior 7x7 window of an HxWxC pair."""
    a = np.asarray(im1, dtype=np.float64)
    b = np.asarray(im2, dtype=np.float64)
    H, W, C = a.shape
    C1, C2 = (K1 * data_range) ** 2, (K2 * data_range) ** 2
    n = WIN * WIN
    out = []
    for c in range(C):
        acc = 0.0
        for y in range(3, H - 3):
            for x in range(3, W - 3):
                wa = a[y - 3:y + 4, x - 3:x + 4, c]
                wb = b[y - 3:y + 4, x - 3:x + 4, c]
                ux, uy = wa.mean(), wb.mean()
                vx = ((wa - ux) ** 2).sum() / (n - 1)
                vy = ((wb - uy) ** 2).sum() / (n - 1)
                vxy = ((wa - ux) * (wb - uy)).sum() / (n - 1)
                acc += ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2))
        out.append(acc / ((H - 6) * (W - 6)))
    return float(np.mean(out))


def batch_metrics(gt: np.ndarray, x: np.ndarray, data_range: float):
    """Per-image (psnr, ssim) of NCHW batches, as evaluate_model computes them per
    block after the CHW -> HWC transpose (evaluate_SIDD.py:59-64)."""
    ps, ss = [], []
    for g, o in zip(gt, x):
        ps.append(psnr(g, o, data_range))
        ss.append(ssim(g, o, data_range, channel_axis=0))
    return np.array(ps), np.array(ss)
