"""Device-side pieces of the train / sample step around the UNet, each one
``librdunet_hip`` launch (no host sync):

* ``interpolate``      — ``alpha*noisy + (1-alpha)*clean`` (diffusion_RDUnet.py:99-100, :33-36)
* ``charbonnier_loss`` / ``combined_loss`` — diffusion_RDUnet.py:57-65, fused
  forward reduction (Charbonnier and MSE in one pass) and fused backward
* ``clip_grad_norm_``  — torch.nn.utils.clip_grad_norm_ (diffusion_RDUnet.py:113)
  on the flat gradient buffer: one norm reduction + one scale, coefficient kept
  on the device
* ``sampling_combine`` — the x_t update of improved_sampling (:45-49)
"""
from __future__ import annotations

import math

import torch

from . import _hip as H
from .engine import FlatParams, find_flat


def _f32c(t):
    t = t.contiguous()
    return t if t.dtype == torch.float32 else t.float()


def interpolate(clean: torch.Tensor, noisy: torch.Tensor, tnorm: torch.Tensor) -> torch.Tensor:
    """x[b] = tnorm[b]*noisy[b] + (1 - tnorm[b])*clean[b] for per-image tnorm [B]."""
    H.require_device(clean, noisy, tnorm)
    clean, noisy = _f32c(clean), _f32c(noisy)
    B = clean.size(0)
    tn = _f32c(tnorm.reshape(-1))
    if tn.numel() != B or clean.shape != noisy.shape:
        raise RuntimeError("interpolate: need per-image t and matching clean/noisy shapes")
    per = clean[0].numel()
    if per % 4:
        raise RuntimeError("interpolate: image size must be a multiple of 4 elements")
    x = torch.empty_like(clean)
    H.check(H.lib().rdn_interp(clean.data_ptr(), noisy.data_ptr(), tn.data_ptr(), B, per, x.data_ptr(),
                               H.stream_ptr()), "interp")
    return x


class _CombinedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, wm, wc, eps):
        pred, target = _f32c(pred), _f32c(target)
        n = pred.numel()
        lib = H.lib()
        ws = torch.empty(max(lib.rdn_reduce_workspace_size(n) // 4, 1), dtype=torch.float32, device=pred.device)
        out = torch.empty(2, dtype=torch.float32, device=pred.device)
        H.check(lib.rdn_charbonnier_fwd(pred.data_ptr(), target.data_ptr(), n, eps, ws.data_ptr(), out.data_ptr(),
                                        H.stream_ptr()), "charbonnier_fwd")
        ctx.save_for_backward(pred, target)
        ctx.wm, ctx.wc, ctx.eps = float(wm), float(wc), float(eps)
        # mse_weight * mse + charbonnier_weight * charbonnier (diffusion_RDUnet.py:65)
        return ctx.wm * out[1] + ctx.wc * out[0]

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        g = _f32c(g.reshape(1))
        dp = torch.empty_like(pred)
        H.check(H.lib().rdn_charbonnier_bwd(pred.data_ptr(), target.data_ptr(), pred.numel(), ctx.eps, ctx.wc, ctx.wm,
                                            g.data_ptr(), dp.data_ptr(), H.stream_ptr()), "charbonnier_bwd")
        dt = -dp if ctx.needs_input_grad[1] else None
        return dp, dt, None, None, None


def charbonnier_loss(pred, target, epsilon=1e-3):
    """mean(sqrt((pred-target)^2 + eps^2)), diffusion_RDUnet.py:57-58."""
    H.require_device(pred, target)
    return _CombinedLoss.apply(pred, target, 0.0, 1.0, epsilon)


def ssim(x, y, data_range=1.0, win_size=11, win_sigma=1.5, K=(0.01, 0.03)):
    """pytorch_msssim.ssim (v1.0.0) restated with torch ops (gaussian 11x11,
    sigma 1.5, valid padding, size_average).  Only evaluated when
    ``ssim_weight != 0``; every reference caller uses weight 0."""
    C = x.size(1)
    coords = torch.arange(win_size, dtype=x.dtype, device=x.device) - win_size // 2
    g = torch.exp(-(coords ** 2) / (2 * win_sigma ** 2))
    g = (g / g.sum()).view(1, 1, 1, -1).repeat(C, 1, 1, 1)

    def filt(t):
        t = torch.nn.functional.conv2d(t, g, groups=C)
        return torch.nn.functional.conv2d(t, g.transpose(2, 3), groups=C)

    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    mu1, mu2 = filt(x), filt(y)
    s11 = filt(x * x) - mu1 * mu1
    s22 = filt(y * y) - mu2 * mu2
    s12 = filt(x * y) - mu1 * mu2
    cs = (2 * s12 + C2) / (s11 + s22 + C2)
    ssim_map = ((2 * mu1 * mu2 + C1) / (mu1 * mu1 + mu2 * mu2 + C1)) * cs
    return torch.flatten(ssim_map, 2).mean(-1).mean()


def combined_loss(pred, target, mse_weight=0, charbonnier_weight=1, ssim_weight=0, epsilon=1e-3):
    """diffusion_RDUnet.py:60-65.  MSE and Charbonnier come out of one fused
    reduction; the weight-0 MSE term is still evaluated so a NaN/inf in pred
    propagates exactly as in the reference (0*inf = NaN)."""
    H.require_device(pred, target)
    loss = _CombinedLoss.apply(pred, target, float(mse_weight), float(charbonnier_weight), epsilon)
    if ssim_weight != 0:
        loss = loss + ssim_weight * (1 - ssim(pred, target, data_range=1.0))
    return loss


def clip_grad_norm_flat(fp: FlatParams, max_norm: float, pre_scale: float = 1.0, want_norm: bool = True):
    """Global L2 norm of the flat gradient and in-place scale by
    min(max_norm/(norm+1e-6), 1) — torch.nn.utils.clip_grad_norm_ semantics,
    without a host synchronisation.  Returns the (device) total norm.
    ``pre_scale``: a factor not yet applied to the gradient (the data-parallel
    1/world average, ddp.GradSync.defer_average), folded into the same scale pass.
    ``want_norm=False`` (the train step, which discards it): no copy of the norm out of
    the workspace (one launch less in the captured step); returns None."""
    lib = H.lib()
    ws = getattr(fp, "_clip_ws", None)
    if ws is None:
        ws = fp._clip_ws = torch.empty(lib.rdn_reduce_workspace_size(fp.numel) // 4 + 2, dtype=torch.float32,
                                       device=fp.device)
        fp._clip_out = torch.empty(2, dtype=torch.float32, device=fp.device)
    st = H.stream_ptr()
    H.check(lib.rdn_sqnorm_scaled(fp.gflat.data_ptr(), fp.numel, float(max_norm), float(pre_scale), ws.data_ptr(),
                                  fp._clip_out.data_ptr(), st), "sqnorm")
    H.check(lib.rdn_clip_scale(fp.gflat.data_ptr(), fp.numel, fp._clip_out[1:].data_ptr(), st), "clip_scale")
    return fp._clip_out[0].clone() if want_norm else None


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, want_norm=True):
    """torch.nn.utils.clip_grad_norm_ drop-in: the fused flat path when the
    parameters are one fused network's, torch's own otherwise."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = list(parameters)
    fp = find_flat(parameters) if norm_type == 2.0 else None
    if fp is not None:
        return clip_grad_norm_flat(fp, max_norm, want_norm=want_norm)
    return torch.nn.utils.clip_grad_norm_(parameters, max_norm, norm_type)


def sampling_combine(x_t, f1, f2, y, a, ap):
    """In place: x_t = x_t - ((1-a)*f1 + a*y) + ((1-ap)*f2 + ap*y); ``a``/``ap``
    are Python floats (1-a rounded in double first, as the reference's scalars)."""
    H.check(H.lib().rdn_sampling_combine(x_t.data_ptr(), f1.data_ptr(), f2.data_ptr(), y.data_ptr(), x_t.numel(),
                                         1.0 - a, a, 1.0 - ap, ap, H.stream_ptr()), "sampling_combine")
    return x_t


def psnr(pred, target):
    """hyperparams_search.py:11-16 convention: denormalise [-1,1] -> [0,1],
    20*log10(1/RMSE) (per batch)."""
    p = pred * 0.5 + 0.5
    t = target * 0.5 + 0.5
    mse = torch.mean((p - t) ** 2)
    return 20 * math.log10(1.0) - 10 * torch.log10(mse)
