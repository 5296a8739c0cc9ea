"""CPU restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

Pure ``torch.nn.functional`` on the CPU, NCHW activations / OIHW weights, in
fp32 (or fp64 for error-budget checks).  It restates, in this build's own
words, the math of:

* the residual-dense UNet blocks ``diffusion_denoising/Unet/Unet_model.py:23-89``
  (Downsample :23-30, Upsample :32-43, Input :45-55, Output :57-67,
  Denoising :69-89) and the networks ``RDUNet_T`` (:92-166) and the plain
  ``RDUNet`` (``UNet/RDUNet_model.py:117-186``);
* the cold-diffusion wrapper ``diffusion_denoising/diffusion_RDUnet.py:27-55``
  (``forward_diffusion`` :33-36, ``improved_sampling`` :38-50) and
  ``direct_sampling`` (``diffusion_denoising/diffusion_RDUnet_direct.py:198-201``);
* the losses ``charbonnier_loss`` / ``combined_loss`` (:57-65);
* the training step ``train_step_checkpointed`` (:76-115): interpolation,
  UNet forward, loss, backward, global-norm gradient clipping.

Parameters are a flat ``{state_dict key: tensor}`` mapping whose keys are the
reference's (``input_block.conv_1.weight`` …), optionally prefixed (``unet.``).
Only tests / smoke / bench's cpu_baseline use this module.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

__all__ = [
    "param_shapes", "rdunet_t_forward", "rdunet_forward", "charbonnier_loss",
    "combined_loss", "improved_sampling", "direct_sampling", "train_step",
    "clip_grad_norm",
]

_LEVEL_BLOCKS = [
    ("input_block", "input"),
    ("block_0_0", 0), ("block_0_1", 0), ("down_0", "down0"),
    ("block_1_0", 1), ("block_1_1", 1), ("down_1", "down1"),
    ("block_2_0", 2), ("block_2_1", 2), ("down_2", "down2"),
    ("block_3_0", 3), ("block_3_1", 3),
    ("up_2", "up2"), ("block_2_2", 2), ("block_2_3", 2),
    ("up_1", "up1"), ("block_1_2", 1), ("block_1_3", 1),
    ("up_0", "up0"), ("block_0_2", 0), ("block_0_3", 0),
    ("output_block", "output"),
]


def param_shapes(base_filters: int = 64, channels: int = 4, out_channels: int = 3) -> "OrderedDict[str, tuple]":
    """state_dict key → shape, in the reference's registration order.

    ``RDUNet_T``: channels=4, out_channels=3 (``Unet_model.py:100,128``);
    ``RDUNet``: channels=3, out_channels=channels (``RDUNet_model.py:125,153``).
    """
    f = [base_filters * (1 << i) for i in range(4)]
    s = OrderedDict()

    def conv(name, cin, cout, k):
        s[name + ".weight"] = (cout, cin, k, k)
        s[name + ".bias"] = (cout,)

    def convt(name, cin, cout, k):
        s[name + ".weight"] = (cin, cout, k, k)
        s[name + ".bias"] = (cout,)

    def prelu(name, c):
        s[name + ".weight"] = (c,)

    for name, kind in _LEVEL_BLOCKS:
        if kind == "input":
            conv(name + ".conv_1", channels, f[0], 3)
            conv(name + ".conv_2", f[0], f[0], 3)
            prelu(name + ".actv_1", f[0]); prelu(name + ".actv_2", f[0])
        elif kind == "output":
            conv(name + ".conv_1", f[0], f[0], 3)
            conv(name + ".conv_2", f[0], out_channels, 3)
            prelu(name + ".actv_1", f[0]); prelu(name + ".actv_2", out_channels)
        elif isinstance(kind, int):
            c, i = f[kind], f[kind] // 2
            conv(name + ".conv_0", c, i, 3)
            conv(name + ".conv_1", c + i, i, 3)
            conv(name + ".conv_2", c + 2 * i, i, 3)
            conv(name + ".conv_3", c + 3 * i, c, 3)
            for k in range(3):
                prelu(name + f".actv_{k}", i)
            prelu(name + ".actv_3", c)
        elif kind.startswith("down"):
            lvl = int(kind[-1])
            conv(name + ".conv", f[lvl], f[lvl + 1], 2)
            prelu(name + ".actv", f[lvl + 1])
        elif kind.startswith("up"):
            lvl = int(kind[-1])  # up_l: in=f[l+1], cat=f[l], out=f[l]
            cin, ccat, cout = f[lvl + 1], f[lvl], f[lvl]
            conv(name + ".conv", cin + ccat, cout, 3)
            convt(name + ".conv_t", cin, cin, 2)
            prelu(name + ".actv", cout)
            prelu(name + ".actv_t", cin)
    return s


def _p(params, prefix, name):
    return params[prefix + name]


def _conv3(params, prefix, name, x):
    return F.conv2d(x, _p(params, prefix, name + ".weight"), _p(params, prefix, name + ".bias"), padding=1)


def _prelu(params, prefix, name, x):
    return F.prelu(x, _p(params, prefix, name + ".weight"))


def _input_block(params, pre, x):          # Unet_model.py:53-55
    x = _prelu(params, pre, "actv_1", _conv3(params, pre, "conv_1", x))
    return _prelu(params, pre, "actv_2", _conv3(params, pre, "conv_2", x))


_output_block = _input_block               # Unet_model.py:65-67 (same dataflow)


def _dense_block(params, pre, x):          # Unet_model.py:81-89
    buf = x
    for k in range(3):
        o = _prelu(params, pre, f"actv_{k}", _conv3(params, pre, f"conv_{k}", buf))
        buf = torch.cat([buf, o], 1)
    return _prelu(params, pre, "actv_3", _conv3(params, pre, "conv_3", buf)) + x


def _down(params, pre, x):                 # Unet_model.py:29-30
    y = F.conv2d(x, _p(params, pre, "conv.weight"), _p(params, pre, "conv.bias"), stride=2)
    return _prelu(params, pre, "actv", y)


def _up(params, pre, low, skip):           # Unet_model.py:40-43
    u = F.conv_transpose2d(low, _p(params, pre, "conv_t.weight"), _p(params, pre, "conv_t.bias"), stride=2)
    u = _prelu(params, pre, "actv_t", u)
    y = F.conv2d(torch.cat([skip, u], 1), _p(params, pre, "conv.weight"), _p(params, pre, "conv.bias"), padding=1)
    return _prelu(params, pre, "actv", y)


def _unet(params, prefix, x, inputs):
    """Shared topology of RDUNet_T.forward (Unet_model.py:138-166) and
    RDUNet.forward (RDUNet_model.py:157-186)."""
    P = lambda n: prefix + n + "."
    o0 = _input_block(params, P("input_block"), x)
    o0 = _dense_block(params, P("block_0_0"), o0)
    o0 = _dense_block(params, P("block_0_1"), o0)
    o1 = _down(params, P("down_0"), o0)
    o1 = _dense_block(params, P("block_1_0"), o1)
    o1 = _dense_block(params, P("block_1_1"), o1)
    o2 = _down(params, P("down_1"), o1)
    o2 = _dense_block(params, P("block_2_0"), o2)
    o2 = _dense_block(params, P("block_2_1"), o2)
    o3 = _down(params, P("down_2"), o2)
    o3 = _dense_block(params, P("block_3_0"), o3)
    o3 = _dense_block(params, P("block_3_1"), o3)
    o4 = _up(params, P("up_2"), o3, o2)
    o4 = _dense_block(params, P("block_2_2"), o4)
    o4 = _dense_block(params, P("block_2_3"), o4)
    o5 = _up(params, P("up_1"), o4, o1)
    o5 = _dense_block(params, P("block_1_2"), o5)
    o5 = _dense_block(params, P("block_1_3"), o5)
    o6 = _up(params, P("up_0"), o5, o0)
    o6 = _dense_block(params, P("block_0_2"), o6)
    o6 = _dense_block(params, P("block_0_3"), o6)
    return _output_block(params, P("output_block"), o6) + inputs


def rdunet_t_forward(params, inputs, t, prefix=""):
    """RDUNet_T.forward (Unet_model.py:133-166): t broadcast to a 4th channel."""
    t = t.expand(inputs.size(0), 1, inputs.size(2), inputs.size(3))
    x = torch.cat((inputs, t), dim=1)
    return _unet(params, prefix, x, inputs)


def rdunet_forward(params, inputs, prefix=""):
    """RDUNet.forward (UNet/RDUNet_model.py:157-186)."""
    return _unet(params, prefix, inputs, inputs)


def charbonnier_loss(pred, target, epsilon=1e-3):
    """diffusion_RDUnet.py:57-58."""
    return torch.mean(torch.sqrt((pred - target) ** 2 + epsilon ** 2))


def combined_loss(pred, target, mse_weight=0, charbonnier_weight=1, ssim_weight=0, epsilon=1e-3):
    """diffusion_RDUnet.py:60-65 with the SSIM term (weight 0 in every caller)
    omitted: for finite inputs 0·(1−SSIM) is exactly 0."""
    if ssim_weight != 0:
        raise NotImplementedError("oracle covers ssim_weight == 0 only")
    mse = torch.mean((pred - target) ** 2)
    return mse_weight * mse + charbonnier_weight * charbonnier_loss(pred, target, epsilon)


def improved_sampling(unet_fn, noisy_image, timesteps):
    """DiffusionModel.improved_sampling (diffusion_RDUnet.py:38-50).
    ``unet_fn(x, t_tensor)`` with t_tensor of shape [1,1,1,1]."""
    x_t = noisy_image
    for t in reversed(range(1, timesteps + 1)):
        a, ap = t / timesteps, (t - 1) / timesteps
        tt = torch.tensor([a], dtype=noisy_image.dtype).view(1, 1, 1, 1)
        ttp = torch.tensor([ap], dtype=noisy_image.dtype).view(1, 1, 1, 1)
        x_tilde = (1 - a) * unet_fn(x_t, tt) + a * noisy_image
        x_tilde_prev = (1 - ap) * unet_fn(x_t, ttp) + ap * noisy_image
        x_t = x_t - x_tilde + x_tilde_prev
    return x_t


def direct_sampling(unet_fn, noisy_image):
    """diffusion_RDUnet_direct.py:198-201: one UNet call at t = 1."""
    t = torch.tensor([1.0], dtype=noisy_image.dtype).view(1, 1, 1, 1)
    return unet_fn(noisy_image, t)


def clip_grad_norm(grads, max_norm, eps=1e-6):
    """torch.nn.utils.clip_grad_norm_ semantics (diffusion_RDUnet.py:113):
    total = ||[g...]||_2; coef = min(max_norm/(total+1e-6), 1); g *= coef."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
    coef = torch.clamp(max_norm / (total + eps), max=1.0)
    return total, [g * coef for g in grads]


def train_step(params, clean, noisy, t_int, timesteps, clip_value=1.0, prefix=""):
    """train_step_checkpointed (diffusion_RDUnet.py:76-115) with the timestep
    draw made explicit (``t_int`` integer steps, shape [B]).

    Returns (loss, denoised, {name: clipped grad}, total_norm)."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    B = clean.size(0)
    t_norm = t_int.to(clean.dtype) / timesteps                          # :90
    t_tensor = t_norm.view(B, 1, 1, 1).expand(-1, 1, clean.size(2), clean.size(3))  # :93
    x = t_tensor * noisy + (1 - t_tensor) * clean                        # :99-100
    y = rdunet_t_forward(leaves, x, t_tensor, prefix)                    # :106
    loss = combined_loss(y, clean)                                       # :109
    loss.backward()                                                      # :110
    names = list(leaves.keys())
    total, clipped = clip_grad_norm([leaves[n].grad for n in names], clip_value)  # :113
    return loss.detach(), y.detach(), dict(zip(names, clipped)), total
