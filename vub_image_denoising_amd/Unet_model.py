"""MI355X-native drop-in for ``diffusion_denoising/Unet/Unet_model.py``.

Same class names, constructor signatures, child-module names and registration
order as the reference, so

* ``state_dict`` keys / shapes are identical (207 tensors, e.g.
  ``block_0_0.conv_1.weight``), and checkpoints round-trip both ways;
* ``torch.manual_seed(s); RDUNet_T(...)`` draws the same initial weights as the
  reference (same module construction order, same ``init_weights`` pass).

``RDUNet_T.forward`` runs the whole network as one fused launch sequence of
hand-written gfx950 kernels (``engine.py`` → ``librdunet_hip.so``); a block's
own ``forward`` runs that block alone through the same engine and kernels.
There is no PyTorch-op or CPU path.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .engine import run_block, run_unet


@torch.no_grad()
def init_weights(init_type='xavier'):
    """Unet_model.py:4-21: xavier/he/orthogonal init of every module whose class
    name contains "Conv2d" (ConvTranspose2d included); biases keep PyTorch's
    default.  The BatchNorm branch is kept for API parity (no BN in the nets)."""
    if init_type == 'xavier':
        init = nn.init.xavier_normal_
    elif init_type == 'he':
        init = nn.init.kaiming_normal_
    else:
        init = nn.init.orthogonal_

    def initializer(m):
        classname = m.__class__.__name__
        if 'Conv2d' in classname:
            init(m.weight)
        elif 'BatchNorm' in classname:
            nn.init.normal_(m.weight, 1.0, 0.01)
            nn.init.zeros_(m.bias)

    return initializer


_RUNTIME = ("_rdn_flat", "_rdn_packs", "_rdn_engines", "_rdn_prog")


class _GpuBlock:
    """A block's own forward: the block as a Program of the fused engine
    (engine.block_program) — NCHW fp32 in/out, same kernels as inside the
    network, autograd through inputs and parameters."""
    compute_dtype = torch.float32

    def set_compute_dtype(self, dtype):
        dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}.get(dtype, dtype)
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute dtype must be fp32 or bf16, got {dtype}")
        self.compute_dtype = dtype
        return self

    def forward(self, x):
        return run_block(self, [x])

    def __getstate__(self):  # engines / packs are runtime state, not pickled
        d = self.__dict__.copy()
        for k in _RUNTIME:
            d.pop(k, None)
        return d


class DownsampleBlock(_GpuBlock, nn.Module):
    """Unet_model.py:23-30: Conv2d(k=2, s=2) + PReLU."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=2, stride=2)
        self.actv = nn.PReLU(out_channels)


class UpsampleBlock(_GpuBlock, nn.Module):
    """Unet_model.py:32-43: ConvTranspose2d(k=2, s=2) + PReLU, cat with the
    skip, Conv2d 3x3 + PReLU."""

    def __init__(self, in_channels, cat_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels + cat_channels, out_channels, 3, padding=1)
        self.conv_t = nn.ConvTranspose2d(in_channels, in_channels, 2, stride=2)
        self.actv = nn.PReLU(out_channels)
        self.actv_t = nn.PReLU(in_channels)

    def forward(self, x):
        upsample, concat = x
        return run_block(self, [upsample, concat])


class InputBlock(_GpuBlock, nn.Module):
    """Unet_model.py:45-55: two Conv2d 3x3 + PReLU."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv_1 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.conv_2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.actv_1 = nn.PReLU(out_channels)
        self.actv_2 = nn.PReLU(out_channels)


class OutputBlock(_GpuBlock, nn.Module):
    """Unet_model.py:57-67: Conv2d 3x3 + PReLU, Conv2d 3x3 + PReLU."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv_1 = nn.Conv2d(in_channels, in_channels, 3, padding=1)
        self.conv_2 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.actv_1 = nn.PReLU(in_channels)
        self.actv_2 = nn.PReLU(out_channels)


class DenoisingBlock(_GpuBlock, nn.Module):
    """Unet_model.py:69-89: residual dense block (4 convs 3x3 + PReLU, dense
    concatenation, ``out_3 + x``)."""

    def __init__(self, in_channels, inner_channels, out_channels):
        super().__init__()
        self.conv_0 = nn.Conv2d(in_channels, inner_channels, 3, padding=1)
        self.conv_1 = nn.Conv2d(in_channels + inner_channels, inner_channels, 3, padding=1)
        self.conv_2 = nn.Conv2d(in_channels + 2 * inner_channels, inner_channels, 3, padding=1)
        self.conv_3 = nn.Conv2d(in_channels + 3 * inner_channels, out_channels, 3, padding=1)
        self.actv_0 = nn.PReLU(inner_channels)
        self.actv_1 = nn.PReLU(inner_channels)
        self.actv_2 = nn.PReLU(inner_channels)
        self.actv_3 = nn.PReLU(out_channels)


class _RDUNetBase(nn.Module):
    def _build(self, channels, base_filters, out_channels):
        filters_0 = base_filters
        filters_1 = 2 * filters_0
        filters_2 = 4 * filters_0
        filters_3 = 8 * filters_0

        self.input_block = InputBlock(channels, filters_0)
        self.block_0_0 = DenoisingBlock(filters_0, filters_0 // 2, filters_0)
        self.block_0_1 = DenoisingBlock(filters_0, filters_0 // 2, filters_0)
        self.down_0 = DownsampleBlock(filters_0, filters_1)

        self.block_1_0 = DenoisingBlock(filters_1, filters_1 // 2, filters_1)
        self.block_1_1 = DenoisingBlock(filters_1, filters_1 // 2, filters_1)
        self.down_1 = DownsampleBlock(filters_1, filters_2)

        self.block_2_0 = DenoisingBlock(filters_2, filters_2 // 2, filters_2)
        self.block_2_1 = DenoisingBlock(filters_2, filters_2 // 2, filters_2)
        self.down_2 = DownsampleBlock(filters_2, filters_3)

        self.block_3_0 = DenoisingBlock(filters_3, filters_3 // 2, filters_3)
        self.block_3_1 = DenoisingBlock(filters_3, filters_3 // 2, filters_3)

        self.up_2 = UpsampleBlock(filters_3, filters_2, filters_2)
        self.block_2_2 = DenoisingBlock(filters_2, filters_2 // 2, filters_2)
        self.block_2_3 = DenoisingBlock(filters_2, filters_2 // 2, filters_2)

        self.up_1 = UpsampleBlock(filters_2, filters_1, filters_1)
        self.block_1_2 = DenoisingBlock(filters_1, filters_1 // 2, filters_1)
        self.block_1_3 = DenoisingBlock(filters_1, filters_1 // 2, filters_1)

        self.up_0 = UpsampleBlock(filters_1, filters_0, filters_0)
        self.block_0_2 = DenoisingBlock(filters_0, filters_0 // 2, filters_0)
        self.block_0_3 = DenoisingBlock(filters_0, filters_0 // 2, filters_0)

        self.output_block = OutputBlock(filters_0, out_channels)

        self.apply(init_weights())

        self.base_filters = base_filters
        self.out_channels = out_channels
        # arithmetic of the kernels: torch.float32 (reference numerics, parity
        # mode) or torch.bfloat16 (bf16 activations/MFMA, fp32 accumulate and
        # fp32 master weights)
        self.compute_dtype = torch.float32

    def set_compute_dtype(self, dtype):
        dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}.get(dtype, dtype)
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute dtype must be fp32 or bf16, got {dtype}")
        self.compute_dtype = dtype
        return self

    def mark_weights_dirty(self):
        """Parameters were written where torch's version counters do not see it
        (``p.data.copy_(...)``, raw pointers): rebuild the GEMM weight packs on
        the next forward.  Optimizer steps, ``load_state_dict`` and in-place ops
        on the parameters themselves are tracked without this."""
        fp = getattr(self, "_rdn_flat", None)
        if fp is not None:
            fp.generation += 1
        return self

    def __getstate__(self):  # engines / flat buffers are runtime state, not pickled
        d = self.__dict__.copy()
        for k in _RUNTIME:
            d.pop(k, None)
        return d


class RDUNet_T(_RDUNetBase):
    """Time-conditioned residual-dense UNet, Unet_model.py:92-166.

    ``forward(inputs [B,3,H,W], t)``: t broadcastable to [B,1,H,W] (a per-image
    map [B,1,H,W] in training, [1,1,1,1] in sampling); it becomes the 4th input
    channel.  Output ``output_block(...) + inputs``, [B,3,H,W] fp32."""

    def __init__(self, channels=4, base_filters=64):
        super().__init__()
        if channels != 4:
            raise ValueError("RDUNet_T expects channels=4 (3 image channels + t), as the reference's "
                             "residual `+ inputs` with a 3-channel output requires")
        self._build(channels, base_filters, 3)
        self.time_conditioned = True
        self.image_channels = channels - 1

    def forward(self, inputs, t):
        return run_unet(self, inputs, t)
