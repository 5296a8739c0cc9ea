"""MI355X-native drop-in for the network of ``UNet/RDUNet_model.py``.

``RDUNet(channels=3, base_filters=64)`` (RDUNet_model.py:117-186): the same
residual-dense UNet without the timestep channel; ``forward(inputs)`` returns
``output_block(...) + inputs``.  The reference module's import-time side
effects (building ``RDUNet(128)`` + AdamW + StepLR and its L1 training loop,
:189-261) are the baseline model's trainer, outside the diffusion hot path.
"""
from __future__ import annotations

from .engine import run_unet
from .Unet_model import (DenoisingBlock, DownsampleBlock, InputBlock, OutputBlock,  # noqa: F401
                         UpsampleBlock, _RDUNetBase, init_weights)


class RDUNet(_RDUNetBase):
    def __init__(self, channels=3, base_filters=64):
        super().__init__()
        if not 1 <= channels <= 8:
            raise ValueError("RDUNet supports 1..8 image channels")
        self._build(channels, base_filters, channels)
        self.time_conditioned = False
        self.image_channels = channels

    def forward(self, inputs):
        return run_unet(self, inputs, None)


def denormalize(tensor):
    """RDUNet_model.py:197-198."""
    return tensor * 0.5 + 0.5
