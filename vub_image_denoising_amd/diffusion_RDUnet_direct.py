"""Drop-in for the definitions ``diffusion_denoising/diffusion_RDUnet_direct.py``
declares inline (:24-343).  It differs from ``main_diffusion_RDUnet.py`` in one
place: the model denoises with a single UNet call at t = 1 —
``DiffusionModel.direct_sampling`` (:198-201) — which is also what its
``forward`` (:203-206) and its trainer's one-batch validation (:290) run.
"""
from __future__ import annotations

from . import diffusion_RDUnet as _base
from .diffusion_RDUnet import (charbonnier_loss, combined_loss, denormalize, device, run_epochs,  # noqa: F401
                               train_step_device)
from . import main_diffusion_RDUnet as _main
from .main_diffusion_RDUnet import CHECKPOINT_DIR, load_checkpoint, train_step_checkpointed  # noqa: F401
from .Unet_model import (DenoisingBlock, DownsampleBlock, InputBlock, OutputBlock, RDUNet_T,  # noqa: F401
                         UpsampleBlock, init_weights)


class DiffusionModel(_base.DiffusionModel):
    """diffusion_RDUnet_direct.py:187-206: forward = forward_diffusion + direct_sampling."""

    def forward(self, clean_image, noisy_image, t):
        noisy_step_image = self.forward_diffusion(clean_image, noisy_image, t)
        return self.direct_sampling(noisy_step_image)


def make_training_objects(base_filters=32, lr=2e-4, dev=None):
    """diffusion_RDUnet_direct.py:219-222 (same objects as main_diffusion_RDUnet.py:228-231)."""
    return _main.make_training_objects(base_filters, lr, dev, model_cls=DiffusionModel)


def _sample(model, x):
    return model.direct_sampling(x)


def train_model_checkpointed(model, train_loader, val_loader, optimizer, scheduler, writer, num_epochs=10,
                             start_epoch=0, accumulation_steps=4, clip_value=1.0, *, accumulation='reference'):
    """diffusion_RDUnet_direct.py:266-327 (validation with direct_sampling)."""
    run_epochs(model, train_loader, val_loader, optimizer, scheduler, writer, CHECKPOINT_DIR, 'uniform', num_epochs,
               start_epoch, accumulation_steps, clip_value, 1, sample=_sample, accumulation=accumulation)
