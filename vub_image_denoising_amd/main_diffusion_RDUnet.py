"""Drop-in for the definitions ``diffusion_denoising/main_diffusion_RDUnet.py``
declares inline (:24-352): the network classes, ``DiffusionModel``, the losses,
``denormalize``, and this script's own trainer signatures, which differ from
``diffusion_RDUnet.py``'s:

* ``train_step_checkpointed(model, clean, noisy, optimizer, accumulation_steps,
  clip_value=0.1)`` — uniform t only (:237-273);
* ``train_model_checkpointed(model, train_loader, val_loader, optimizer, scheduler,
  writer, num_epochs=10, start_epoch=0, accumulation_steps=4, clip_value=1.0)`` —
  improved_sampling validation, checkpoints under ``checkpoints/`` (:275-336);
* ``load_checkpoint(model, optimizer, scheduler, checkpoint_path)`` — restores
  the scheduler unconditionally (:339-352).

The script's module-level model / Adam(2e-4) / CosineAnnealingLR(T_max=10)
(:228-231) stay in the user's script; ``make_training_objects`` builds the same
four objects for callers that want them.
"""
from __future__ import annotations

import os

import torch
import torch.optim as optim
from torch.optim.lr_scheduler import CosineAnnealingLR

from .diffusion_RDUnet import (DiffusionModel, charbonnier_loss, combined_loss, denormalize, device,  # noqa: F401
                               run_epochs, train_step_device)
from .Unet_model import (DenoisingBlock, DownsampleBlock, InputBlock, OutputBlock, RDUNet_T,  # noqa: F401
                         UpsampleBlock, init_weights)

CHECKPOINT_DIR = "checkpoints"


def make_training_objects(base_filters=32, lr=2e-4, dev=None, model_cls=None):
    """main_diffusion_RDUnet.py:228-231: RDUNet_T(32), DiffusionModel, Adam(lr, (0.9, 0.999)),
    CosineAnnealingLR(T_max=10)."""
    dev = dev or device
    unet = RDUNet_T(base_filters=base_filters).to(dev)
    model = (model_cls or DiffusionModel)(unet).to(dev)
    optimizer = optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999))
    scheduler = CosineAnnealingLR(optimizer, T_max=10)
    return unet, model, optimizer, scheduler


def train_step_checkpointed(model, clean_images, noisy_images, optimizer, accumulation_steps, clip_value=0.1):
    """main_diffusion_RDUnet.py:237-273 (uniform t; returns ``loss.item()``)."""
    return train_step_device(model, clean_images, noisy_images, optimizer, 'uniform', clip_value).item()


def _sample(model, x):
    return model.improved_sampling(x)


def train_model_checkpointed(model, train_loader, val_loader, optimizer, scheduler, writer, num_epochs=10,
                             start_epoch=0, accumulation_steps=4, clip_value=1.0, *, accumulation='reference'):
    """main_diffusion_RDUnet.py:275-336."""
    run_epochs(model, train_loader, val_loader, optimizer, scheduler, writer, CHECKPOINT_DIR, 'uniform', num_epochs,
               start_epoch, accumulation_steps, clip_value, 1, sample=_sample, accumulation=accumulation)


def load_checkpoint(model, optimizer, scheduler, checkpoint_path):
    """main_diffusion_RDUnet.py:339-352 (weights-only safe load)."""
    if os.path.isfile(checkpoint_path):
        print(f"Loading checkpoint '{checkpoint_path}'")
        dev = next(model.parameters()).device
        checkpoint = torch.load(checkpoint_path, map_location=dev, weights_only=True)
        model.load_state_dict(checkpoint['model_state_dict'])
        optimizer.load_state_dict(checkpoint['optimizer_state_dict'])
        scheduler.load_state_dict(checkpoint['scheduler_state_dict'])
        start_epoch = checkpoint['epoch']
        print(f"Loaded checkpoint '{checkpoint_path}' (epoch {start_epoch})")
        return start_epoch
    print(f"No checkpoint found at '{checkpoint_path}'")
    return 0
