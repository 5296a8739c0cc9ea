"""MI355X-native drop-in for ``diffusion_denoising/diffusion_RDUnet.py``
(and the identical definitions inlined in ``main_diffusion_RDUnet.py`` /
``diffusion_RDUnet_direct.py``).

Same names and signatures: ``DiffusionModel`` (forward_diffusion,
improved_sampling, direct_sampling, forward), ``charbonnier_loss``,
``combined_loss``, ``denormalize``, ``sample_biased``,
``train_step_checkpointed``, ``train_model_checkpointed``, ``load_checkpoint``,
``load_data(args)``, ``train(args, train_loader, val_loader)`` and the argparse
CLI (``python -m vub_image_denoising_amd.diffusion_RDUnet``).

Numerics follow the reference, including its two quirks:
``train_step_checkpointed`` zeroes gradients at its top, so with
``accumulation_steps=4`` only every 4th batch's (clipped) gradient reaches
``optimizer.step()`` (:78, :126-128); and the UNet's residual adds the
3-channel input after the output PReLU.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.distributions as dist
import torch.nn as nn
import torch.optim as optim
from torch.optim.lr_scheduler import CosineAnnealingLR

from . import functional as Fn
from .Unet_model import RDUNet_T, init_weights  # noqa: F401

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


class DiffusionModel(nn.Module):
    """diffusion_RDUnet.py:27-55 (+ direct_sampling, diffusion_RDUnet_direct.py:198-201)."""

    def __init__(self, unet, timesteps=20):
        super(DiffusionModel, self).__init__()
        self.unet = unet
        self.timesteps = timesteps

    def forward_diffusion(self, clean_image, noisy_image, t):
        alpha = t / self.timesteps
        if isinstance(alpha, torch.Tensor) and alpha.numel() == clean_image.size(0) and clean_image.is_cuda:
            return Fn.interpolate(clean_image, noisy_image, alpha.reshape(-1))
        return alpha * noisy_image + (1 - alpha) * clean_image

    def improved_sampling(self, noisy_image):
        """2T UNet forwards (t = T..1): x_t <- x_t - x~(t) + x~(t-1), :38-50."""
        from .sampling import improved_sampling
        return improved_sampling(self, noisy_image)

    def direct_sampling(self, noisy_image):
        t = torch.tensor([1.0], device=noisy_image.device).unsqueeze(0).unsqueeze(2).unsqueeze(3)
        return self.unet(noisy_image, t)

    def forward(self, clean_image, noisy_image, t):
        noisy_step_image = self.forward_diffusion(clean_image, noisy_image, t)
        return self.improved_sampling(noisy_step_image)


charbonnier_loss = Fn.charbonnier_loss
combined_loss = Fn.combined_loss


def denormalize(tensor):
    return tensor * 0.5 + 0.5


def sample_biased(num_samples, timesteps, alpha=2.0):
    """Beta(alpha, 1) * timesteps, drawn on the CPU as the reference does (:71-73)."""
    beta_dist = dist.Beta(alpha, 1.0)
    return beta_dist.sample((num_samples,)) * timesteps


def _draw_t(batch_size, timesteps, distribution_choice, dev):
    if distribution_choice == 'biased':
        return sample_biased(batch_size, timesteps).to(dev)
    return torch.randint(0, timesteps + 1, (batch_size,), device=dev).float()


def _forward_loss(model, clean_images, noisy_images, distribution_choice, t):
    B = clean_images.size(0)
    T = model.timesteps
    if t is None:
        t = _draw_t(B, T, distribution_choice, clean_images.device)
    t_normalized = t.to(device=clean_images.device, dtype=torch.float32) / T           # :90
    interpolated = Fn.interpolate(clean_images, noisy_images, t_normalized)            # :99-100
    t_tensor = t_normalized.view(B, 1, 1, 1).expand(-1, 1, clean_images.size(2), clean_images.size(3))  # :93
    denoised = model.unet(interpolated, t_tensor)                                      # :106
    return combined_loss(denoised, clean_images)                                       # :109


def train_step_device(model, clean_images, noisy_images, optimizer, distribution_choice='uniform',
                      clip_value=0.1, t=None, zero_grad=True, clip=True):
    """The body of train_step_checkpointed without the host sync: returns the
    loss as a device tensor.  ``t`` (integer steps, [B]) overrides the draw.
    ``zero_grad=False, clip=False`` accumulates into the existing gradients
    (the fixed accumulation mode of run_epochs)."""
    model.train()
    if zero_grad:
        optimizer.zero_grad()
    loss = _forward_loss(model, clean_images, noisy_images, distribution_choice, t)
    # data-parallel: the clip right after the backward also applies the 1/world
    # average of the all-reduced gradient (one pass instead of two, ddp.py)
    # -- only when the gradients are this backward's alone (zero_grad): accumulated
    # ones already hold averaged sums from earlier calls, which must not be scaled again
    fp = getattr(model.unet, "_rdn_flat", None)
    sync = getattr(fp, "grad_sync", None) if clip else None
    fold = sync is not None and sync.world > 1 and zero_grad
    if fold:
        sync.defer_average = True
    try:
        loss.backward()                                                                # :110
    finally:
        if fold:
            sync.defer_average = False
    if clip:
        pre = sync.take_pending() if fold else None
        params = list(model.parameters())
        flat = Fn.find_flat(params) if pre is not None else None
        if pre is not None and flat is None:
            sync._average()   # gradients not the flat views: average them first
            pre = None
        if pre is not None:
            Fn.clip_grad_norm_flat(flat, clip_value, pre_scale=pre, want_norm=False)   # :113
        else:
            Fn.clip_grad_norm_(params, clip_value, want_norm=False)                    # :113
    return loss


def forward_step_device(model, clean_images, noisy_images, distribution_choice='uniform', t=None, need_loss=True):
    """A train step whose gradient the reference throws away (diffusion_RDUnet.py:78:
    the next step's zero_grad): the same timestep draw (so the RNG streams stay the
    reference's) and, when the loss is logged, the same forward + loss without
    saved activations; no backward, no clip, no gradient all-reduce."""
    if not need_loss:
        if t is None:
            _draw_t(clean_images.size(0), model.timesteps, distribution_choice, clean_images.device)
        return None
    model.train()
    with torch.no_grad():
        return _forward_loss(model, clean_images, noisy_images, distribution_choice, t)


def train_step_checkpointed(model, clean_images, noisy_images, optimizer, accumulation_steps,
                            distribution_choice='uniform', clip_value=0.1, *, t=None):
    """diffusion_RDUnet.py:76-115 (returns ``loss.item()`` like the reference).
    ``main_diffusion_RDUnet.py``'s variant has no ``distribution_choice``; passing
    the clip value positionally there works the same (a float is taken as the
    clip value)."""
    if isinstance(distribution_choice, (int, float)) and not isinstance(distribution_choice, bool):
        clip_value, distribution_choice = float(distribution_choice), 'uniform'
    loss = train_step_device(model, clean_images, noisy_images, optimizer, distribution_choice, clip_value, t=t)
    return loss.item()


def train_model_checkpointed(model, train_loader, val_loader, optimizer, scheduler, writer, output_dir,
                             distribution_choice='uniform', num_epochs=10, start_epoch=0, accumulation_steps=4,
                             clip_value=1.0, log_every=1, accumulation='reference'):
    """diffusion_RDUnet.py:117-178: epochs of train steps with the reference's
    every-``accumulation_steps`` optimizer step, one-batch improved_sampling
    validation, scheduler step and a checkpoint dict per epoch.  ``log_every``
    > 1 rate-limits the per-batch ``loss.item()`` host sync; ``accumulation``
    selects the reference's update rule or the fixed one (see run_epochs)."""
    run_epochs(model, train_loader, val_loader, optimizer, scheduler, writer, output_dir, distribution_choice,
               num_epochs, start_epoch, accumulation_steps, clip_value, log_every,
               sample=lambda m, x: m.improved_sampling(x), accumulation=accumulation)


ACCUMULATION_MODES = ("reference", "fixed")


def run_epochs(model, train_loader, val_loader, optimizer, scheduler, writer, output_dir, distribution_choice,
               num_epochs, start_epoch, accumulation_steps, clip_value, log_every, sample, accumulation='reference',
               skip_discarded=True):
    """The epoch loop shared by the three reference trainers (diffusion_RDUnet.py:117-178,
    main_diffusion_RDUnet.py:275-336, diffusion_RDUnet_direct.py:266-327); they
    differ only in the validation sampler and the checkpoint directory.

    accumulation='reference' keeps the reference's update rule:
    train_step_checkpointed zeroes the gradients at its top (:78), so only the
    clipped gradient of every ``accumulation_steps``-th batch reaches
    ``optimizer.step()`` (:126-128).  The other batches' backward, clip and (DDP)
    all-reduce are skipped -- their gradient is discarded by the reference -- while
    their timestep draw and, when logged, their forward loss still run, so the
    parameters are the reference's bit for bit at a third of those batches' cost.
    accumulation='fixed' accumulates the gradients of ``accumulation_steps``
    batches and clips + steps once (the rule of UNet/RDUNet_model.py:201-215).
    ``skip_discarded=False`` runs the discarded backward passes anyway (the
    reference's literal work; tests compare the two bit for bit)."""
    if accumulation not in ACCUMULATION_MODES:
        raise ValueError(f"accumulation must be one of {ACCUMULATION_MODES}, got {accumulation!r}")
    dev = next(model.parameters()).device
    for epoch in range(start_epoch, num_epochs):
        model.train()
        optimizer.zero_grad()
        n_batches = len(train_loader) if hasattr(train_loader, "__len__") else 0
        for batch_idx, (noisy_images, clean_images) in enumerate(train_loader):
            noisy_images, clean_images = noisy_images.to(dev), clean_images.to(dev)
            step_now = (batch_idx + 1) % accumulation_steps == 0
            log_now = batch_idx % log_every == 0
            if accumulation == 'fixed':
                loss_t = train_step_device(model, clean_images, noisy_images, optimizer, distribution_choice,
                                           clip_value, zero_grad=False, clip=False)
                if step_now:
                    Fn.clip_grad_norm_(model.parameters(), clip_value)
            elif step_now or not skip_discarded:
                loss_t = train_step_device(model, clean_images, noisy_images, optimizer, distribution_choice,
                                           clip_value)
            else:
                loss_t = forward_step_device(model, clean_images, noisy_images, distribution_choice,
                                             need_loss=log_now)
            if step_now:
                optimizer.step()
                optimizer.zero_grad()
            if log_now:
                loss = loss_t.item()
                print(f"Epoch [{epoch + 1}/{num_epochs}], Batch [{batch_idx + 1}/{n_batches}], Loss: {loss:.4f}")
                if writer is not None:
                    writer.add_scalar('Loss/train', loss, epoch * n_batches + batch_idx)
        model.eval()
        validation_loss = float("nan")
        if val_loader is not None:
            with torch.no_grad():
                val_noisy_images, val_clean_images = next(iter(val_loader))
                val_noisy_images, val_clean_images = val_noisy_images.to(dev), val_clean_images.to(dev)
                denoised_images = sample(model, val_noisy_images)
                validation_loss = combined_loss(denoised_images, val_clean_images).item()
        print(f"Epoch [{epoch + 1}/{num_epochs}], Validation Loss: {validation_loss:.4f}")
        if writer is not None:
            writer.add_scalar('Loss/validation', validation_loss, epoch + 1)
            if hasattr(writer, "flush"):
                writer.flush()
        if scheduler is not None:
            scheduler.step()
        checkpoint_path = os.path.join(output_dir, f"diffusion_RDUNet_model_checkpointed_epoch_{epoch + 1}.pth")
        os.makedirs(os.path.dirname(checkpoint_path) or ".", exist_ok=True)
        torch.save({
            'epoch': epoch + 1,
            'model_state_dict': model.state_dict(),
            'optimizer_state_dict': optimizer.state_dict(),
            'scheduler_state_dict': scheduler.state_dict() if scheduler is not None else None,
        }, checkpoint_path)
        print(f"Model checkpoint saved at {checkpoint_path}")


def load_checkpoint(model, optimizer, scheduler, checkpoint_path):
    """diffusion_RDUnet.py:180-193 (weights-only safe load)."""
    if (checkpoint_path is not None) and os.path.isfile(checkpoint_path):
        print(f"Loading checkpoint '{checkpoint_path}'")
        dev = next(model.parameters()).device
        checkpoint = torch.load(checkpoint_path, map_location=dev, weights_only=True)
        model.load_state_dict(checkpoint['model_state_dict'])
        optimizer.load_state_dict(checkpoint['optimizer_state_dict'])
        if scheduler is not None and checkpoint.get('scheduler_state_dict') is not None:
            scheduler.load_state_dict(checkpoint['scheduler_state_dict'])
        start_epoch = checkpoint['epoch']
        print(f"Loaded checkpoint '{checkpoint_path}' (epoch {start_epoch})")
        return start_epoch
    print(f"No checkpoint found at '{checkpoint_path}'")
    return 0


def load_data(args):
    """diffusion_RDUnet.py:222-228 dispatch on ``args.dataset_choice``."""
    from .data_loader import load_data as load_div2k_data, load_sidd_data
    if args.dataset_choice == 'DIV2K':
        return load_div2k_data('dataset/DIV2K_train_HR.nosync', batch_size=args.batch_size, augment=args.augment,
                               dataset_percentage=args.dataset_percentage, validation_split=args.validation_split,
                               use_rgb=True, num_workers=args.num_workers)
    return load_sidd_data('dataset/SIDD_dataset.nosync/SIDD_Medium_Srgb', batch_size=args.batch_size,
                          augment=args.augment, dataset_percentage=args.dataset_percentage,
                          validation_split=args.validation_split, use_rgb=True, num_workers=args.num_workers)


def make_optimizer(args, params):
    """diffusion_RDUnet.py:264-276 choices."""
    if args.optimizer_choice == 'adam':
        optimizer = optim.Adam(params, lr=args.lr, betas=(0.9, 0.999))
        scheduler = CosineAnnealingLR(optimizer, T_max=10)
    elif args.optimizer_choice == 'adamw':
        optimizer = optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay)
        scheduler = optim.lr_scheduler.StepLR(optimizer, step_size=3, gamma=0.5)
    else:
        optimizer = optim.Adadelta(params, lr=args.lr)
        scheduler = optim.lr_scheduler.StepLR(optimizer, step_size=3, gamma=0.5)
    return optimizer, scheduler


def train(args, train_loader=None, val_loader=None):
    """diffusion_RDUnet.py:230-288 (TensorBoard if importable)."""
    try:
        from torch.utils.tensorboard import SummaryWriter
        writer = SummaryWriter(log_dir=os.path.join("runs", "diffusion_checkpointed", os.path.basename(args.output_dir)))
    except Exception:  # tensorboard is optional
        writer = None
    if train_loader is None or val_loader is None:
        train_loader, val_loader = load_data(args)
    unet = RDUNet_T(base_filters=args.base_filters).to(device)
    unet.set_compute_dtype(getattr(args, "dtype", "fp32"))
    model = DiffusionModel(unet, timesteps=args.timesteps).to(device)
    unet.apply(init_weights())
    optimizer, scheduler = make_optimizer(args, model.parameters())
    start_epoch = load_checkpoint(model, optimizer, scheduler, args.checkpoint_path)
    train_model_checkpointed(model, train_loader, val_loader, optimizer, scheduler, writer, args.output_dir,
                             args.distribution_choice, num_epochs=args.num_epochs, start_epoch=start_epoch,
                             accumulation=getattr(args, "accumulation", "reference"))
    final_model_path = os.path.join(args.output_dir, "diffusion_RDUNet_model_checkpointed_final.pth")
    torch.save(model.state_dict(), final_model_path)
    print(f"Final model saved at {final_model_path}")
    if writer is not None:
        writer.close()


def build_parser():
    """diffusion_RDUnet.py:293-309, plus --dtype."""
    parser = argparse.ArgumentParser(description="Train a diffusion model with optional optimizer and scheduler choice.")
    parser.add_argument('--dataset_choice', type=str, default='SIDD', choices=['DIV2K', 'SIDD'])
    parser.add_argument('--checkpoint_path', type=str, default=None)
    parser.add_argument('--num_epochs', type=int, default=300)
    parser.add_argument('--batch_size', type=int, default=8)
    parser.add_argument('--num_workers', type=int, default=8)
    parser.add_argument('--validation_split', type=float, default=0.2)
    parser.add_argument('--augment', action='store_false')
    parser.add_argument('--dataset_percentage', type=float, default=0.1)
    parser.add_argument('--base_filters', type=int, default=32)
    parser.add_argument('--timesteps', type=int, default=20)
    parser.add_argument('--optimizer_choice', type=str, default='adamw', choices=['adam', 'adamw', 'adadelta'])
    parser.add_argument('--scheduler_choice', type=str, default='step', choices=['cosine', 'step'])
    parser.add_argument('--output_dir', type=str, default='checkpoints')
    parser.add_argument('--lr', type=float, default=1e-4)
    parser.add_argument('--weight_decay', type=float, default=1e-4)
    parser.add_argument('--distribution_choice', type=str, default='uniform', choices=['uniform', 'biased'])
    parser.add_argument('--dtype', type=str, default='fp32', choices=['fp32', 'bf16'])
    parser.add_argument('--accumulation', type=str, default='reference', choices=list(ACCUMULATION_MODES),
                        help="reference: only every 4th batch's gradient is applied (the reference's rule, "
                             "without the discarded backward passes); fixed: accumulate 4 batches")
    return parser


if __name__ == "__main__":
    train(build_parser().parse_args())
    sys.exit(0)
