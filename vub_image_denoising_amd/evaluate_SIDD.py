"""SIDD validation-block evaluation (evaluate_SIDD/evaluate_SIDD.py) on the GPU.

Same entry points as the reference: ``SIDDMatDataset(noisy_mat_file,
gt_mat_file)`` (:18-40) and ``evaluate_model(model, dataloader, device)`` (:42-78)
returning ``(avg_psnr, avg_ssim, avg_inference_time_ms, sample_images)``; plus
``denormalize`` (:80-82) and ``main()`` (:102-148, minus the plot window).

What changes underneath: the reference moves every denoised block to the host
and scores it with scikit-image (:59-64).  Here the blocks stay in HBM and a whole
batch is scored by ``rdn_image_metrics`` (metrics.py / csrc/metrics.hip, the same
skimage 0.22 definitions, data_range=2, channel_axis=-1); only the per-block
float64 scores and the few sample images come back.  ``.mat`` files are read with
``scipy.io.loadmat`` (plain arrays, nothing executed).  torchvision is not needed:
``ToTensor`` + ``Normalize(0.5, 0.5)`` is ``uint8 / 255 * 2 - 1`` in fp32.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, Subset

from .metrics import image_metrics


def _to_tensor_normalized(block: np.ndarray) -> torch.Tensor:
    """transforms.ToTensor() + Normalize(mean=[0.5], std=[0.5]) of an HWC uint8 block."""
    t = torch.from_numpy(np.ascontiguousarray(block)).permute(2, 0, 1).float().div_(255.0)
    return t.sub_(0.5).div_(0.5)


class SIDDMatDataset(Dataset):
    """evaluate_SIDD.py:18-40: the SIDD sRGB validation blocks
    (``ValidationNoisyBlocksSrgb`` / ``ValidationGtBlocksSrgb``, [images, blocks,
    256, 256, 3] uint8); item = (noisy, gt) CHW fp32 in [-1, 1]."""

    def __init__(self, noisy_mat_file, gt_mat_file, noisy_key="ValidationNoisyBlocksSrgb",
                 gt_key="ValidationGtBlocksSrgb"):
        import scipy.io
        self.noisy_data = scipy.io.loadmat(noisy_mat_file)[noisy_key]
        self.gt_data = scipy.io.loadmat(gt_mat_file)[gt_key]
        if self.noisy_data.shape != self.gt_data.shape:
            raise ValueError(f"noisy {self.noisy_data.shape} and gt {self.gt_data.shape} blocks differ")

    def __len__(self):
        return self.noisy_data.shape[0] * self.noisy_data.shape[1]

    def __getitem__(self, idx):
        img_idx = idx // self.noisy_data.shape[1]
        patch_idx = idx % self.noisy_data.shape[1]
        return (_to_tensor_normalized(self.noisy_data[img_idx, patch_idx]),
                _to_tensor_normalized(self.gt_data[img_idx, patch_idx]))


def evaluate_model(model, dataloader, device, sampler=None):
    """evaluate_SIDD.py:42-78.  Per block: ``improved_sampling`` (timed like the
    reference, wall clock around the call; here with a device sync so the time is
    the GPU's), PSNR and SSIM on the GPU; averages over blocks.  ``sampler``
    overrides ``model.improved_sampling`` (e.g. a captured SamplerGraph)."""
    psnr_values, ssim_values, inference_times, sample_images = [], [], [], []
    run = sampler if sampler is not None else model.improved_sampling
    model.eval()
    block = 0
    with torch.no_grad():
        for noisy, gt in dataloader:
            noisy = noisy.to(device, non_blocking=True)
            gt = gt.to(device, non_blocking=True)
            torch.cuda.synchronize(device)
            start = time.time()
            denoised = run(noisy)
            torch.cuda.synchronize(device)
            per_block_ms = (time.time() - start) * 1000 / noisy.size(0)
            psnr, ssim = image_metrics(gt, denoised, data_range=2.0)
            psnr_values.extend(psnr.tolist())
            ssim_values.extend(ssim.tolist())
            inference_times.extend([per_block_ms] * noisy.size(0))
            for k in range(noisy.size(0)):   # blocks 11..14, HWC numpy (reference :67-68)
                if 10 < block + k < 15:
                    sample_images.append(tuple(t[k].permute(1, 2, 0).cpu().numpy() for t in (noisy, gt, denoised)))
            block += noisy.size(0)
    return float(np.mean(psnr_values)), float(np.mean(ssim_values)), float(np.mean(inference_times)), sample_images


def denormalize(img):
    img = (img + 1) / 2
    return np.clip(img, 0, 1)


def main(noisy_mat_file="evaluate_SIDD/ValidationNoisyBlocksSrgb.mat",
         gt_mat_file="evaluate_SIDD/ValidationGtBlocksSrgb.mat",
         checkpoint_path="checkpoints/diffusion_RDUNet_model_checkpointed_epoch_40.pth",
         evaluation_percentage=0.1, batch_size=1, base_filters=32, timesteps=20, out_csv="benchmark_results.csv"):
    """evaluate_SIDD.py:102-148 (the checkpoint is read with weights_only=True)."""
    from .diffusion_RDUnet import DiffusionModel
    from .Unet_model import RDUNet_T
    dataset = SIDDMatDataset(noisy_mat_file, gt_mat_file)
    indices = np.random.choice(len(dataset), int(len(dataset) * evaluation_percentage), replace=False)
    dataloader = DataLoader(Subset(dataset, indices), batch_size=batch_size, shuffle=False, num_workers=4)
    device = torch.device("cuda")
    model = DiffusionModel(RDUNet_T(base_filters=base_filters), timesteps=timesteps).to(device)
    if not os.path.exists(checkpoint_path):   # the reference's torch.load raises too
        raise FileNotFoundError(f"checkpoint not found: {checkpoint_path}")
    ckpt = torch.load(checkpoint_path, map_location=device, weights_only=True)
    model.load_state_dict(ckpt["model_state_dict"])
    avg_psnr, avg_ssim, avg_time, samples = evaluate_model(model, dataloader, device)
    print(f"Average PSNR: {avg_psnr:.2f}")
    print(f"Average SSIM: {avg_ssim:.4f}")
    print(f"Average Inference Time: {avg_time:.2f} ms")
    import pandas as pd
    pd.DataFrame({"Method": ["YourModel"], "MACs (G)": ["Your MACs"], "Inference Time (ms)": [avg_time],
                  "PSNR": [avg_psnr], "SSIM": [avg_ssim]}).to_csv(out_csv, index=False)
    return avg_psnr, avg_ssim, avg_time, samples


if __name__ == "__main__":
    main()
