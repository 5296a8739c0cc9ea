"""vub_image_denoising_amd — MI355X (gfx950) native implementation of the
diffusion-RDUNet denoising hot path of pierregab/VUB_Image_denoising.

Drop-in modules (same names/signatures as the reference):
  Unet_model        RDUNet_T, InputBlock, OutputBlock, DenoisingBlock,
                    DownsampleBlock, UpsampleBlock, init_weights
  RDUNet_model      RDUNet
  diffusion_RDUnet  DiffusionModel, charbonnier_loss, combined_loss,
                    train_step_checkpointed, train_model_checkpointed, ...
  data_loader       load_data (DIV2K-style folder loader, synthetic loader)
Compute runs in librdunet_hip.so (hand-written HIP kernels, C ABI in
include/rdunet_hip.h); see DESIGN.md.
"""
from .Unet_model import (DenoisingBlock, DownsampleBlock, InputBlock, OutputBlock, RDUNet_T,  # noqa: F401
                         UpsampleBlock, init_weights)
from .RDUNet_model import RDUNet  # noqa: F401
from .diffusion_RDUnet import (DiffusionModel, charbonnier_loss, combined_loss, denormalize,  # noqa: F401
                               sample_biased, train_step_checkpointed, train_model_checkpointed, load_checkpoint)

__version__ = "0.1.0"
