"""Host-side cost of the bench train step: time to ISSUE K steps (no sync) vs
the GPU time of the same K steps, plus a cProfile of the issuing thread.
If issue time ~ GPU time, the step is host-bound."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vub_image_denoising_amd as vm  # noqa: E402
from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device  # noqa: E402
from vub_image_denoising_amd.optim import FusedAdamW  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
unet = vm.RDUNet_T(base_filters=32).to(dev).set_compute_dtype("bf16")
model = DiffusionModel(unet, timesteps=20)
clean = torch.rand(16, 3, 256, 256, device=dev) * 2 - 1
noisy = clean + 0.2 * torch.randn_like(clean)


class NoOpt:
    def zero_grad(self, set_to_none=True):
        for p in model.parameters():
            p.grad = None


train_step_device(model, clean, noisy, NoOpt(), "uniform", 1.0)
opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)


def step():
    train_step_device(model, clean, noisy, opt, "uniform", 1.0)
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
K = 20
t0 = time.perf_counter()
for _ in range(K):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"issue {1e3 * (t1 - t0) / K:.3f} ms/step, total {1e3 * (t2 - t0) / K:.3f} ms/step", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
