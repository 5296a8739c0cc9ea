"""Generate the golden vectors in ``tests/golden/`` by importing the REFERENCE.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/make_golden.py``.

The reference modules are imported read-only from ``/root/reference`` with
``sys.dont_write_bytecode = True``; modules it imports that are absent from
this image (tensorboard, torchvision, pytorch_msssim, the dataset loaders)
are replaced by inert ``sys.modules`` stubs.  ``pytorch_msssim.ssim`` is
stubbed to 0: it enters ``combined_loss`` with weight 0
(``diffusion_denoising/diffusion_RDUnet.py:60-65``), so loss and gradients
are unaffected for finite values.

Parameters come from the portable hash generator (``oracle/weights.py``) and
are loaded into the reference modules with ``load_state_dict``; inputs come
from the same generator.  Only inputs, ``t`` draws and outputs are written —
no reference source travels.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle.weights import make_params, hash_images, hash_gauss_images  # noqa: E402


def _install_stubs():
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # inert
        def __init__(self, *a, **k): pass
        def add_scalar(self, *a, **k): pass
        def add_image(self, *a, **k): pass
        def flush(self): pass
        def close(self): pass

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    tv = types.ModuleType("torchvision")
    tvu = types.ModuleType("torchvision.utils")
    tvu.make_grid = lambda x, **k: x
    tvt = types.ModuleType("torchvision.transforms")
    tv.utils, tv.transforms = tvu, tvt
    sys.modules.update({"torchvision": tv, "torchvision.utils": tvu, "torchvision.transforms": tvt})
    ms = types.ModuleType("pytorch_msssim")
    ms.ssim = lambda x, y, **k: torch.zeros((), dtype=x.dtype)
    sys.modules["pytorch_msssim"] = ms
    for name in ("dataset_creation", "dataset_creation.data_loader", "dataset_creation.SIDD_dataset"):
        m = types.ModuleType(name)
        m.load_data = lambda *a, **k: (None, None)
        sys.modules[name] = m


def _load(modname, path):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def _params_for(model, seed, prefix=""):
    shapes = {k[len(prefix):]: tuple(v.shape) for k, v in model.state_dict().items() if k.startswith(prefix)}
    p = make_params(shapes, seed)
    return {prefix + k: torch.from_numpy(v) for k, v in p.items()}


def _sample_idx(name, n, k=64):
    from oracle.weights import hash_uniform
    if n <= 4096:
        return np.arange(n)
    return np.unique((hash_uniform(7, name, k, 0, n).astype(np.int64)) % n)


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    unet_mod = _load("diffusion_denoising.Unet.Unet_model", os.path.join(REF, "diffusion_denoising/Unet/Unet_model.py"))
    diff_mod = _load("ref_diffusion_RDUnet", os.path.join(REF, "diffusion_denoising/diffusion_RDUnet.py"))
    direct_mod = _load("ref_diffusion_RDUnet_direct", os.path.join(REF, "diffusion_denoising/diffusion_RDUnet_direct.py"))
    RDUNet_T = unet_mod.RDUNet_T
    out = {}

    # (0) initial weights: torch.manual_seed(0); RDUNet_T(16) (reference RNG stream)
    torch.manual_seed(0)
    m0 = RDUNet_T(base_filters=16)
    out["init16_sums"] = np.array([v.double().sum().item() for v in m0.state_dict().values()])

    # (1) RDUNet_T(F0=16) forward, 1x3x64x64, scalar t=0.35 (sampling form [1,1,1,1])
    torch.manual_seed(0)
    m = RDUNet_T(base_filters=16).eval()
    m.load_state_dict(_params_for(m, seed=11))
    x = torch.from_numpy(hash_gauss_images(1, "fwd16.x", (1, 3, 64, 64)))
    t = torch.full((1, 1, 1, 1), 0.35)
    with torch.no_grad():
        y = m(x, t)
    out.update({"fwd16_x": x.numpy(), "fwd16_t": t.numpy(), "fwd16_y": y.numpy(), "fwd16_seed": np.array(11)})

    # (2) RDUNet_T(F0=32) forward, B=2, 32x32, per-sample t map [2,1,32,32] (training form)
    torch.manual_seed(0)
    m32 = RDUNet_T(base_filters=32).eval()
    m32.load_state_dict(_params_for(m32, seed=12))
    x = torch.from_numpy(hash_images(2, "fwd32.x", (2, 3, 32, 32)))
    t = torch.tensor([0.25, 0.9]).view(2, 1, 1, 1).expand(2, 1, 32, 32)
    with torch.no_grad():
        y = m32(x, t)
    out.update({"fwd32_x": x.numpy(), "fwd32_t": t.contiguous().numpy(), "fwd32_y": y.numpy(), "fwd32_seed": np.array(12)})

    # (3) train_step_checkpointed (reference), RDUNet_T(16), B=2, 32x32, uniform t, clip 1.0
    torch.manual_seed(0)
    unet = RDUNet_T(base_filters=16)
    model = diff_mod.DiffusionModel(unet, timesteps=20)
    model.load_state_dict(_params_for(model, seed=13, prefix="unet."))
    clean = torch.from_numpy(hash_images(3, "ts.clean", (2, 3, 32, 32)))
    noisy = clean + (25.0 / 255.0 * 2.0) * torch.from_numpy(hash_gauss_images(3, "ts.noise", (2, 3, 32, 32)))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    torch.manual_seed(123)
    t_draw = torch.randint(0, 21, (2,))
    torch.manual_seed(123)
    loss = diff_mod.train_step_checkpointed(model, clean, noisy, opt, 4, "uniform", clip_value=1.0)
    names = [k for k, _ in model.named_parameters()]
    gnorm = np.array([model.get_parameter(n).grad.norm().item() for n in names], dtype=np.float64)
    out.update({"ts_clean": clean.numpy(), "ts_noisy": noisy.numpy(), "ts_t": t_draw.numpy(),
                "ts_loss": np.array(loss, dtype=np.float64), "ts_seed": np.array(13),
                "ts_names": np.array(names), "ts_gnorm": gnorm})
    for n in names:
        g = model.get_parameter(n).grad.detach().reshape(-1).numpy()
        idx = _sample_idx(n, g.size)
        out[f"ts_gidx::{n}"] = idx
        out[f"ts_gval::{n}"] = g[idx]
    opt.step()  # one AdamW step on the clipped gradients (diffusion_RDUnet.py:126-128 order)
    for n in names:
        d = (model.get_parameter(n).detach() - before[n]).reshape(-1).numpy()
        idx = out[f"ts_gidx::{n}"]
        out[f"ts_dval::{n}"] = d[idx]

    # (4) improved_sampling T=4 and (5) direct_sampling, RDUNet_T(16), 1x3x32x32
    torch.manual_seed(0)
    unet = RDUNet_T(base_filters=16).eval()
    dm = diff_mod.DiffusionModel(unet, timesteps=4)
    dm.load_state_dict(_params_for(dm, seed=14, prefix="unet."))
    noisy = torch.from_numpy(hash_images(4, "samp.noisy", (1, 3, 32, 32)))
    with torch.no_grad():
        ys = dm.improved_sampling(noisy)
        dd = direct_mod.DiffusionModel(dm.unet, timesteps=4)
        yd = dd.direct_sampling(noisy)
    out.update({"samp_noisy": noisy.numpy(), "samp_improved": ys.numpy(), "samp_direct": yd.numpy(),
                "samp_seed": np.array(14), "samp_T": np.array(4)})

    # (6) plain RDUNet(F0=64) forward on one 1x3x64x64 Gaussian-noise tensor (config 1)
    rd_mod = _load("ref_RDUNet_model", os.path.join(REF, "UNet/RDUNet_model.py"))
    torch.manual_seed(0)
    rd = rd_mod.RDUNet(channels=3, base_filters=64).eval()
    rd.load_state_dict(_params_for(rd, seed=15))
    x = torch.from_numpy(hash_gauss_images(5, "plain.x", (1, 3, 64, 64)))
    with torch.no_grad():
        y = rd(x)
    out.update({"plain64_x": x.numpy(), "plain64_y": y.numpy(), "plain64_seed": np.array(15)})

    path = os.path.join(HERE, "golden_rdunet.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes;", len(out), "arrays")


if __name__ == "__main__":
    main()
