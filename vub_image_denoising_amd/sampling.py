"""Reverse-diffusion samplers on the GPU.

``improved_sampling`` restates ``DiffusionModel.improved_sampling``
(diffusion_denoising/diffusion_RDUnet.py:38-50): for t = T..1 two UNet calls on
the same x_t at t/T and (t-1)/T, then
``x_t = x_t - ((1-a)*f1 + a*y) + ((1-a')*f2 + a'*y)`` — one fused
``rdn_sampling_combine`` launch per step.  The t scalars live in a small device
table (no per-step host→device copies), so the whole loop is a fixed launch
sequence that ``SamplerGraph`` can capture into one hipGraph.
"""
from __future__ import annotations

import torch

from . import functional as Fn


_TABLES = {}


def _t_table(T, dev):
    # t/T rounded from double exactly as torch.tensor([t / T]) does (:43,:46);
    # cached so a graph capture never issues a host->device copy
    key = (T, str(dev))
    tab = _TABLES.get(key)
    if tab is None:
        tab = _TABLES[key] = torch.tensor([t / T for t in range(T + 1)], dtype=torch.float32, device=dev)
    return tab


def improved_sampling(model, noisy_image: torch.Tensor) -> torch.Tensor:
    T = model.timesteps
    y = noisy_image.contiguous().float()
    tt = _t_table(T, y.device)
    x_t = y.clone()
    for t in reversed(range(1, T + 1)):
        a, ap = t / T, (t - 1) / T
        f1 = model.unet(x_t, tt[t].view(1, 1, 1, 1))
        f2 = model.unet(x_t, tt[t - 1].view(1, 1, 1, 1))
        Fn.sampling_combine(x_t, f1, f2, y, a, ap)
    return x_t


class SamplerGraph:
    """hipGraph capture of the full improved_sampling (or direct_sampling) loop
    for a fixed input shape: one host launch per call after capture."""

    def __init__(self, model, shape, direct=False):
        self.model = model
        self.direct = direct
        dev = next(model.parameters()).device
        self.inp = torch.zeros(shape, dtype=torch.float32, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.no_grad(), torch.cuda.stream(s):
            for _ in range(2):  # warm up: engines, packs, workspaces allocated outside capture
                self._body()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = self._body()

    def _body(self):
        if self.direct:
            return self.model.unet(self.inp, _t_table(1, self.inp.device)[1].view(1, 1, 1, 1))
        return improved_sampling(self.model, self.inp)

    def __call__(self, noisy_image):
        self.inp.copy_(noisy_image)
        for packs in self.model.unet._rdn_packs.values():  # weights changed since capture -> repack first
            packs.refresh()
        self.graph.replay()
        return self.out
