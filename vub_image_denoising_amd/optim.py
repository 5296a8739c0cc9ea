"""Fused Adam / AdamW over the flat parameter buffer: one ``rdn_adam_step``
launch per step instead of torch's per-tensor (foreach) kernels.

Same update as ``torch.optim.Adam`` / ``AdamW`` (the optimizers of
diffusion_RDUnet.py:264-268 and main_diffusion_RDUnet.py:230), same
``param_groups`` (so LR schedulers work) and a ``state_dict`` in torch's
per-parameter format (``step``, ``exp_avg``, ``exp_avg_sq``), whose moment
tensors are views of the flat moment buffers.  ``load_state_dict`` restores the
moments and the step count into those buffers, so a resumed run continues
bit-identically (diffusion_RDUnet.py:180-193 resume path).
"""
from __future__ import annotations

import torch

from . import _hip as H
from .engine import find_flat


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False,
                 grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam works on one parameter group (the fused network's flat buffer)")
        self.decoupled = decoupled
        self.grad_scale = grad_scale
        self._fp = None
        self._step = 0
        self._step_dev = None   # device step counter (use_device_step)

    def _bind(self):
        params = self.param_groups[0]["params"]
        fp = find_flat(params)
        if fp is None:
            raise RuntimeError("FusedAdam needs the parameters of one GPU RDUNet (run a forward/backward first); "
                               "use torch.optim.Adam(W) otherwise")
        if self._fp is not fp:
            # moments already in self.state (a load_state_dict before the first step,
            # or a previous flat buffer) are carried over into the new flat buffers
            self._fp = fp
            self._m = torch.zeros_like(fp.flat)
            self._v = torch.zeros_like(fp.flat)
            self._steps = torch.zeros((), dtype=torch.float32)
            self._load_moments()
        return fp

    def _load_moments(self):
        """Copy the moments / step count held in ``self.state`` (torch's per-parameter
        format) INTO the existing flat buffers and device step counter, then make the
        state entries views of them again.  In place, so a TrainStepGraph captured
        over these buffers keeps replaying on the loaded state."""
        fp = self._fp
        old = {p: self.state[p] for p in fp.params if p in self.state}
        steps = set()
        self._m.zero_()
        self._v.zero_()
        for p, off in zip(fp.params, fp.offsets):
            n = p.numel()
            st = old.get(p)
            if st and "exp_avg" in st:
                self._m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self._v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise RuntimeError(f"FusedAdam: parameters were saved at different step counts {sorted(steps)}")
        self._step = steps.pop() if steps else 0
        self._steps.fill_(self._step)
        if self._step_dev is not None:
            if self._step_dev.device == fp.device:
                self._step_dev.fill_(self._step)
            else:
                self._step_dev = torch.full((), self._step, dtype=torch.int64, device=fp.device)
        self._views()

    def reset_state(self):
        """Forget the moments and the step count, in place (the flat moment buffers
        and device step counter keep their addresses, so a TrainStepGraph captured
        over them replays from a fresh optimizer: re-initialised training runs)."""
        self.state.clear()
        if self._fp is not None:
            self._load_moments()
        else:
            self._step = 0

    def use_device_step(self):
        """Keep the step count in device memory, incremented and read by the
        update kernels, so a hipGraph-captured step stays exact on every replay
        (train_graph.TrainStepGraph); the host count mirrors it."""
        fp = self._bind()
        if self._step_dev is None:
            self._step_dev = torch.full((), self._step, dtype=torch.int64, device=fp.device)
        return self

    def _replayed(self):
        """A captured step ran (host mirror of the device step count)."""
        self._step += 1
        self._steps.fill_(self._step)
        self._fp.generation += 1

    def _views(self):
        fp = self._fp
        for p, off in zip(fp.params, fp.offsets):
            n = p.numel()
            self.state[p] = {"step": self._steps, "exp_avg": self._m[off:off + n].view_as(p),
                             "exp_avg_sq": self._v[off:off + n].view_as(p)}

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        if self._fp is None:
            return                        # moments are taken over at the first bind
        fp = find_flat(self.param_groups[0]["params"])
        if fp is self._fp or fp is None:
            # same flat buffers (the usual resume): loaded into the existing moment
            # buffers and step counter, whose addresses a captured graph holds
            self._load_moments()
        else:
            self._fp = None
            self._bind()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        fp = self._bind()
        g = self.param_groups[0]
        self._step += 1
        self._steps.fill_(self._step)
        b1, b2 = g["betas"]
        lib, st = H.lib(), H.stream_ptr()
        sd = None
        if self._step_dev is not None:
            H.check(lib.rdn_counter_inc(self._step_dev.data_ptr(), st), "counter_inc")
            sd = self._step_dev.data_ptr()
        H.check(lib.rdn_adam_step(fp.flat.data_ptr(), fp.gflat.data_ptr(), self._m.data_ptr(), self._v.data_ptr(),
                                  fp.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                  float(g["weight_decay"]), 1 if self.decoupled else 0, self._step, sd,
                                  float(self.grad_scale), st), "adam_step")
        fp.generation += 1  # weights changed behind torch's version counters: repack
        return loss

    def zero_grad(self, set_to_none: bool = True):
        fp = find_flat(self.param_groups[0]["params"])
        if fp is not None and not set_to_none:
            fp.gflat.zero_()
            return
        super().zero_grad(set_to_none=set_to_none)


class FusedAdamW(FusedAdam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decoupled=True,
                         grad_scale=grad_scale)
