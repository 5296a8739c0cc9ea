"""hipGraph capture of one whole train step: the t draw, the interpolation, the
fused RDUNet_T forward, the Charbonnier loss, the backward, clip_grad_norm_ and
the fused Adam(W) update (diffusion_RDUnet.py:76-115 + ``optimizer.step()``),
replayed with ONE host launch per step instead of ~700 kernel launches issued
from Python.

What makes the step capturable:

* every buffer the step touches exists before capture (engine activations and
  launch descriptors, the flat gradient buffer, clip and Adam workspaces):
  warm-up steps build them, then their effect on the weights, the Adam moments,
  the step count and the RNG is rolled back, so the first replay IS the model's
  next step;
* the Adam step count lives in device memory (FusedAdam.use_device_step), so
  bias corrections advance on every replay;
* ``torch.randint`` t draws use torch's graph-safe Philox generator (every
  replay advances its offset exactly as an eager step does); the 'biased'
  distribution draws on the CPU in the reference (:71-73), so its t are drawn
  on the host per call and copied into the graph's t input;
* values baked into the graph — lr, betas, eps, weight decay, clip value,
  compute dtype — are compared on every call; a change (an LR scheduler step)
  re-captures.

The graph owns the parameters' ``.grad`` (views of the flat gradient buffer its
backward writes); an eager step in between is allowed and does not disturb it.
"""
from __future__ import annotations

import os

import torch

from .diffusion_RDUnet import sample_biased, train_step_device
from .engine import find_flat
from .optim import FusedAdam


class GraphCaptureUnsafe(RuntimeError):
    """Capturing the data-parallel step is not safe on this torch build."""


def _drain_collectives(fp) -> None:
    """Before a capture: wait until ProcessGroupNCCL's watchdog has retired every
    eager collective (the warm-up steps' all-reduces).  Its loop queries each
    pending work's end event, recorded on the group's RCCL stream; once that stream
    is pulled into the capture, HIP refuses the query (hipErrorCapturedEvent) and the
    watchdog aborts the process -- seen in the world-1 graph test on MI355X, round 4,
    whenever the capture began before the watchdog's next sweep."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    sync = getattr(fp, "grad_sync", None) if fp is not None else None
    groups = [dist.group.WORLD] + ([sync.group] if sync is not None and sync.group is not None else [])
    for pg in groups:
        try:
            if dist.get_backend(pg) != "nccl":
                continue
        except (RuntimeError, ValueError):
            continue
        if os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE") != "0":
            # with the event cache on, an eager collective's cached event can be re-recorded
            # inside the capture and the watchdog's query of it aborts the process (ddp.capture_safe_env)
            raise GraphCaptureUnsafe("capturing an RCCL train step needs TORCH_NCCL_CUDA_EVENT_CACHE=0 set before "
                                     "init_process_group (call ddp.capture_safe_env() first)")
        wait = getattr(pg, "_wait_for_pending_works", None)
        if wait is None:   # (a private ProcessGroupNCCL method; a build without it cannot capture safely)
            raise GraphCaptureUnsafe(
                "torch.distributed's NCCL process group has no _wait_for_pending_works(): the watchdog may query "
                "a captured event and abort the process, so the RCCL train step is not captured (run eagerly)")
        wait()


def _node_count(g):
    """Kernel/memset/copy nodes of a captured graph (None if not exposed)."""
    try:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        raw = g.raw_cuda_graph()
        n = ctypes.c_size_t(0)
        if hip.hipGraphGetNodes(ctypes.c_void_p(raw), None, ctypes.byref(n)) != 0:
            return None
        return n.value
    except Exception:
        return None


class TrainStepGraph:
    def __init__(self, model, optimizer, shape, distribution_choice='uniform', clip_value=1.0, t_input=False,
                 warmup=2):
        if not isinstance(optimizer, FusedAdam):
            raise TypeError("TrainStepGraph needs the fused optimizer (optim.FusedAdam / FusedAdamW)")
        self.model, self.opt = model, optimizer
        self.dist, self.clip = distribution_choice, clip_value
        dev = next(model.parameters()).device
        self.dev = dev
        self.clean = torch.zeros(shape, dtype=torch.float32, device=dev)
        self.noisy = torch.zeros(shape, dtype=torch.float32, device=dev)
        self.host_t = distribution_choice == 'biased'
        self.t = torch.zeros(shape[0], dtype=torch.float32, device=dev) if (t_input or self.host_t) else None
        self.graph = None
        self._build(warmup)

    # ------------------------------------------------------------------
    def _hyper(self):
        """Everything baked into the captured graph: hyperparameters, the compute
        dtype, and the addresses of the buffers the optimizer updates (a rebound
        optimizer or a re-flattened model re-captures instead of replaying onto
        freed memory)."""
        g = self.opt.param_groups[0]
        o = self.opt
        ptrs = tuple(0 if b is None else b.data_ptr()
                     for b in (getattr(o, "_m", None), getattr(o, "_v", None), o._step_dev,
                               None if o._fp is None else o._fp.flat))
        return (float(g["lr"]), tuple(g["betas"]), float(g["eps"]), float(g["weight_decay"]), float(self.clip),
                float(self.opt.grad_scale), self.model.unet.compute_dtype, ptrs)

    def _body(self):
        loss = train_step_device(self.model, self.clean, self.noisy, self.opt, self.dist, self.clip, t=self.t)
        self.opt.step()
        return loss

    def _build(self, warmup):
        rng = torch.cuda.get_rng_state(self.dev)
        params = list(self.model.parameters())
        side = torch.cuda.Stream(device=self.dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            if find_flat(params) is None or self.opt._fp is None:
                # gradients as flat views, so the optimizer can bind (no update yet)
                train_step_device(self.model, self.clean, self.noisy, self.opt, self.dist, self.clip, t=self.t)
            self.opt.use_device_step()
            fp, opt = self.opt._fp, self.opt
            snap = (fp.flat.clone(), opt._m.clone(), opt._v.clone(), opt._step)
            for _ in range(max(1, warmup)):
                self._body()
            fp.flat.copy_(snap[0])
            opt._m.copy_(snap[1])
            opt._v.copy_(snap[2])
            opt._step = snap[3]
            opt._steps.fill_(opt._step)
            opt._step_dev.fill_(opt._step)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize(self.dev)
        _drain_collectives(fp)
        fp.generation += 1
        for wp in self.model.unet._rdn_packs.values():
            wp.key = None          # the weight repack is the graph's first launch
        self.graph = None
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g):
            self.loss = self._body().detach()
        self.graph_nodes = _node_count(g)
        g.instantiate()
        self.graph = g
        self._captured = self._hyper()
        # capture ran nothing: undo its host-side effects (step count, pack keys)
        opt._step = snap[3]
        opt._steps.fill_(opt._step)
        fp.generation += 1
        torch.cuda.set_rng_state(rng, self.dev)

    # ------------------------------------------------------------------
    def __call__(self, clean_images, noisy_images, t=None):
        """One train step on this batch; returns the loss (a device tensor, valid
        until the next call)."""
        if self._hyper() != self._captured:
            self._build(1)
        self.clean.copy_(clean_images)
        self.noisy.copy_(noisy_images)
        if self.t is not None:
            if t is None:
                if not self.host_t:
                    raise ValueError("this graph was built with t_input=True: pass t")
                t = sample_biased(self.clean.size(0), self.model.timesteps)
            self.t.copy_(t)
        elif t is not None:
            raise ValueError("this graph draws t itself (build it with t_input=True to pass t)")
        self.graph.replay()
        self.opt._replayed()
        return self.loss


class TrainStepGraphs:
    """One captured train step per input shape (config 5's mixed 128/256 patch
    stream, synth.MixedPatchLoader): a batch of a new shape captures its own
    TrainStepGraph (its own engine, activations and graph); the graphs share the
    model's flat parameters, gradient buffer and the optimizer's state (Adam moments
    and the device step counter), and replays run one after another on the stream,
    so the alternation is the same sequence of steps as eager training."""

    def __init__(self, model, optimizer, distribution_choice='uniform', clip_value=1.0, t_input=False, warmup=2):
        self.model, self.opt = model, optimizer
        self.kw = dict(distribution_choice=distribution_choice, clip_value=clip_value, t_input=t_input,
                       warmup=warmup)
        self.graphs = {}
        self.captures = 0

    def __call__(self, clean_images, noisy_images, t=None):
        shape = tuple(clean_images.shape)
        g = self.graphs.get(shape)
        if g is None:
            g = self.graphs[shape] = TrainStepGraph(self.model, self.opt, shape, **self.kw)
            self.captures += 1
        return g(clean_images, noisy_images, t)
