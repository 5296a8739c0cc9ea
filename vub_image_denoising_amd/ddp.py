"""Data-parallel gradient synchronisation over RCCL (torch.distributed "nccl"
backend on ROCm), overlapped with the fused backward.

The reference has no distributed code; this is the new
capability of config 3.  Images are independent (no BatchNorm), so DP is exact:
the all-reduced mean gradient equals the single-process gradient of the
concatenated batch.

Design for MI355X (xGMI point-to-point mesh):

* a backward writes its gradients into ONE flat fp32 buffer
  (``engine.ParamSet.grad_buffer``; ``.grad`` become views of it), laid out in
  module registration order (input block first), which is the REVERSE of
  backward completion order; that buffer is what is all-reduced (the engine
  passes it to ``begin``), so with gradient accumulation only the new
  contribution goes over the links, as with torch DDP;
* it is cut into ~``bucket_mb`` buckets of contiguous parameter ranges; a bucket
  is launched (``all_reduce``, sum) on a side stream as soon as the engine's
  backward has finished the last layer whose gradients it holds, so RCCL rings
  run on the links while the remaining layers' dgrad/wgrad run on the compute
  stream;
* the 1/world average is one in-place scale after the last bucket (so
  clip_grad_norm_ sees the mean gradient, as torch DDP would) -- or, when the
  caller clips right after the backward (``defer_average``, set by
  train_step_device), it is folded into the clip's own scale pass
  (rdn_sqnorm_scaled): one pass over the 41.6 MB gradient instead of two.

No wrapper around the model: ``train_step_checkpointed`` calls
``model.unet(...)`` directly (diffusion_RDUnet.py:106), which would bypass a DDP
wrapper around DiffusionModel anyway.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def exposure_from_stamps(samples, ticks_per_ms):
    """Exposed all-reduce time (ms per step) from GradSync stamp triples (t_bwd,
    t_comm, t_after) read after each replay: (t_comm - t_bwd) less the launch gap of two
    back-to-back stamp kernels (t_after - t_comm), floored at 0 -- the time the
    compute stream waited for the last bucket's all-reduce after its own backward.
    Returns {per_step, mean, max, raw_mean} or None without samples."""
    if not samples or ticks_per_ms <= 0:
        return None
    raw = [(b - a) / ticks_per_ms for a, b, _ in samples]
    exp = [max(0.0, (b - a) - (c - b)) / ticks_per_ms for a, b, c in samples]
    return {"per_step": [round(x, 4) for x in exp], "mean": round(sum(exp) / len(exp), 4),
            "max": round(max(exp), 4), "raw_mean": round(sum(raw) / len(raw), 4)}


def capture_safe_env() -> None:
    """Environment for RCCL collectives inside a captured hipGraph; call before
    ``init_process_group``: no NCCL event cache (every work item owns its events, so
    no event of an eager collective is re-recorded inside a capture).  The capture
    itself first drains the watchdog's pending works (train_graph._drain_collectives)."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def plan_buckets(sizes, offsets, bucket_elems, tail_elems=0):
    """Group parameters (given in flat order) into contiguous buckets, filling
    from the END of the flat buffer (first gradients to complete).  Returns a
    list of (lo, hi, first_param_index) with flat ranges [lo, hi).

    ``tail_elems``: the bucket at the START of the buffer (input block and encoder
    level 0/1: the gradients that complete last) is its all-reduce that nothing
    overlaps; it is cut down to the parameters within the first ``tail_elems``
    elements, the rest of it becoming a bucket of its own that is launched as soon
    as the encoder's deeper levels are done (39.7 MB at base_filters 32, 25-MB buckets:
    21.3 + 18.4 MB -> 21.3 + 15.3 + 3.1 MB, the exposed tail 6x smaller)."""
    n = len(sizes)
    buckets = []
    hi_idx = n
    while hi_idx > 0:
        lo_idx = hi_idx - 1
        acc = sizes[lo_idx]
        while lo_idx > 0 and acc + sizes[lo_idx - 1] <= bucket_elems:
            lo_idx -= 1
            acc += sizes[lo_idx]
        lo = offsets[lo_idx]
        hi = offsets[hi_idx] if hi_idx < n else None
        buckets.append((lo, hi, lo_idx))
        hi_idx = lo_idx
    if tail_elems > 0 and buckets:
        lo, hi, first = buckets[-1]
        end = hi if hi is not None else (offsets[-1] + sizes[-1])
        if end - lo <= tail_elems:
            return buckets
        k = 0
        while k + 1 < n and offsets[k + 1] <= tail_elems and (hi is None or offsets[k + 1] < hi):
            k += 1
        if 0 < k and offsets[k] < end:
            buckets[-1] = (offsets[k], hi, k)
            buckets.append((0, offsets[k], 0))
    return buckets


class GradSync:
    """Bucketed, backward-overlapped gradient all-reduce for a FlatParams."""

    def __init__(self, fp, bucket_mb: float = 25.0, group=None, overlap: bool = True, tail_mb: float = 4.0):
        self.fp = fp
        self.group = group
        self.world = dist.get_world_size(group)
        sizes = [p.numel() for p in fp.params]
        offs = list(fp.offsets)
        raw = plan_buckets(sizes, offs, int(bucket_mb * 2 ** 20 / 4), int(tail_mb * 2 ** 20 / 4))
        self.buckets = []
        self.param_bucket = [0] * len(sizes)
        hi_idx = len(sizes)
        for b, (lo, hi, lo_idx) in enumerate(raw):
            self.buckets.append((lo, fp.numel if hi is None else hi))
            for i in range(lo_idx, hi_idx):
                self.param_bucket[i] = b
            hi_idx = lo_idx
        self.counts = [self.param_bucket.count(b) for b in range(len(self.buckets))]
        self.overlap = overlap and fp.gflat.is_cuda
        self.stream = torch.cuda.Stream(device=fp.gflat.device) if self.overlap else None
        self._works = []
        self._remaining = list(self.counts)
        self._launched = [False] * len(self.buckets)
        self._srcs = [[] for _ in self.buckets]
        self._inv = None
        self.buf = fp.gflat
        # defer_average: finish() leaves the sum and records the 1/world factor in
        # `pending` for the caller's clip (take_pending) instead of scaling
        self.defer_average = False
        self.pending = None
        # set to a list to time each finish(): (backward done, last bucket's all-reduce
        # done) event pairs on the compute stream -- the all-reduce time the backward did
        # not hide (bench.py exposed_allreduce_ms)
        self.timing = None
        # set to a device int64 tensor of 3 slots to stamp every finish() with the device
        # wall clock (rdn_stamp): [0] backward done, [1] last bucket's all-reduce done, [2]
        # right after [1] (the launch gap to subtract).  Unlike events, the stamps are
        # kernels, so a captured train step replays them: the exposed all-reduce time of
        # the graph path (bench.py exposed_allreduce_ms_graph, exposure_from_stamps)
        self.stamps = None

    # --- engine hooks -------------------------------------------------
    def begin(self, buf=None):
        """A backward starts producing its gradients into ``buf`` (a flat
        buffer of ``fp``'s layout; default ``fp.gflat``)."""
        self.buf = self.fp.gflat if buf is None else buf
        self.pending = None
        self._works = []
        self._remaining = list(self.counts)
        self._launched = [False] * len(self.buckets)
        self._srcs = [[] for _ in self.buckets]

    def params_done(self, indices, stream=None):
        """The gradients of these parameter indices are final on ``stream`` (the
        stream whose launch wrote them last -- the engine's weight-gradient side
        stream, or the compute stream for the fused layers; default: the current
        stream); launch every bucket that just became complete, ordered after
        EVERY stream that wrote one of its gradients.  Every rank runs the same
        backward, so buckets are issued in the same order everywhere."""
        if self.overlap:
            s = stream if stream is not None else torch.cuda.current_stream()
        for i in indices:
            b = self.param_bucket[i]
            if self.overlap and all(x.cuda_stream != s.cuda_stream for x in self._srcs[b]):
                self._srcs[b].append(s)
            self._remaining[b] -= 1
            if self._remaining[b] == 0:
                self._launch(b)

    def _launch(self, b):
        if self._launched[b]:
            return
        self._launched[b] = True
        lo, hi = self.buckets[b]
        view = self.buf[lo:hi]
        if self.overlap:
            # the host issues this after every launch that wrote the bucket, so
            # waiting on each writer stream's current tail orders the all-reduce
            # after all of them (and the finish() path after the compute stream)
            srcs = self._srcs[b] or [torch.cuda.current_stream()]
            for s in srcs:
                self.stream.wait_stream(s)
            with torch.cuda.stream(self.stream):
                self._works.append(dist.all_reduce(view, group=self.group, async_op=True))
        else:
            self._works.append(dist.all_reduce(view, group=self.group, async_op=True))

    def finish(self):
        """Launch what is left (in bucket order), wait, and average."""
        e0 = None
        if self.timing is not None and self.overlap:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream())   # the backward's last kernel is behind this
        if self.stamps is not None and self.overlap:
            self._stamp(0)
        for b in range(len(self.buckets)):
            if not self._launched[b] and self.overlap:
                self._srcs[b].append(torch.cuda.current_stream())
            self._launch(b)
        for w in self._works:
            w.wait()
        if self.overlap:
            torch.cuda.current_stream().wait_stream(self.stream)
        if e0 is not None:
            # (ProcessGroupNCCL runs an async all-reduce on its own stream, which waits on
            # self.stream -- not the other way round: an event on self.stream marks only
            # the launch.  w.wait() made the current stream wait on the collectives, so an
            # event recorded here completes when the last all-reduce has)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(torch.cuda.current_stream())
            self.timing.append((e0, e1))
        if self.stamps is not None and self.overlap:
            self._stamp(1)
            self._stamp(2)
        self._works = []
        if self.world > 1:
            if self.defer_average:
                self.pending = 1.0 / self.world
            else:
                self._average()

    def exposed_ms(self):
        """Mean over the timed finish() calls of max(0, comm end - backward end), ms
        (synchronises the device); None if nothing was timed."""
        if not self.timing:
            return None
        torch.cuda.synchronize()
        xs = [max(0.0, a.elapsed_time(b)) for a, b in self.timing]
        return sum(xs) / len(xs)

    def _stamp(self, slot):
        from . import _hip as H
        H.check(H.lib().rdn_stamp(self.stamps.data_ptr(), slot, H.stream_ptr()), "stamp")

    def take_pending(self):
        """The 1/world factor a deferred finish() left unapplied (None if none);
        the caller applies it (clip_grad_norm_flat's pre_scale)."""
        p, self.pending = self.pending, None
        return p

    def _average(self):
        g = self.buf
        if g.is_cuda:
            from . import _hip as H
            if self._inv is None:
                self._inv = torch.full((1,), 1.0 / self.world, dtype=torch.float32, device=g.device)
            H.check(H.lib().rdn_clip_scale(g.data_ptr(), g.numel(), self._inv.data_ptr(), H.stream_ptr()), "avg")
        else:
            g.mul_(1.0 / self.world)

    def sync(self):
        """Non-overlapped form: all buckets after backward."""
        self.begin()
        self.finish()
