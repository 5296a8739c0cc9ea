"""Fused RDUNet execution engine: the whole forward / backward of ``RDUNet_T`` or
``RDUNet`` as a fixed sequence of ``librdunet_hip`` launches over NHWC buffers.

Layout in HBM (per engine = per (batch, H, W, dtype, train) shape):

* level l (l = 0..3) has P_l = B*(H>>l)*(W>>l) pixels and F_l = base_filters*2^l
  channels.  Every dense block owns one buffer ``[P_l, F_l + 3*F_l/2]``: conv_k
  reads the channel prefix and writes its F_l/2 outputs behind it, so the
  reference's ``torch.cat`` calls (Unet_model.py:83,85,87) never copy.
* conv_3 (+PReLU + residual, :88-89) writes straight into the next consumer's
  buffer (the next block, or the skip/concat buffer ``CAT_l = [skip F_l | up
  F_{l+1}]`` read by ``down_l`` and ``up_l``), so ``torch.cat([concat, upsample])``
  (:43) is free as well.
* the PReLU input of every conv is kept (``PRE_*``) for the backward, as aten
  autograd keeps it; gradients of activations mirror the activation buffers.
* parameters and their gradients live in one flat fp32 buffer each (the
  nn.Parameters are views), so grad-norm clipping, the optimizer and the DDP
  all-reduce are single flat launches.

Ordering of the backward (what is stored vs accumulated) follows the
dependency order of the reference's autograd graph; see DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import warnings
import weakref
from dataclasses import dataclass, field

import torch

from . import _hip as H

_ALIGN = 64  # elements


def _ru(x, m):
    return (x + m - 1) // m * m


# ----------------------------------------------------------------- parameters
_GPOOL_MAX = 4


def _storage_refs(t: torch.Tensor) -> int:
    """Tensors sharing ``t``'s storage (``t`` itself included)."""
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata) - 1


class ParamSet:
    """A module's parameters in a fixed order at aligned offsets of one flat fp32
    index space, and the flat buffers their gradients are produced into.

    The backward writes every weight gradient of one pass into ONE flat buffer
    and hands autograd a fresh view per parameter: ``AccumulateGrad`` adopts a
    view as ``p.grad`` when ``p.grad`` is None (the usual ``zero_grad()`` loop,
    so ``.grad`` tensors are views of one flat buffer and clipping / the fused
    optimizer / the DDP all-reduce stay single launches) and adds it into
    ``p.grad`` otherwise, exactly as it does for aten's gradients;
    ``torch.autograd.grad`` returns the views themselves.  A buffer is reused only
    when no tensor references its storage any more (``p.grad`` views, grads a
    caller kept), so a pass never overwrites a gradient anyone still holds."""

    def _layout(self, module: torch.nn.Module, device):
        self.params = list(module.parameters())
        self.names = [n for n, _ in module.named_parameters()]
        self.index = {n: i for i, n in enumerate(self.names)}
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o = _ru(o + p.numel(), _ALIGN)
        self.numel = o
        self.offsets = offs
        self.device = device
        self._shapes = [tuple(p.shape) for p in self.params]
        self._strides = [torch.empty(s, device="meta").stride() for s in self._shapes]
        self._gpool = [torch.zeros(o, dtype=torch.float32, device=device)]
        self._gcur = self._gpool[0]
        self._gexpect = {}
        self.grad_sync = None   # ddp.GradSync attached by data-parallel training

    @property
    def gflat(self) -> torch.Tensor:
        """The flat buffer the ``.grad`` tensors are views of (after
        ``grads_are_views()``), else the last one a backward produced."""
        return self._gcur

    def grad_buffer(self) -> torch.Tensor:
        """A flat gradient buffer nothing references (the caller zero-fills it)."""
        for b in self._gpool:
            if _storage_refs(b) == 1:
                return b
        b = torch.empty(self.numel, dtype=torch.float32, device=self.device)
        if len(self._gpool) < _GPOOL_MAX:
            self._gpool.append(b)
        return b

    def grad_views(self, buf: torch.Tensor, which=None) -> list:
        """Fresh per-parameter views of a flat gradient buffer (None where
        ``which[i]`` is false)."""
        st = torch.as_strided
        if which is None:
            return [st(buf, s, r, o) for s, r, o in zip(self._shapes, self._strides, self.offsets)]
        return [st(buf, s, r, o) if w else None for s, r, o, w in zip(self._shapes, self._strides, self.offsets, which)]

    def grads_are_views(self) -> bool:
        """Every ``p.grad`` is its view of one pooled flat buffer; that buffer
        becomes ``gflat``."""
        ptrs = [0 if p.grad is None else p.grad.data_ptr() for p in self.params]
        for b in self._gpool:
            exp = self._gexpect.get(b.data_ptr())
            if exp is None:
                base = b.data_ptr()
                exp = self._gexpect[base] = [base + 4 * o for o in self.offsets]
            if ptrs == exp:
                self._gcur = b
                return True
        return False


class FlatParams(ParamSet):
    """Flat fp32 storage for a module's parameters (and gradients).

    The module's ``nn.Parameter`` objects keep their identity (optimizers and
    ``state_dict`` see the usual tensors) but their ``.data`` become views of
    ``self.flat``; ``.grad`` become views of a flat gradient buffer (ParamSet)."""

    def __init__(self, module: torch.nn.Module, device):
        self._layout(module, device)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.views = []
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                v = self.flat[off:off + p.numel()].view_as(p)
                v.copy_(p.data.to(device=device, dtype=torch.float32))
                p.data = v
                self.views.append(v)
        self._ptrs = [v.data_ptr() for v in self.views]
        self.generation = 0
        _FLAT_REGISTRY[:] = [r for r in _FLAT_REGISTRY if r() is not None]
        _FLAT_REGISTRY.append(weakref.ref(self))

    def intact(self) -> bool:
        """Every parameter's storage is still its view of ``flat`` (host-cheap:
        one pointer list compare; runs several times per training step)."""
        f32 = torch.float32
        return [p.data_ptr() for p in self.params] == self._ptrs and all(p.dtype is f32 for p in self.params)

    def version_key(self):
        return (self.generation, sum(p._version for p in self.params))


class BlockParams(ParamSet):
    """The parameters of one block run on its own (``DenoisingBlock(...)(x)``):
    used in place (no flat copy, so a block that is also part of a fused
    network keeps sharing the network's storage); its GEMM packs are rebuilt
    on every forward, as nothing tracks raw-pointer writes into that storage."""

    def __init__(self, module: torch.nn.Module, device):
        for n, p in module.named_parameters():
            if p.device != device or p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError(f"{type(module).__name__}: parameter {n} must be a contiguous fp32 tensor "
                                   f"on {device} (got {p.dtype} on {p.device})")
        self._layout(module, device)
        self._ptrs = [p.data_ptr() for p in self.params]
        self.generation = 0

    def intact(self) -> bool:
        return [p.data_ptr() for p in self.params] == self._ptrs

    def version_key(self):
        self.generation += 1
        return self.generation


_FLAT_REGISTRY: list = []

# Optional launch tracer (bench.py): an object with start(info) -> token|None and
# stop(token); info = (phase, layer, kernel key, algorithmic flops, algorithmic bytes).
TRACER = None

# PReLU backward is fused into a layer's dgrad/wgrad loaders when its weight-gradient
# kernel reads the gated operand in ONE input-channel chunk (re-gating it per chunk
# cost more than the separate pass it saves, r02 A/B)
FUSE_PRELU = os.environ.get("RDN_FUSE_PRELU", "1") != "0"
# weight gradients on a side stream (overlapped with the dgrad chain) and the depth
# of the dYpre ring that decouples the two chains
WGRAD_STREAM = os.environ.get("RDN_WGRAD_STREAM", "1") != "0"
# (a ring of 6 slots: 1690 / 1691 img/s against 1672 / 1673 with 4, 1681-1684 with 8,
# 1678-1682 with 12, profiles/r03_v9_slots_ab.txt; one slot per layer -- no dgrad-chain
# waits on the weight-gradient stream at all, each a ~6 us cross-queue gap in the
# replayed graph -- 1739 / 1742 against 1723 / 1724 with 6, profiles/r03_v11_slots_ab.txt;
# all interleaved on one box.  Memory: the dYpre / partial / slab buffers of every layer,
# ~1.5 GB at B16)
WGRAD_SLOTS = int(os.environ.get("RDN_WGRAD_SLOTS", "0"))   # 0: one slot per layer (within SLOT_BUDGET)
SLOT_BUDGET = float(os.environ.get("RDN_SLOT_BUDGET", "0.25"))   # fraction of free device memory
# With one slot per layer the captured graph has no edge from the weight-gradient branch
# back into the dgrad chain, and the replay enqueues the whole chain before the branch:
# harmless while the host enqueues a replay in ~1 ms, but under a profiler (slower
# enqueue) the branch then ran after the chain (10.3 vs 9.4 ms per step traced,
# profiles/r03_v13_prof_modes.txt).  Every ORDER_EVERY layers the chain therefore waits
# for the branch ORDER_EVERY layers back (a few cross-queue edges per step) to pin the
# replay order.
ORDER_EVERY = int(os.environ.get("RDN_ORDER_EVERY", "12"))
# bench.py's per-kernel profiling pass serialises the backward (isolated kernel times)
SERIAL_BWD = False
# channel-blocked ("planar") activation buffers: a level-l buffer is [C/cb, P, cb] with
# cb = F_l/2 (one plane per dense-block growth slice), so a conv reading or writing a
# channel slice touches only its planes (include/rdunet_hip.h, *_pl fields)
PLANAR = os.environ.get("RDN_PLANAR", "1") != "0"
# gated level-0 convs: input + weight gradient in one fused kernel on the compute
# stream (rdn_conv_dgrad_wgrad) instead of dgrad there and wgrad on the side stream
FUSE_DW = os.environ.get("RDN_DW", "1") != "0"
# PReLU backward of a layer fused into the input-gradient epilogue of its last
# consumer in backward order (rdn_conv_desc.gout: conv_k+1 finishes dense slice
# out_k, up_l.conv finishes up_l.conv_t's output), instead of a separate pass.
# Per launch it saves 0.5-6 us at levels 2/3 (scripts/gate_kbench.py,
# profiles/r03_v9_gate_kbench.json); with the r03 ring of dYpre slots the whole step
# measured 1666-1674 img/s with it against 1680-1691 without (profiles/r03_v9_slots_ab.txt:
# the longer finisher launches sat on the critical path beside the weight-gradient
# stream).  Round 4 (one slot per layer, column-half dw, conv3_big prefetch), interleaved:
# +0.2 % B16 / +0.2 % B32 on top of the prefetch (profiles/r04_v5_big_pf_gate_out_ab.txt):
# on by default.  Tested both ways (tests/test_gpu_gateout.py).
GATE_OUT = os.environ.get("RDN_GATE_OUT", "1") == "1"
# gate-out in the fused dgrad+wgrad kernel (conv3_dw ",go": up_0.conv finishing
# up_0.conv_t, the level-1 conv_0s finishing down_0 / the previous block's conv_3)
GATE_OUT_DW = os.environ.get("RDN_GATE_OUT_DW", "1") == "1"
# round 5: the level-1 conv_3 (160 input channels, 64 dY channels) as ONE fused dgrad +
# wgrad launch in five 32-channel parts (conv3_dw "h5") instead of conv3_big dgrad on
# the compute stream + wgrad3_glds on the side stream.  Pre-gated: the kernel reads the
# layer's dYpre, gated once by a gate-out finisher or the PReLU-backward pass (gated in
# each part's loader, the five parts gated the same tile five times: 143 vs 101 us per
# launch at B16, profiles/r05_*); RDN_DW_PREGATED=0 gates in the loaders instead
DW_PREGATED = os.environ.get("RDN_DW_PREGATED", "1") != "0"
# the fused layers' split-K reduces of consecutive fused layers in one launch
# (rdn_wgrad_reduce_batch; RDN_REDUCE_BATCH=0: one launch per layer)
REDUCE_BATCH = os.environ.get("RDN_REDUCE_BATCH", "1") != "0"
# conv_0..conv_2 of every level-0 DenoisingBlock (base_filters 32, bf16) as ONE
# launch that reads x once and keeps out_0 / out_1 on chip (rdn_dense3_fwd)
FUSE_DENSE = os.environ.get("RDN_DENSE", "1") != "0"
# round 6: the level-1 blocks' conv_0..2 as one launch too (conv3_dense1.hip); RDN_DENSE1=0
# keeps them on the three rdn_conv_fwd launches (A/B)
FUSE_DENSE1 = os.environ.get("RDN_DENSE1", "1") != "0"
# round 6: 3x3 forwards whose pixel grid covers under half of the CUs (a batch-1
# forward's deep levels) run split-K (rdn_conv_fwd_splitk; RDN_SPLITK=0: off)
SPLITK = os.environ.get("RDN_SPLITK", "1") != "0"
# round 6: the weight-gradient stream's split-K reduces of this many consecutive
# layers in one rdn_wgrad_reduce_batch launch (each layer its own slab of a ring;
# RDN_SIDE_BATCH=1: one reduce launch per layer, as before)
SIDE_BATCH = max(1, min(8, int(os.environ.get("RDN_SIDE_BATCH", "4"))))
# forward-only batches are run in chunks of at most this many pixels (run_unet)
FWD_CHUNK_PIXELS = 1 << 23


def find_flat(params):
    """The FlatParams whose parameter list is exactly ``params`` (same objects,
    same order) with every gradient its view of one flat gradient buffer
    (which becomes its ``gflat``), else None."""
    params = list(params)
    for ref in _FLAT_REGISTRY:
        fp = ref()
        if fp is None or len(fp.params) != len(params):
            continue
        if all(a is b for a, b in zip(fp.params, params)) and fp.intact() and fp.grads_are_views():
            return fp
    return None


def flat_params(module: torch.nn.Module, device) -> FlatParams:
    fp = getattr(module, "_rdn_flat", None)
    if fp is None or fp.device != device or not fp.intact():
        fp = FlatParams(module, device)
        module._rdn_flat = fp
        module._rdn_packs = {}
        module._rdn_engines = {}
    return fp


def block_params(module: torch.nn.Module, device) -> BlockParams:
    bp = getattr(module, "_rdn_flat", None)
    if bp is None or bp.device != device or not bp.intact():
        bp = BlockParams(module, device)
        module._rdn_flat = bp
        module._rdn_packs = {}
        module._rdn_engines = {}
    return bp


# ----------------------------------------------------------------- layer plan
@dataclass
class Slice:
    """An NHWC channel slice: buffer name, channel offset."""
    buf: str
    c0: int = 0


@dataclass
class ConvLayer:
    name: str                 # module prefix, e.g. "block_0_0.conv_1"
    act: str                  # PReLU prefix, e.g. "block_0_0.actv_1"
    kind: str                 # "c3" | "down" | "up"
    level: int                # level of the GEMM rows in forward (c3/down: output; up: input)
    cin: int                  # real input channels
    cin_pad: int
    cout: int                 # real output channels
    cout_pad: int
    src: Slice                # forward input
    dst: Slice | None         # forward output (None -> NCHW image)
    pre: str                  # pre-activation buffer name
    resid: Slice | None = None  # residual added after PReLU (dense conv_3)
    resid_c: int = 0
    dsrc: Slice | None = None   # gradient of the input slice (None -> not needed)
    accum: bool = False         # dgrad accumulates (else stores)
    ddst: Slice | None = None   # gradient arriving at dst (None -> NCHW dy)
    fwd_desc: object = None
    dgrad_desc: object = None
    wgrad_desc: object = None
    wgrad_splits: int = 0
    pack_fwd: tuple = ()
    pack_dgrad: tuple = ()
    extra: dict = field(default_factory=dict)


@dataclass
class Program:
    """What one engine runs: forward-ordered convs over named NHWC buffers
    ``{name: (level, channels)}`` (level l = the input grid halved l times).

    ``inputs`` are the NCHW fp32 tensors of forward, each stored at channel 0 of
    its buffer ``(buffer, level, channels)``; ``image_input``: input 0 is the network's
    image, packed into 8-channel rows by ``rdn_pack_input``, with the broadcast t
    map as its next channel when ``time_input`` (RDUNet_T).  The last conv writes
    the NCHW fp32 output of level ``out_level``, adding ``inputs[0]`` when
    ``resid_input`` (the network's ``+ inputs``, Unet_model.py:166, or a dense
    block's ``out_3 + x``, :89).  ``cb``: level -> plane width of the
    channel-blocked buffers of that level (none: plain NHWC)."""
    layers: list
    bufs: dict
    inputs: list
    out_level: int
    out_channels: int
    resid_input: bool
    time_input: bool = False
    image_input: bool = False
    cb: dict = field(default_factory=dict)
    min_div: int = 1


def _plan(F0: int, cin_img: int, has_t: bool, cout_img: int) -> Program:
    """The whole network (Unet_model.py:92-166 / RDUNet_model.py)."""
    F = [F0 << l for l in range(4)]
    D = [f + 3 * (f // 2) for f in F]
    bufs = {"IN": (0, 8), "IB1": (0, F[0]), "O6": (0, F[0]), "OB1": (0, F[0]),
            "PRE_OUT": (0, 8)}
    for l in range(4):
        for k in range(4 if l < 3 else 2):
            bufs[f"B{l}{k}"] = (l, D[l])
        if l < 3:
            bufs[f"CAT{l}"] = (l, F[l] + F[l + 1])
        if l > 0:
            bufs[f"U{l}"] = (l, F[l])
    layers: list[ConvLayer] = []

    def c3(name, act, level, cin, cout, src, dst, pre_c, resid=None, resid_c=0, cin_pad=None, cout_pad=None):
        pre = f"PRE_{name}"
        bufs[pre] = (level, cout_pad or cout)
        layers.append(ConvLayer(name, act, "c3", level, cin, cin_pad or cin, cout, cout_pad or cout,
                                src, dst, pre, resid, resid_c))

    cin_in = cin_img + (1 if has_t else 0)
    c3("input_block.conv_1", "input_block.actv_1", 0, cin_in, F[0], Slice("IN"), Slice("IB1"), 0, cin_pad=8)
    c3("input_block.conv_2", "input_block.actv_2", 0, F[0], F[0], Slice("IB1"), Slice("B00"), 0)

    def dense(blk, l, buf, dst):
        C_, i = F[l], F[l] // 2
        for k in range(3):
            c3(f"{blk}.conv_{k}", f"{blk}.actv_{k}", l, C_ + k * i, i, Slice(buf), Slice(buf, C_ + k * i), 0)
        c3(f"{blk}.conv_3", f"{blk}.actv_3", l, C_ + 3 * i, C_, Slice(buf), dst, 0, resid=Slice(buf), resid_c=C_)

    def down(l):
        pre = f"PRE_down_{l}"
        bufs[pre] = (l + 1, F[l + 1])
        layers.append(ConvLayer(f"down_{l}.conv", f"down_{l}.actv", "down", l + 1, F[l], F[l], F[l + 1], F[l + 1],
                                Slice(f"CAT{l}"), Slice(f"B{l + 1}0"), pre))

    def up(l):
        # ConvTranspose2d(F[l+1] -> F[l+1]) then Conv2d(F[l] + F[l+1] -> F[l])
        pre = f"PRE_up_{l}_t"
        bufs[pre] = (l, F[l + 1])
        layers.append(ConvLayer(f"up_{l}.conv_t", f"up_{l}.actv_t", "up", l + 1, F[l + 1], F[l + 1], F[l + 1],
                                F[l + 1], Slice(f"U{l + 1}"), Slice(f"CAT{l}", F[l]), pre))
        c3(f"up_{l}.conv", f"up_{l}.actv", l, F[l] + F[l + 1], F[l], Slice(f"CAT{l}"), Slice(f"B{l}2"), 0)

    dense("block_0_0", 0, "B00", Slice("B01"))
    dense("block_0_1", 0, "B01", Slice("CAT0"))
    down(0)
    dense("block_1_0", 1, "B10", Slice("B11"))
    dense("block_1_1", 1, "B11", Slice("CAT1"))
    down(1)
    dense("block_2_0", 2, "B20", Slice("B21"))
    dense("block_2_1", 2, "B21", Slice("CAT2"))
    down(2)
    dense("block_3_0", 3, "B30", Slice("B31"))
    dense("block_3_1", 3, "B31", Slice("U3"))
    up(2)
    dense("block_2_2", 2, "B22", Slice("B23"))
    dense("block_2_3", 2, "B23", Slice("U2"))
    up(1)
    dense("block_1_2", 1, "B12", Slice("B13"))
    dense("block_1_3", 1, "B13", Slice("U1"))
    up(0)
    dense("block_0_2", 0, "B02", Slice("B03"))
    dense("block_0_3", 0, "B03", Slice("O6"))
    c3("output_block.conv_1", "output_block.actv_1", 0, F[0], F[0], Slice("O6"), Slice("OB1"), 0)
    layers.append(ConvLayer("output_block.conv_2", "output_block.actv_2", "c3", 0, F[0], F[0], cout_img, 8,
                            Slice("OB1"), None, "PRE_OUT"))
    return Program(layers, bufs, [("IN", 0, cin_img)], 0, cout_img, True, time_input=has_t, image_input=True,
                   cb={l: F[l] // 2 for l in range(4)}, min_div=8)


def block_program(block) -> Program:
    """One block of Unet_model.py:23-89 on its own: NCHW fp32 in and out, the
    same kernels and buffer conventions as inside the network.  Channel counts
    on a conv's input side must be multiples of 8 (the NHWC K chunks); the
    input block's image channels and the output block's image channels are
    padded to 8."""
    kind = type(block).__name__
    bufs: dict = {}
    layers: list[ConvLayer] = []

    def need8(*cs):
        for c in cs:
            if c % 8:
                raise ValueError(f"{kind}: the GPU kernels need channel counts that are multiples of 8; got {c}")

    def c3(name, act, cin, cout, src, dst, cout_pad=None):
        bufs[f"PRE_{name}"] = (0, cout_pad or cout)
        layers.append(ConvLayer(name, act, "c3", 0, cin, _ru(cin, 8), cout, cout_pad or cout, src, dst,
                                f"PRE_{name}"))

    if kind == "DenoisingBlock":       # :69-89
        C_, i, Co = block.conv_0.in_channels, block.conv_0.out_channels, block.conv_3.out_channels
        if Co != C_:
            raise ValueError(f"DenoisingBlock: out_3 + x needs out_channels == in_channels ({Co} != {C_})")
        need8(C_, i)
        bufs["X"] = (0, C_ + 3 * i)
        for k in range(3):
            c3(f"conv_{k}", f"actv_{k}", C_ + k * i, i, Slice("X"), Slice("X", C_ + k * i))
        c3("conv_3", "actv_3", C_ + 3 * i, Co, Slice("X"), None)
        return Program(layers, bufs, [("X", 0, C_)], 0, Co, True)
    if kind == "InputBlock":           # :45-55
        cin, F = block.conv_1.in_channels, block.conv_1.out_channels
        need8(F)
        bufs["X"], bufs["Y1"] = (0, _ru(cin, 8)), (0, F)
        c3("conv_1", "actv_1", cin, F, Slice("X"), Slice("Y1"))
        c3("conv_2", "actv_2", F, F, Slice("Y1"), None)
        return Program(layers, bufs, [("X", 0, cin)], 0, F, False)
    if kind == "OutputBlock":          # :57-67
        F, co = block.conv_1.in_channels, block.conv_2.out_channels
        need8(F)
        bufs["X"], bufs["Y1"] = (0, F), (0, F)
        c3("conv_1", "actv_1", F, F, Slice("X"), Slice("Y1"))
        c3("conv_2", "actv_2", F, co, Slice("Y1"), None, cout_pad=_ru(co, 8))
        return Program(layers, bufs, [("X", 0, F)], 0, co, False)
    if kind == "DownsampleBlock":      # :23-30
        cin, co = block.conv.in_channels, block.conv.out_channels
        need8(cin, co)
        bufs["X"], bufs["PRE_conv"] = (0, cin), (1, co)
        layers.append(ConvLayer("conv", "actv", "down", 1, cin, cin, co, co, Slice("X"), None, "PRE_conv"))
        return Program(layers, bufs, [("X", 0, cin)], 1, co, False, min_div=2)
    if kind == "UpsampleBlock":        # :32-43, forward((upsample, concat))
        cu, co = block.conv_t.in_channels, block.conv.out_channels
        cc = block.conv.in_channels - cu
        need8(cu, cc, co)
        bufs["U"], bufs["CAT"], bufs["PRE_conv_t"] = (1, cu), (0, cc + cu), (0, cu)
        layers.append(ConvLayer("conv_t", "actv_t", "up", 1, cu, cu, cu, cu, Slice("U"), Slice("CAT", cc),
                                "PRE_conv_t"))
        c3("conv", "actv", cc + cu, co, Slice("CAT"), None)
        return Program(layers, bufs, [("U", 1, cu), ("CAT", 0, cc)], 0, co, False)
    raise TypeError(f"no GPU program for {kind}")


def _assign_backward(layers):
    """Gradient routing: which slice receives each layer's input gradient and
    whether it is the first (store) or a later (accumulate) contribution, in
    backward (reverse) execution order."""
    written = set()
    # gradient arriving at a layer's output = gradient slice of its dst
    for L in layers:
        L.ddst = None if L.dst is None else Slice("d" + L.dst.buf, L.dst.c0)
    for L in reversed(layers):
        L.dsrc = Slice("d" + L.src.buf, L.src.c0)
        L.accum = L.dsrc.buf in written
        written.add(L.dsrc.buf)


# ----------------------------------------------------------------- weight packing
class WeightPacks:
    """Packed (GEMM-operand) copies of the conv weights for one dtype, rebuilt
    when the parameters change (optimizer step, load_state_dict).  Shared by
    every engine (input shape) of the module."""

    def __init__(self, module, fp: FlatParams, layers, dtype):
        self.dtype = dtype
        self.code = H.dtype_code(dtype)
        self.fp = fp
        self.key = None
        self.fwd, self.dgrad = {}, {}
        named = dict(module.named_parameters())
        dev = fp.device

        lib = H.lib()

        def mk(mode, w, d0, d1, kh, kw, pad0, pad1, rows, kp, ck=0):
            out = torch.zeros(_ru(rows, 128), _ru(kp, 64), dtype=dtype, device=dev)
            return (mode, w, d0, d1, kh, kw, pad0, pad1, out, out.shape[0], out.shape[1], ck)

        def chunk(c):
            ck, kp = lib.rdn_conv3_chunk(c, self.code), lib.rdn_conv3_packed_k(c, self.code)
            if ck <= 0 or kp <= 0:
                raise RuntimeError(f"conv3 K side of {c} channels unsupported")
            return ck, kp

        for L in layers:
            w = named[L.name + ".weight"]
            if L.kind == "c3":       # Conv2d 3x3 W[co][ci][3][3], chunked K for the halo kernel
                ck, kp = chunk(L.cin_pad)
                self.fwd[L.name] = mk(H.PACK_CONV_FWD, w, L.cout, L.cin, 3, 3, 0, L.cin_pad, L.cout, kp, ck)
                ck, kp = chunk(L.cout_pad)
                self.dgrad[L.name] = mk(H.PACK_CONV_DGRAD, w, L.cout, L.cin, 3, 3, L.cout_pad, 0, L.cin, kp, ck)
            elif L.kind == "down":   # Conv2d 2x2 s2 W[co][ci][2][2]
                self.fwd[L.name] = mk(H.PACK_CONV_FWD, w, L.cout, L.cin, 2, 2, 0, L.cin, L.cout, 4 * L.cin)
                self.dgrad[L.name] = mk(H.PACK_GEMM_T, w, L.cout, L.cin, 2, 2, L.cout, 0, 4 * L.cin, L.cout)
            else:                    # ConvTranspose2d 2x2 s2 W[ci][co][2][2]
                self.fwd[L.name] = mk(H.PACK_GEMM_T, w, L.cin, L.cout, 2, 2, L.cin, 0, 4 * L.cout, L.cin)
                self.dgrad[L.name] = mk(H.PACK_CONV_FWD, w, L.cin, L.cout, 2, 2, 0, L.cout, L.cin, 4 * L.cout)
        self.items = list(self.fwd.values()) + list(self.dgrad.values())
        arr = (H.PackItem * len(self.items))()
        for i, (mode, w, d0, d1, kh, kw, pad0, pad1, out, rows, kp, ck) in enumerate(self.items):
            arr[i] = H.PackItem(w.data_ptr(), out.data_ptr(), mode, d0, d1, kh, kw, pad0, pad1, rows, kp, ck)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.items_dev = raw.to(dev)   # device copy of the descriptors: one launch packs all

    def attach(self, layers):
        for L in layers:
            L.pack_fwd = self.fwd[L.name]
            L.pack_dgrad = self.dgrad[L.name]

    def refresh(self):
        key = self.fp.version_key()
        if key == self.key:
            return
        H.check(H.lib().rdn_pack_weights_batched(self.items_dev.data_ptr(), len(self.items), self.code,
                                                 H.stream_ptr()), "pack_weights_batched")
        self.key = key


def weight_packs(module, fp, layers, dtype) -> WeightPacks:
    wp = module._rdn_packs.get(dtype)
    if wp is None:
        wp = WeightPacks(module, fp, layers, dtype)
        module._rdn_packs[dtype] = wp
    return wp


# ----------------------------------------------------------------- engine
# descriptor pointers that select a kernel variant (kept as they are by the probes)
_CONV_SELECT = ("gate", "gate_alpha", "gout", "gout_pre", "gout_alpha", "gout_part")


class UNetEngine:
    """Buffers and prebuilt launch descriptors of one Program (the network, or
    one block) for one input shape (B, H, W of level 0)."""

    def __init__(self, module, B, Hh, Ww, dtype, train: bool, prog: Program | None = None, params=None,
                 scratch: dict | None = None):
        if prog is None:
            F0 = module.base_filters
            if F0 % 16:
                raise RuntimeError(f"base_filters must be a multiple of 16 for the NHWC/MFMA layout; got {F0}")
            prog = _plan(F0, module.image_channels, module.time_conditioned, module.out_channels)
        if Hh % prog.min_div or Ww % prog.min_div:
            raise RuntimeError(f"{type(module).__name__} needs H and W divisible by {prog.min_div}; got {Hh}x{Ww}")
        self.module = module
        self.prog = prog
        # backward-only buffers (activation gradients, dYpre / partial / slab slots,
        # workspaces), shared by every grad-enabled engine of one (shape, dtype) pool:
        # backwards run one after another on the compute stream (each ends by waiting
        # for its weight-gradient stream), so one set serves all of them and a pooled
        # engine costs only its forward activations and PReLU inputs
        self.scratch = {} if scratch is None else scratch
        self.B, self.H, self.W = B, Hh, Ww
        self.dtype = dtype
        self.code = H.dtype_code(dtype)
        self.train = train
        self.module_training = bool(getattr(module, "training", False))
        dev = next(module.parameters()).device
        self.device = dev
        self.fp = params if params is not None else flat_params(module, dev)
        layers, bufspec = prog.layers, prog.bufs
        _assign_backward(layers)
        self.layers = layers
        self.packs = weight_packs(module, self.fp, layers, dtype)
        self.packs.attach(layers)
        self.P = [B * (Hh >> l) * (Ww >> l) for l in range(4)]
        self.grid = [(B, Hh >> l, Ww >> l) for l in range(4)]
        self.bufs = {}
        self.geo = {}   # buffer name -> (pixel stride ps, plane stride pl); pl = 0: plain NHWC
        in_bufs = {b for b, _, _ in prog.inputs}
        # buffers no layer writes in forward (pure inputs): their layers' input
        # gradients are only computed when that input needs a gradient
        self.pure_inputs = in_bufs - {L.dst.buf for L in layers if L.dst is not None}

        def alloc(name, lvl, ch, shared=False):
            cb = prog.cb.get(lvl, 0)
            if (PLANAR and cb and name not in in_bufs and name[1:] not in in_bufs and not name.startswith("PRE_")
                    and ch % cb == 0 and ch > cb):
                pl = self.P[lvl] * cb
                shape = (ch // cb, pl)
                self.geo[name] = (cb, pl)
            else:
                shape = (self.P[lvl], ch)
                self.geo[name] = (ch, 0)
            if shared:
                t = self._shared(("buf", name), lambda: torch.zeros(shape, dtype=dtype, device=dev))
            else:
                t = torch.zeros(shape, dtype=dtype, device=dev)
            self.bufs[name] = t

        for name, (lvl, ch) in bufspec.items():
            if not train and name.startswith("PRE_"):
                continue
            alloc(name, lvl, ch)
        self.named = dict(module.named_parameters())
        self._build_fwd()
        self._plan_dense3()
        if train:
            for name, (lvl, ch) in bufspec.items():
                if name.startswith("PRE_"):
                    continue
                alloc("d" + name, lvl, ch, shared=True)
            # weight gradients (wgrad + reduce) run on a side stream, overlapped with
            # the dgrad chain; the dYpre / PReLU-partial / slab buffers they read live in
            # SLOTS slots (layer b of the backward order uses slot b % SLOTS), each sized
            # for the largest layer that uses it; the dgrad chain waits for the side
            # stream only where it reuses a slot (default: one slot per layer, no waits)
            # (a high-priority side stream measured 1215 vs 1892 img/s B16, r06: not kept)
            self.side = torch.cuda.Stream(device=dev) if (dev.type == "cuda" and WGRAD_STREAM) else None
            if self.side is None:
                self.slots = 1
            elif WGRAD_SLOTS > 0:
                self.slots = min(WGRAD_SLOTS, len(layers))
            else:
                # one slot per layer while its dYpre buffers stay within a quarter of the
                # free device memory (1.5 GB at B16 256^2, 6 GB at B64 or 512^2 crops;
                # RDN_SLOT_BUDGET), else the 6-slot ring of round 3 (-1 % step)
                # (decided once per pool: its engines share the slot buffers)
                def pick():
                    need = sum(self.P[self._out_level(L)] * L.cout_pad for L in layers) * (2 if dtype == torch.bfloat16 else 4)
                    free = torch.cuda.mem_get_info(dev)[0]
                    return len(layers) if need <= SLOT_BUDGET * free else min(6, len(layers))
                self.slots = self._shared("slots", pick)
            sizes = [0] * self.slots
            for b, L in enumerate(reversed(layers)):
                sizes[b % self.slots] = max(sizes[b % self.slots], self.P[self._out_level(L)] * L.cout_pad)
            self.dyp = [self._shared(("dyp", i), lambda n=n: torch.zeros(n, dtype=dtype, device=dev))
                        for i, n in enumerate(sizes)]
            self._build_bwd()
        self._build_info()
        self.lease = None   # weakref to the autograd graph's lease while it owns the activations
        self.lease_seq = 0

    # ------------------------------------------------------------------
    def _shared(self, key, make):
        """A backward scratch buffer of this engine's pool (made on first use)."""
        t = self.scratch.get(key)
        if t is None:
            t = self.scratch[key] = make()
        return t

    def _out_level(self, L):
        return L.level - 1 if L.kind == "up" else L.level

    def _buf(self, name):
        return self.bufs[name]

    def _slice(self, sl):
        """(pointer, ps, c0, pl) of a channel slice of a buffer."""
        ps, pl = self.geo[sl.buf]
        return self.bufs[sl.buf].data_ptr(), ps, sl.c0, pl

    def _build_fwd(self):
        lib = H.lib()
        for L in self.layers:
            d = H.ConvDesc()
            d.dtype = self.code
            n, h, w = self.grid[L.level]
            d.n, d.h, d.w = n, h, w
            d.x, d.x_ps, d.x_c0, d.x_pl = self._slice(L.src)
            packed = L.pack_fwd[8]
            d.wp, d.kp = packed.data_ptr(), packed.shape[1]
            d.bias = self.named[L.name + ".bias"].data_ptr()
            d.alpha = self.named[L.act + ".weight"].data_ptr()
            flags = H.EPI_BIAS | H.EPI_PRELU
            pre = self.bufs.get(L.pre)
            if self.train:
                flags |= H.EPI_STORE_PRE
                d.pre, d.pre_ps = pre.data_ptr(), pre.shape[1]
            if L.kind == "c3":
                d.gather = H.RDN_G_CONV3
                d.hin, d.win = h, w
                d.cin = L.cin_pad
                d.ncols, d.cout = L.cout, L.cout
            elif L.kind == "down":
                d.gather = H.RDN_G_S2
                d.hin, d.win = 2 * h, 2 * w
                d.cin = L.cin
                d.ncols, d.cout = L.cout, L.cout
            else:
                d.gather = H.RDN_G_PIX
                d.hin, d.win = h, w
                d.cin = L.cin
                d.ncols, d.cout = 4 * L.cout, L.cout
                flags |= H.EPI_SCATTER2
            if L.dst is None:
                flags |= H.EPI_OUT_NCHW
                if self.prog.resid_input:   # + inputs (Unet_model.py:166) / out_3 + x (:89)
                    flags |= H.EPI_RESID
            else:
                d.out, d.out_ps, d.out_c0, d.out_pl = self._slice(L.dst)
                if L.resid is not None:
                    flags |= H.EPI_RESID
                    d.res, d.res_ps, d.res_c0, d.res_pl = self._slice(L.resid)
                    d.res_climit = L.resid_c
            d.flags = flags
            L.fwd_desc = d
        self._plan_splitk()

    def _plan_splitk(self):
        """Split-K slices of the forwards whose tile grid leaves most CUs idle
        (rdn_conv_fwd_splits > 0: a batch-1 forward's level-2/3 convs, 256 / 64 pixels
        at 64^2) and one workspace for their fp32 slices; forward-only engines (the
        samplers, config 1's RDUNet forward)."""
        if not SPLITK or self.train or self.module_training:
            # (forward-only engines of a module in eval mode: the samplers, inference.  A
            # train step's gradients at batch 1 are sums over a few thousand pixels, so the
            # fp32 reordering can flip a PReLU gate whose input is within noise of 0 and
            # move a whole gradient by ~1/sqrt(pixels): train engines keep the single-pass
            # launches; and a train-mode forward-only call -- the logged loss of a step whose
            # gradient the reference discards, diffusion_RDUnet.forward_step_device -- keeps
            # the train engine's kernels, so its loss is the train step's bit for bit)
            return
        lib = H.lib()
        need = 0
        for L in self.layers:
            s = lib.rdn_conv_fwd_splits(C.byref(L.fwd_desc))
            if s > 0:
                L.extra["splitk"] = s
                need = max(need, lib.rdn_conv_fwd_splitk_workspace_size(C.byref(L.fwd_desc), s))
        if need:
            self.ws_fwd = torch.empty(need // 4 + 4, dtype=torch.float32, device=self.device)

    def _plan_dense3(self):
        """Dense blocks whose conv_0..conv_2 forward runs as one rdn_dense3_fwd launch
        (Unet_model.py:81-87): level 0 (x = 32 channels, growth 16, 16-channel planes)
        and, round 6, level 1 (x = 64 channels, growth 32, 32-channel planes; the
        level-1 grid a multiple of 16).  The three layers read the block buffer's
        channel prefix and write its next planes; the launch goes at conv_0, the other
        two are skipped."""
        if not FUSE_DENSE or self.code != H.RDN_BF16:
            return
        by_name = {L.name: L for L in self.layers}
        for L0 in self.layers:
            if not L0.name.endswith(".conv_0") or L0.kind != "c3" or L0.level not in (0, 1):
                continue
            lvl = L0.level
            if lvl == 1 and not FUSE_DENSE1:
                continue
            n, h, w = self.grid[lvl]
            if (lvl == 0 and (h % 8 or w % 16)) or (lvl == 1 and (h % 16 or w % 16)):
                continue
            g, x_c = (16, 32) if lvl == 0 else (32, 64)
            blk = L0.name[:-len(".conv_0")]
            Ls = [by_name.get(f"{blk}.conv_{k}") for k in range(3)]
            if any(L is None or L.kind != "c3" or L.level != lvl for L in Ls):
                continue
            buf = L0.src.buf
            ps, pl = self.geo[buf]
            if (ps != g or not pl or any(L.src.buf != buf or L.src.c0 != 0 or L.dst is None or L.dst.buf != buf
                                           or L.cout != g or L.cout_pad != g or L.resid is not None for L in Ls)
                    or [L.cin for L in Ls] != [x_c, x_c + g, x_c + 2 * g]
                    or [L.dst.c0 for L in Ls] != [x_c, x_c + g, x_c + 2 * g]):
                continue
            d = H.Dense3Desc()
            d.n, d.h, d.w = n, h, w
            d.x_c = x_c
            d.x, d.x_pl = self.bufs[buf].data_ptr(), pl
            for k, L in enumerate(Ls):
                ptr, _, c0, _ = self._slice(L.dst)
                d.out[k] = ptr + 2 * (c0 // ps) * pl
                pre = self.bufs.get(L.pre)
                d.pre[k] = pre.data_ptr() if pre is not None else None   # (forward-only: none kept)
                packed = L.pack_fwd[8]
                d.wp[k], d.kp[k] = packed.data_ptr(), packed.shape[1]
                d.bias[k] = self.named[L.name + ".bias"].data_ptr()
                d.alpha[k] = self.named[L.act + ".weight"].data_ptr()
            L0.extra["dense3"] = d
            for L in Ls[1:]:
                L.extra["dense3_skip"] = True

    def _build_bwd(self):
        lib = H.lib()
        ws_need = 0
        for b, L in enumerate(reversed(self.layers)):   # backward order -> ring slot
            L.extra["slot"] = b % self.slots
            L.extra["bidx"] = b
            L.extra["dyp"] = self.dyp[L.extra["slot"]].data_ptr()
        for L in self.layers:
            olvl = self._out_level(L)
            dyp = L.extra["dyp"]
            # 3x3 convs whose output gradient arrives as an NHWC slice run the
            # PReLU backward inside their dgrad / wgrad loaders (gate = saved
            # PReLU input); the output conv (NCHW dy) and the 2x2 convs keep
            # the separate rdn_prelu_bwd pass producing dYpre.
            gate_ok = (L.kind == "c3" and L.ddst is not None) and FUSE_PRELU
            fused = gate_ok
            if fused:  # only when the wgrad reads operand A (with the gate) in one chunk
                n_, h_, w_ = self.grid[L.level]
                probe = H.WgradDesc(dtype=self.code, gather=H.RDN_G_CONV3, n=n_, h=h_, w=w_, hin=h_, win=w_,
                                    mdim=L.cout, ndim=L.cin_pad)
                fused = lib.rdn_wgrad_chunks(C.byref(probe)) == 1
            pre = self.bufs[L.pre]
            alpha = self.named[L.act + ".weight"]
            pure = L.src.buf in self.pure_inputs

            def build(fused):
                # --- input gradient (dgrad) as a forward-shaped conv over dYpre
                d = H.ConvDesc()
                d.dtype = self.code
                packed = L.pack_dgrad[8]
                d.wp, d.kp = packed.data_ptr(), packed.shape[1]
                d.x, d.x_c0 = dyp, 0
                flags = 0
                if L.kind == "c3":
                    n, h, w = self.grid[L.level]
                    d.gather, d.hin, d.win = H.RDN_G_CONV3, h, w
                    d.x_ps, d.cin = L.cout_pad, L.cout_pad
                    d.ncols = d.cout = L.cin
                    if fused:
                        d.x, d.x_ps, d.x_c0, d.x_pl = self._slice(L.ddst)
                        d.gate, d.gate_ps, d.gate_alpha = pre.data_ptr(), pre.shape[1], alpha.data_ptr()
                elif L.kind == "down":       # per-pixel GEMM on the low-res grid, scattered to 2x2
                    n, h, w = self.grid[L.level]
                    d.gather, d.hin, d.win = H.RDN_G_PIX, h, w
                    d.x_ps, d.cin = L.cout, L.cout
                    d.ncols, d.cout = 4 * L.cin, L.cin
                    flags |= H.EPI_SCATTER2
                else:                        # conv-s2 gather of the hi-res dYpre
                    n, h, w = self.grid[L.level]
                    d.gather, d.hin, d.win = H.RDN_G_S2, 2 * h, 2 * w
                    d.x_ps, d.cin = L.cout, L.cout
                    d.ncols = d.cout = L.cin
                d.n, d.h, d.w = n, h, w
                d.out, d.out_ps, d.out_c0, d.out_pl = self._slice(L.dsrc)
                if L.accum:
                    flags |= H.EPI_ACCUM
                if L.resid is not None:      # d(x) += dOut through "out_3 + x" (Unet_model.py:89)
                    flags |= H.EPI_RESID
                    d.res, d.res_ps, d.res_c0, d.res_pl = self._slice(L.ddst)
                    d.res_climit = L.resid_c
                d.flags = flags
                # --- weight gradient
                wg = H.WgradDesc()
                wg.dtype = self.code
                if L.kind == "c3":
                    n, h, w = self.grid[L.level]
                    wg.gather, wg.n, wg.h, wg.w, wg.hin, wg.win = H.RDN_G_CONV3, n, h, w, h, w
                    wg.a, wg.a_ps, wg.a_c0, wg.mdim = dyp, L.cout_pad, 0, L.cout
                    wg.b, wg.b_ps, wg.b_c0, wg.b_pl = self._slice(L.src)
                    wg.ndim = L.cin_pad
                    taps, ndim_real = 9, L.cin
                    if fused:
                        wg.a, wg.a_ps, wg.a_c0, wg.a_pl = self._slice(L.ddst)
                        wg.a_gate, wg.a_gate_ps, wg.a_gate_alpha = pre.data_ptr(), pre.shape[1], alpha.data_ptr()
                elif L.kind == "down":
                    n, h, w = self.grid[L.level]
                    wg.gather, wg.n, wg.h, wg.w, wg.hin, wg.win = H.RDN_G_S2, n, h, w, 2 * h, 2 * w
                    wg.a, wg.a_ps, wg.a_c0, wg.mdim = dyp, L.cout, 0, L.cout
                    wg.b, wg.b_ps, wg.b_c0, wg.b_pl = self._slice(L.src)
                    wg.ndim = L.cin
                    taps, ndim_real = 4, L.cin
                else:
                    n, h, w = self.grid[L.level]
                    wg.gather, wg.n, wg.h, wg.w, wg.hin, wg.win = H.RDN_G_S2, n, h, w, 2 * h, 2 * w
                    wg.a, wg.a_ps, wg.a_c0, wg.a_pl = self._slice(L.src)
                    wg.mdim = L.cin
                    wg.b, wg.b_ps, wg.b_c0, wg.ndim = dyp, L.cout, 0, L.cout
                    taps, ndim_real = 4, L.cout
                return d, wg, taps, ndim_real

            d, wg, taps, ndim_real = build(fused)
            dw = 0
            pregated = False
            if gate_ok and FUSE_DW and not pure and not fused and DW_PREGATED:
                # the pre-gated fused kernel (dYpre from the PReLU pass / a gate-out finisher)
                pregated = lib.rdn_conv_dgrad_wgrad_splits(C.byref(d), C.byref(wg)) > 0
            if gate_ok and FUSE_DW and not pure and not pregated:
                # the fused dgrad + wgrad kernel gates in its own loader, also for the
                # multi-chunk level-1 convs (column halves, rdn_conv_dgrad_wgrad_cols)
                dg, wgg, _, _ = (d, wg, taps, ndim_real) if fused else build(True)
                wgg.splits = 0
                wgg.splits = lib.rdn_wgrad_splits(C.byref(wgg))
                dw = lib.rdn_conv_dgrad_wgrad_splits(C.byref(dg), C.byref(wgg))
                if dw > 0 and not fused:
                    fused, d, wg = True, dg, wgg
            L.extra["fused"] = fused
            L.dgrad_desc = d
            wg.splits = 0
            splits = lib.rdn_wgrad_splits(C.byref(wg))
            wg.splits = splits
            dw = 0
            if (fused or pregated) and FUSE_DW and L.src.buf not in self.pure_inputs:
                dw = lib.rdn_conv_dgrad_wgrad_splits(C.byref(d), C.byref(wg))
            L.extra["dw"] = dw > 0
            L.extra["dw_bytes"] = 0
            L.extra["dw_cols"] = wg.ndim
            if dw > 0:   # the fused kernel's slabs: one per block of its persistent grid
                splits = wg.splits = dw
                L.extra["dw_bytes"] = dw * wg.mdim * 9 * wg.ndim * 4
                L.extra["dw_cols"] = lib.rdn_conv_dgrad_wgrad_cols(C.byref(d), C.byref(wg))
            else:
                ws_need = max(ws_need, lib.rdn_wgrad_workspace_size(C.byref(wg)))
            # dalpha / dbias partials: the fused loaders' per-split rows, else the
            # separate PReLU-backward pass's per-block rows
            L.extra["part_bytes"] = (splits * 2 * wg.mdim * 4 if fused else
                                     lib.rdn_prelu_bwd_workspace_size(self.code, self.P[olvl], L.cout, L.cout_pad))
            L.wgrad_desc = wg
            L.extra["wgrad"] = (splits, wg.mdim, wg.ndim, ndim_real, taps)
            pidx = [self.fp.index[n] for n in (L.name + ".weight", L.name + ".bias", L.act + ".weight")]
            L.extra["pidx"] = pidx
            L.extra["goff"] = [4 * self.fp.offsets[i] for i in pidx]   # byte offsets in a flat gradient buffer
            L.extra["olvl"] = olvl
        self._plan_gate_out()
        self.ws = self._shared("ws", lambda: torch.zeros(max(ws_need // 4, 4), dtype=torch.float32,
                                                          device=self.device))
        # per slot: fused layers' slabs (written from the compute stream while the side
        # stream may still reduce an earlier layer's) and the dalpha/dbias partials
        dwb, pwb = [0] * self.slots, [16] * self.slots
        for L in self.layers:
            sl = L.extra["slot"]
            dwb[sl] = max(dwb[sl], L.extra["dw_bytes"])
            pwb[sl] = max(pwb[sl], L.extra["part_bytes"])
        f32 = dict(dtype=torch.float32, device=self.device)
        self.ws_dw = [self._shared(("ws_dw", i), lambda n=n: torch.zeros((n // 4 + 3) // 4 * 4, **f32)) if n else None
                      for i, n in enumerate(dwb)]
        self.pws = [self._shared(("pws", i), lambda n=n: torch.zeros((n // 4 + 3) // 4 * 4, **f32))
                    for i, n in enumerate(pwb)]
        # the weight-gradient stream's layers (not fused): a ring of SIDE_BATCH slabs in
        # backward order, so SIDE_BATCH consecutive layers' reduces can go in one launch
        self.side_batch = SIDE_BATCH if self.side is not None else 1
        self.ws_side = [self.ws] + [self._shared(("ws_side", i), lambda: torch.zeros(max(ws_need // 4, 4), **f32))
                                    for i in range(1, self.side_batch)]
        k = 0
        for L in reversed(self.layers):
            if not L.extra["dw"]:
                L.extra["side_slab"] = k % self.side_batch
                k += 1
        for L in self.layers:
            L.extra["pws"] = self.pws[L.extra["slot"]].data_ptr()
            L.wgrad_desc.ws = (self.ws_dw[L.extra["slot"]].data_ptr() if L.extra["dw"]
                               else self.ws_side[L.extra["side_slab"]].data_ptr())
            if L.extra["fused"]:
                L.wgrad_desc.part = L.extra["pws"]
        for L in self.layers:   # the finisher's epilogue writes the gated layer's partials
            K = L.extra.get("gates")
            if K is not None:
                L.dgrad_desc.gout_part = K.extra["pws"]
        if self.side is not None:   # per layer: dYpre ready (compute stream) / slot free (side stream)
            for L in self.layers:
                L.extra["ev_ready"] = torch.cuda.Event()
                L.extra["ev_done"] = torch.cuda.Event()
            self.ev_begin = torch.cuda.Event()
            self.ev_end = torch.cuda.Event()

    def _plan_gate_out(self) -> None:
        """Pair every layer that still needs a separate PReLU-backward pass with the
        last consumer of its output in backward order when that consumer's input
        gradient has the layer's output as the tail of its columns (dense conv_k+1
        for slice out_k, Unet_model.py:81-87; up_l.conv for up_l.conv_t's output,
        :43), and let that epilogue write the layer's dYpre and dalpha/dbias
        partials (rdn_conv_desc.gout).  The partials' bytes go into the gated layer's
        ``part_bytes`` (sized into its slot's pws buffer)."""
        if not GATE_OUT:
            return
        lib = H.lib()
        index = {id(L): i for i, L in enumerate(self.layers)}
        for K in self.layers:
            if K.extra["fused"] or K.dst is None or K.kind == "down" or K.cout != K.cout_pad:
                continue
            lo, hi = K.dst.c0, K.dst.c0 + K.cout
            cons = [L for L in self.layers if index[id(L)] > index[id(K)] and L.src.buf == K.dst.buf
                    and L.src.c0 < hi and L.src.c0 + L.cin > lo]
            if not cons:
                continue
            J = min(cons, key=lambda L: index[id(L)])   # last in backward order
            dwj = bool(J.extra["dw"])
            # a residual reader of the slice adds its gradient in its own dgrad epilogue;
            # the fused dgrad+wgrad finisher runs after every such reader in backward
            # order (the next block's conv_3 before its conv_0), the others never do
            resid = [L for L in self.layers if L.resid is not None and L.resid.buf == K.dst.buf and
                     L.resid.c0 < hi and L.resid.c0 + L.resid_c > lo]
            if resid and not (dwj and all(index[id(L)] > index[id(J)] for L in resid)):
                continue
            # (level 0 with a conv3_big / conv3_halo finisher: its 8-byte-per-lane epilogue
            # streamed the extra PReLU input slower than the separate pass -- up_0: +13 us
            # per step; the fused dgrad+wgrad finisher prefetches it with the dX operand)
            if self._out_level(K) == 0 and not dwj:
                continue
            if (J.kind != "c3" or J.extra.get("gates") is not None or J.src.buf in self.pure_inputs
                    or J.cin != J.cin_pad or J.src.c0 + J.cin != hi or J.src.c0 > lo):
                continue
            pre = self.bufs[K.pre]
            d = J.dgrad_desc
            d.gout, d.gout_ps = K.extra["dyp"], K.cout_pad
            d.gout_pre, d.gout_pre_ps = pre.data_ptr(), pre.shape[1]
            d.gout_alpha = self.named[K.act + ".weight"].data_ptr()
            d.gout_part = 4096   # stand-in until the workspace exists (rows probe)
            d.gout_c0 = lo - J.src.c0
            if dwj:   # one partial row per block of the fused kernel's persistent grid
                if K.resid is not None:   # K's own dgrad reads its dY again (residual operand)
                    d.flags |= H.EPI_GOUT_KEEP
                wq = self._probe_copy(J.wgrad_desc, H.WgradDesc, ("a_gate", "a_gate_alpha"))   # (part: stand-in)
                rows = lib.rdn_conv_dgrad_wgrad_gate_rows(C.byref(d), C.byref(wq)) if GATE_OUT_DW else 0
            else:
                rows = lib.rdn_conv_gate_rows(C.byref(d))
            if rows <= 0:
                d.flags &= ~H.EPI_GOUT_KEEP
                d.gout = d.gout_pre = d.gout_alpha = d.gout_part = None
                d.gout_ps = d.gout_pre_ps = d.gout_c0 = 0
                continue
            J.extra["gates"] = K
            K.extra["gated_by"] = J
            K.extra["part_rows"] = rows
            K.extra["part_bytes"] = max(K.extra["part_bytes"], rows * 2 * K.cout * 4)

    @staticmethod
    def _probe_copy(desc, cls, keep):
        """Copy of a descriptor whose per-call pointers (bound at launch time) are
        stand-ins, for the dispatch probe; pointers that select a kernel variant
        (`keep`) stay as they are."""
        d = cls.from_buffer_copy(desc)
        for name, typ in cls._fields_:
            if name not in keep and issubclass(typ, (C.c_void_p, C._Pointer)) and not getattr(d, name):
                setattr(d, name, C.cast(C.c_void_p(4096), typ) if typ is not C.c_void_p else 4096)
        return d

    def _kernel_key(self, desc):
        """Name of the kernel instantiation a conv descriptor launches, as the
        library's own dispatch decides it (rdn_conv_kernel_name)."""
        d = self._probe_copy(desc, H.ConvDesc, _CONV_SELECT)
        buf = C.create_string_buffer(128)
        H.check(H.lib().rdn_conv_kernel_name(C.byref(d), buf, 128), "rdn_conv_kernel_name")
        return buf.value.decode()

    def _wgrad_key(self, wg):
        d = self._probe_copy(wg, H.WgradDesc, ("a_gate", "a_gate_alpha", "part"))
        buf = C.create_string_buffer(128)
        H.check(H.lib().rdn_wgrad_kernel_name(C.byref(d), buf, 128), "rdn_wgrad_kernel_name")
        return buf.value.decode()

    @staticmethod
    def _dense3_key(d3):
        """Kernel instantiation (tile geometry) the fused conv_0..2 launch takes."""
        buf = C.create_string_buffer(128)
        H.check(H.lib().rdn_dense3_kernel_name(C.byref(d3), buf, 128), "rdn_dense3_kernel_name")
        return buf.value.decode()

    def _dw_key(self, d, wg):
        dc = self._probe_copy(d, H.ConvDesc, _CONV_SELECT)
        wc = self._probe_copy(wg, H.WgradDesc, ("a_gate", "a_gate_alpha", "part"))
        buf = C.create_string_buffer(128)
        H.check(H.lib().rdn_conv_dgrad_wgrad_kernel_name(C.byref(dc), C.byref(wc), buf, 128),
                "rdn_conv_dgrad_wgrad_kernel_name")
        return buf.value.decode()

    def _build_info(self):
        """Per launch: kernel instantiation key + algorithmic FLOPs and bytes
        (each operand read once, each output written once)."""
        es = 2 if self.code == H.RDN_BF16 else 4
        for L in self.layers:
            olvl = self._out_level(L)
            Pout, Pin = self.P[olvl], self.P[L.level if L.kind == "up" else (L.level - 1 if L.kind == "down" else L.level)]
            taps = 9 if L.kind == "c3" else 4
            if L.kind == "up":
                macs = self.P[L.level] * 4 * L.cout * L.cin
            else:
                macs = Pout * L.cout * taps * L.cin
            fwd_bytes = es * (Pin * L.cin + Pout * L.cout * (2 if self.train else 1) +
                              (Pout * L.cout if L.resid is not None else 0))
            fkey = self._kernel_key(L.fwd_desc) + (f",splitk{L.extra['splitk']}" if "splitk" in L.extra else "")
            info = {"fwd": ("fwd", L.name, fkey, 2 * macs, fwd_bytes)}
            if "dense3" in L.extra:   # conv_0..2 in one launch: their algorithmic work summed below
                info["dense3"] = None
            if self.train:
                # a fused PReLU backward (gate in the loader) also reads the saved
                # PReLU input of the output slice
                gate = Pout * L.cout if L.extra.get("fused") else 0
                gout = Pin * L.extra["gates"].cout if L.extra.get("gates") is not None else 0
                if L.dgrad_desc.flags & H.EPI_GOUT_KEEP:   # (dY stored beside its dYpre)
                    gout *= 2
                dg_bytes = es * (Pout * L.cout + gate + Pin * L.cin * (2 if L.accum else 1) + gout +
                                 (Pin * L.resid_c if L.resid is not None else 0))
                # (a fused layer's dgrad descriptor is the fused kernel's: no separate key)
                dkey = "conv3_dw_kernel" if L.extra.get("dw") else self._kernel_key(L.dgrad_desc)
                info["dgrad"] = ("dgrad", L.name, dkey, 2 * macs, dg_bytes)
                info["wgrad"] = ("wgrad", L.name, self._wgrad_key(L.wgrad_desc), 2 * macs,
                                 es * (Pout * L.cout + gate + Pin * L.cin))
                if not (L.extra.get("fused") or "gated_by" in L.extra):
                    # the separate PReLU-backward pass: dY + PReLU input read, dYpre written
                    info["prelu"] = ("prelu", L.name, "prelu_bwd_kernel", 0, 3 * es * Pout * L.cout)
                if L.extra.get("dw"):   # one pass: dY + gate + X read once, dX written
                    info["dw"] = ("dwgrad", L.name, self._dw_key(L.dgrad_desc, L.wgrad_desc), 4 * macs,
                                  dg_bytes + es * Pin * L.cin)
            L.extra["info"] = info
        # the fused conv_0..2 launch: the three convs' algorithmic FLOPs and bytes (each
        # conv's input read once, output + PReLU input written once), as unfused
        by_name = {L.name: L for L in self.layers}
        for L in self.layers:
            if "dense3" in L.extra:
                blk = L.name[:-len(".conv_0")]
                parts = [by_name[f"{blk}.conv_{k}"].extra["info"]["fwd"] for k in range(3)]
                # 6th entry: the fused launch's own minimal bytes (x read once, each
                # conv's output and PReLU input written once: 32 + 3 x 32 channels)
                Ls = [by_name[f"{blk}.conv_{k}"] for k in range(3)]
                fused_min = es * self.P[L.level] * (Ls[0].cin + sum(2 * x.cout for x in Ls))
                L.extra["info"]["dense3"] = ("fwd", f"{blk}.conv_0-2", self._dense3_key(L.extra["dense3"]),
                                             sum(p[3] for p in parts), sum(p[4] for p in parts), fused_min)

    # ------------------------------------------------------------------
    def forward(self, xs, t: torch.Tensor | None = None) -> torch.Tensor:
        """``xs``: the Program's NCHW fp32 inputs (contiguous, on the device)."""
        lib, st = H.lib(), H.stream_ptr()
        prog = self.prog
        if len(xs) != len(prog.inputs):
            raise RuntimeError(f"expected {len(prog.inputs)} inputs, got {len(xs)}")
        for (bname, lvl, ch), x in zip(prog.inputs, xs):
            n, h, w = self.grid[lvl]
            if tuple(x.shape) != (n, ch, h, w):
                raise RuntimeError(f"input for {bname}: expected {(n, ch, h, w)}, got {tuple(x.shape)}")
        self.packs.refresh()
        x0 = xs[0]
        if prog.image_input:
            # network image input (+ the broadcast t map as channel cin_img), 8-channel rows
            B, Hh, Ww = self.B, self.H, self.W
            IN, cin = self.bufs["IN"], prog.inputs[0][2]
            if prog.time_input:
                te = t.to(device=x0.device, dtype=torch.float32).expand(B, 1, Hh, Ww)
                rc = lib.rdn_pack_input(self.code, x0.data_ptr(), B, cin, Hh, Ww, te.data_ptr(), te.stride(0),
                                        te.stride(2), te.stride(3), 1, IN.data_ptr(), 8, st)
            else:
                rc = lib.rdn_pack_input(self.code, x0.data_ptr(), B, cin, Hh, Ww, None, 0, 0, 0, 0,
                                        IN.data_ptr(), 8, st)
            H.check(rc, "pack_input")
        else:
            for (bname, lvl, ch), x in zip(prog.inputs, xs):
                ptr, ps, c0, pl = self._slice(Slice(bname))
                n, h, w = self.grid[lvl]
                H.check(lib.rdn_nchw_to_nhwc(self.code, x.data_ptr(), n, ch, h, w, ptr, ps, c0, pl, 0, st),
                        "nchw_to_nhwc")
        n, h, w = self.grid[prog.out_level]
        y = torch.empty(n, prog.out_channels, h, w, dtype=torch.float32, device=x0.device)
        last = self.layers[-1].fwd_desc
        last.out_nchw = y.data_ptr()
        last.res_nchw = x0.data_ptr() if prog.resid_input else None
        fwd = lib.rdn_conv_fwd
        tr = TRACER
        for L in self.layers:
            if "dense3_skip" in L.extra:
                continue
            d3 = L.extra.get("dense3")
            tok = tr.start(L.extra["info"]["dense3" if d3 is not None else "fwd"]) if tr is not None else None
            sk = L.extra.get("splitk")
            if d3 is not None:
                rc = lib.rdn_dense3_fwd(C.byref(d3), st)
            elif sk:
                rc = lib.rdn_conv_fwd_splitk(C.byref(L.fwd_desc), sk, self.ws_fwd.data_ptr(), st)
            else:
                rc = fwd(C.byref(L.fwd_desc), st)
            if tok is not None:
                tr.stop(tok)
            if rc:
                H.check(rc, f"conv_fwd[{L.name}]")
        return y

    def backward(self, dy: torch.Tensor, need_dx):
        """Reverse sweep; returns (input gradients (None where ``need_dx[i]`` is
        false), the flat buffer holding every weight gradient of this pass).

        Compute stream: PReLU backward (unfused layers) and the dgrad chain.  Side
        stream (when enabled): each layer's wgrad + reduce, which only wait for
        that layer's dYpre (event ``ev_ready``); a layer's unfused PReLU backward
        waits for the side stream to release its ring slot (the ``ev_done`` of
        the layer SLOTS earlier in backward order).  Gradient buffers are never
        aliased (one per activation buffer) and a slice's gradient is complete
        before its producer layer is reached, so the two chains share nothing
        else but these slots."""
        if not self.train:
            raise RuntimeError("engine was built without saved activations (no_grad forward)")
        lib, st = H.lib(), H.stream_ptr()
        prog = self.prog
        need_buf = {b: bool(nd) for (b, _, _), nd in zip(prog.inputs, need_dx)}
        gbuf = self.fp.grad_buffer()
        gbuf.zero_()
        gbase = gbuf.data_ptr()
        sync = self.fp.grad_sync
        if sync is not None:
            sync.begin(gbuf)
        dy = dy.contiguous()
        side = None if SERIAL_BWD else self.side
        if side is not None:
            main = torch.cuda.current_stream()
            sst = side.cuda_stream
            self.ev_begin.record(main)
            side.wait_event(self.ev_begin)   # gradient buffer zeroed
        else:
            sst = st
        tr = TRACER
        rev = list(reversed(self.layers))
        pending = []   # fused layers whose split-K reduces wait for one batched launch
        spending = []  # weight-gradient-stream layers whose reduces wait for one batched launch
        batch_side = side is not None and self.side_batch > 1

        def flush_side():
            if not spending:
                return
            jl = [j for _, j in spending]
            H.check(lib.rdn_wgrad_reduce_batch((H.ReduceJob * len(jl))(*jl), len(jl), sst), "wgrad_reduce_batch(side)")
            for Lp, _ in spending:
                Lp.extra["ev_done"].record(side)
                if sync is not None:
                    sync.params_done(Lp.extra["pidx"], stream=side)
            spending.clear()

        def flush():
            if not pending:
                return
            jl = [j for _, js in pending for j in js]
            for i in range(0, len(jl), H.REDUCE_BATCH_MAX):
                n_ = min(H.REDUCE_BATCH_MAX, len(jl) - i)
                H.check(lib.rdn_wgrad_reduce_batch((H.ReduceJob * n_)(*jl[i:i + n_]), n_, st), "wgrad_reduce_batch")
            for Lp, _ in pending:
                if side is not None:
                    Lp.extra["ev_done"].record(main)
                if sync is not None:
                    sync.params_done(Lp.extra["pidx"], stream=None if side is None else main)
            pending.clear()

        def wait_done(Lw):
            """The compute stream waits for layer Lw's weight-gradient work (its slot
            free / an ordering edge); a still-batched layer is flushed first, so its
            event is recorded in this pass before the wait."""
            if any(Lp is Lw for Lp, _ in pending):
                flush()
            if any(Lp is Lw for Lp, _ in spending):
                flush_side()
            main.wait_event(Lw.extra["ev_done"])

        for b, L in enumerate(rev):
            if pending and not L.extra["dw"]:
                flush()
            info = L.extra["info"]
            olvl = L.extra["olvl"]
            n, h, w = self.grid[olvl]
            P = self.P[olvl]
            pre = self.bufs[L.pre]
            fused = L.extra["fused"]
            if side is not None and ORDER_EVERY and b >= ORDER_EVERY and b % ORDER_EVERY == 0 and b < self.slots:
                # ordering edge only (no buffer is reused): see ORDER_EVERY
                wait_done(rev[b - ORDER_EVERY])
            dyp, pws = L.extra["dyp"], L.extra["pws"]
            # unfused: the PReLU-backward pass leaves its dalpha/dbias partials in
            # pws for this layer's rdn_wgrad_reduce to sum (no finalize launch);
            # gated-out: the previous layer's dgrad epilogue already did (below)
            if fused or "gated_by" in L.extra:
                rc = 0
            else:
                if side is not None and b >= self.slots:
                    wait_done(rev[b - self.slots])
                if L.ddst is None:
                    tok = tr.start(info["prelu"]) if tr is not None else None
                    rc = lib.rdn_prelu_bwd(self.code, P, n, h, w, L.cout, L.cout_pad, None, 0, 0, 0, dy.data_ptr(),
                                           pre.data_ptr(), pre.shape[1], self.named[L.act + ".weight"].data_ptr(),
                                           dyp, None, None, pws, st)
                else:
                    dd_ptr, dd_ps, dd_c0, dd_pl = self._slice(L.ddst)
                    tok = tr.start(info["prelu"]) if tr is not None else None
                    rc = lib.rdn_prelu_bwd(self.code, P, n, h, w, L.cout, L.cout_pad, dd_ptr, dd_ps,
                                           dd_c0, dd_pl, None, pre.data_ptr(), pre.shape[1],
                                           self.named[L.act + ".weight"].data_ptr(), dyp, None, None, pws, st)
                if tok is not None:
                    tr.stop(tok)
            if rc:
                H.check(rc, f"prelu_bwd[{L.name}]")
            dw = L.extra["dw"]
            if dw:
                # fused input + weight gradient on the compute stream; its slabs and
                # partials go to this ring slot's buffers, free once the side stream
                # reduced the layer that used the slot before
                if side is not None and b >= self.slots:
                    wait_done(rev[b - self.slots])
                K = L.extra.get("gates")
                if K is not None and side is not None and K.extra["bidx"] >= self.slots:
                    # (gate-out) this epilogue writes K's dYpre / partials into K's ring slot
                    wait_done(rev[K.extra["bidx"] - self.slots])
                tok = tr.start(info["dw"]) if tr is not None else None
                rc = lib.rdn_conv_dgrad_wgrad(C.byref(L.dgrad_desc), C.byref(L.wgrad_desc), st)
                if tok is not None:
                    tr.stop(tok)
                if rc:
                    H.check(rc, f"dgrad_wgrad[{L.name}]")
                if side is not None:
                    L.extra["ev_ready"].record(main)
            else:
                if side is not None:
                    L.extra["ev_ready"].record(main)
                K = L.extra.get("gates")
                if K is not None and side is not None and K.extra["bidx"] >= self.slots:
                    # this epilogue writes K's dYpre / partials into K's ring slot
                    wait_done(rev[K.extra["bidx"] - self.slots])
                if L.src.buf not in self.pure_inputs or need_buf[L.src.buf]:
                    tok = tr.start(info["dgrad"]) if tr is not None else None
                    rc = lib.rdn_conv_fwd(C.byref(L.dgrad_desc), st)
                    if tok is not None:
                        tr.stop(tok)
                    if rc:
                        H.check(rc, f"dgrad[{L.name}]")
            # stream of this layer's reduce: a fused layer's right behind its kernel on
            # the main stream (interleaved step A/B 1652 vs 1636 img/s on the side
            # stream -- at level 0 the side stream has nothing else to overlap)
            rst = sst
            if dw:
                rst = st
            elif side is not None:
                side.wait_event(L.extra["ev_ready"])
            if not dw:
                tok = tr.start(info["wgrad"], side) if tr is not None else None
                rc = lib.rdn_conv_wgrad(C.byref(L.wgrad_desc), sst)
                if tok is not None:
                    tr.stop(tok)
                if rc:
                    H.check(rc, f"wgrad[{L.name}]")
            splits, mdim, ndim, ndim_real, taps = L.extra["wgrad"]
            part_splits = (0 if fused else L.extra["part_rows"] if "gated_by" in L.extra
                           else lib.rdn_prelu_bwd_blocks(self.code, P, L.cout_pad))
            ow, ob, oa = L.extra["goff"]
            cols = L.extra["dw_cols"]
            if dw and REDUCE_BATCH:
                # (a fused layer's reduce joins the batch of consecutive fused layers,
                # one launch on the compute stream: flushed before the next unfused layer)
                jobs = []
                nh = ndim // cols
                sh = splits // nh
                for hh in range(nh):
                    jobs.append(H.ReduceJob(
                        ws=L.wgrad_desc.ws + hh * sh * mdim * taps * cols * 4, grad=gbase + ow,
                        part=pws if hh == 0 else None, dalpha=gbase + oa, dbias=gbase + ob,
                        splits=sh, mdim=mdim, ndim=cols if nh > 1 else ndim, ndim_real=cols if nh > 1 else ndim_real,
                        taps=taps, gstride=ndim_real, gci0=hh * cols, accumulate=1,
                        part_splits=sh if (nh > 1 and fused) else part_splits))
                pending.append((L, jobs))
                continue
            if batch_side and not dw:
                # the weight-gradient stream's reduce joins the batch of consecutive such
                # layers (their slabs are distinct ring entries: side_slab)
                spending.append((L, H.ReduceJob(
                    ws=L.wgrad_desc.ws, grad=gbase + ow, part=pws, dalpha=gbase + oa, dbias=gbase + ob,
                    splits=splits, mdim=mdim, ndim=ndim, ndim_real=ndim_real, taps=taps, gstride=ndim_real,
                    gci0=0, accumulate=1, part_splits=part_splits)))
                if len(spending) >= min(self.side_batch, H.REDUCE_BATCH_MAX):
                    flush_side()
                continue
            if cols < ndim:
                # column halves of the fused kernel: each half's slabs hold its input
                # channels; the dalpha/dbias partials are half 0's rows
                nh, sh = ndim // cols, splits // (ndim // cols)
                for hh in range(nh):
                    rc = lib.rdn_wgrad_reduce_cols(L.wgrad_desc.ws + hh * sh * mdim * taps * cols * 4, sh, mdim, cols,
                                                   taps, gbase + ow, ndim_real, hh * cols, 1,
                                                   pws if hh == 0 else None, sh if fused else part_splits,
                                                   gbase + oa, gbase + ob, rst)
                    if rc:
                        break
            else:
                rc = lib.rdn_wgrad_reduce(L.wgrad_desc.ws, splits, mdim, ndim, ndim_real, taps, gbase + ow, 1, pws,
                                          part_splits, gbase + oa, gbase + ob, rst)
            if rc:
                H.check(rc, f"wgrad_reduce[{L.name}]")
            if side is not None:
                L.extra["ev_done"].record(main if rst == st else side)
            if sync is not None:   # the stream this layer's gradients were completed on
                sync.params_done(L.extra["pidx"], stream=None if side is None else (main if rst == st else side))
        flush()
        flush_side()
        if side is not None:
            self.ev_end.record(side)
            main.wait_event(self.ev_end)
        if sync is not None:
            sync.finish()
        dxs = []
        for i, ((bname, lvl, ch), nd) in enumerate(zip(prog.inputs, need_dx)):
            if not nd:
                dxs.append(None)
                continue
            n, h, w = self.grid[lvl]
            if i == 0 and prog.resid_input:   # the residual's share: d(y)/d(input 0) = 1
                dx, acc = dy.clone(), 1
            else:
                dx, acc = torch.empty(n, ch, h, w, dtype=torch.float32, device=dy.device), 0
            ptr, ps, c0, pl = self._slice(Slice("d" + bname))
            H.check(lib.rdn_nhwc_to_nchw(self.code, ptr, ps, c0, pl, n, ch, h, w, dx.data_ptr(), acc, st),
                    "nhwc_to_nchw")
            dxs.append(dx)
        return dxs, gbuf


class _Lease:
    """Held by one autograd graph while its engine's saved activations are its own."""
    __slots__ = ("__weakref__",)


def _engine_free(eng) -> bool:
    return eng.lease is None or eng.lease() is None


# engines per (shape, dtype) that grad-enabled forwards may hold at once (each holds
# its forward activations and PReLU inputs; the backward scratch is one per pool).
# Past the cap the least recently leased engine is taken over, and backward through
# the graph that held it raises (RDN_MAX_TRAIN_ENGINES; 0 = no cap)
MAX_TRAIN_ENGINES = int(os.environ.get("RDN_MAX_TRAIN_ENGINES", "16"))
_LEASE_SEQ = [0]
_WARNED_POOL: list = []


class _EngineFunction(torch.autograd.Function):
    """One engine forward as one autograd node.  Inputs: the Program's input
    tensors, then every parameter of the module, so ``torch.autograd.grad``,
    ``requires_grad_(False)``, hooks and AccumulateGrad see the weights as the
    reference's graph has them."""

    @staticmethod
    def forward(ctx, engine, lease, t, n_in, *tensors):
        ctx.engine, ctx.lease, ctx.n_in = engine, lease, n_in
        return engine.forward(tensors[:n_in], t)

    @staticmethod
    def backward(ctx, dy):
        eng, n = ctx.engine, ctx.n_in
        if eng.lease is None or eng.lease() is not ctx.lease:
            raise RuntimeError("this graph's saved RDUNet activations were released by an earlier backward "
                               "(use retain_graph=True to backward through it twice)")
        needs = ctx.needs_input_grad
        dxs, gbuf = eng.backward(dy, needs[4:4 + n])
        if not torch._C._autograd._get_current_graph_task_keep_graph():
            eng.lease = None          # activations free for the next forward
        return (None, None, None, None, *dxs, *eng.fp.grad_views(gbuf, needs[4 + n:]))


def _run(module, key_shape, xs, t, params, make_engine):
    need_grad = torch.is_grad_enabled() and (any(x.requires_grad for x in xs) or
                                             any(p.requires_grad for p in params.params))
    key = key_shape + (module.compute_dtype, bool(need_grad))
    pool = module._rdn_engines.setdefault(key, [])
    if not need_grad:
        if not pool:
            pool.append(make_engine(False, None))
        with torch.no_grad():
            return pool[0].forward(xs, t)
    # a graph owns its engine's activations until its backward (or until it is
    # freed): a second forward before that backward gets a second engine, up to
    # MAX_TRAIN_ENGINES per shape; past that the least recently leased engine is
    # taken over and the graph that held it raises if it is ever backwarded
    eng = next((e for e in pool if _engine_free(e)), None)
    if eng is None:
        if MAX_TRAIN_ENGINES <= 0 or len(pool) < MAX_TRAIN_ENGINES:
            eng = make_engine(True, pool[0].scratch if pool else None)
            pool.append(eng)
        else:
            eng = min(pool, key=lambda e: e.lease_seq)
            if not _WARNED_POOL:
                _WARNED_POOL.append(True)
                warnings.warn(f"{type(module).__name__}: {MAX_TRAIN_ENGINES} grad-enabled forwards of one shape are "
                              "alive without a backward; reusing the oldest one's saved activations, so a backward "
                              "through that forward will raise (raise the cap with RDN_MAX_TRAIN_ENGINES, or run "
                              "evaluation under torch.no_grad()).", RuntimeWarning, stacklevel=3)
    lease = _Lease()
    eng.lease = weakref.ref(lease)
    _LEASE_SEQ[0] += 1
    eng.lease_seq = _LEASE_SEQ[0]
    return _EngineFunction.apply(eng, lease, t, len(xs), *xs, *params.params)


def _f32_input(x, what):
    if not isinstance(x, torch.Tensor) or x.dim() != 4:
        raise RuntimeError(f"{what}: expected a [B,C,H,W] tensor")
    return x.contiguous() if x.dtype == torch.float32 else x.float().contiguous()


def run_unet(module, x: torch.Tensor, t: torch.Tensor | None) -> torch.Tensor:
    """Entry used by ``RDUNet_T.forward`` / ``RDUNet.forward``."""
    H.require_device(x, *(p for p in [next(module.parameters())]))
    if t is not None:
        H.require_device(t)
    if x.dim() != 4 or x.size(1) != module.image_channels:
        raise RuntimeError(f"expected input [B,{module.image_channels},H,W], got {tuple(x.shape)}")
    x = _f32_input(x, type(module).__name__)
    fp = flat_params(module, x.device)
    B, Hh, Ww = x.size(0), x.size(2), x.size(3)
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in fp.params))
    if not need_grad and B > 1 and B * Hh * Ww > FWD_CHUNK_PIXELS:
        # a forward-only batch past 2^23 pixels (config 4: 64 x 512^2) runs as chunks of
        # images: its channel-blocked level-0 buffers would otherwise put byte offsets
        # past the 32-bit buffer-descriptor range of the fast conv kernels (conv3_ws /
        # conv3_big / conv3_dense*, which then decline the launch), and the images are
        # independent (no batch statistics), so the result is the same
        bc = max(1, FWD_CHUNK_PIXELS // (Hh * Ww))
        ys = []
        for i in range(0, B, bc):
            tc = t[i:i + bc] if (t is not None and t.dim() > 0 and t.size(0) == B) else t
            ys.append(run_unet(module, x[i:i + bc], tc))
        return torch.cat(ys, 0)
    return _run(module, (B, Hh, Ww), [x], t, fp,
                lambda train, scratch: UNetEngine(module, B, Hh, Ww, module.compute_dtype, train, scratch=scratch))


def run_block(block, xs) -> torch.Tensor:
    """Entry of the blocks' standalone ``forward`` (Unet_model.py:23-89)."""
    xs = [_f32_input(x, type(block).__name__) for x in xs]
    H.require_device(*xs, next(block.parameters()))
    bp = block_params(block, xs[0].device)
    prog = getattr(block, "_rdn_prog", None)
    if prog is None:
        prog = block._rdn_prog = block_program(block)
    lvl0 = prog.inputs[0][1]
    B, Hh, Ww = xs[0].size(0), xs[0].size(2) << lvl0, xs[0].size(3) << lvl0
    return _run(block, (B, Hh, Ww), xs, None, bp,
                lambda train, scratch: UNetEngine(block, B, Hh, Ww, block.compute_dtype, train,
                                                  prog=block_program(block), params=bp, scratch=scratch))
