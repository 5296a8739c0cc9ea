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
import weakref
from dataclasses import dataclass, field

import torch

from . import _hip as H

_ALIGN = 64  # elements


def _ru(x, m):
    return (x + m - 1) // m * m


# ----------------------------------------------------------------- parameters
class FlatParams:
    """Flat fp32 storage for a module's parameters (and gradients).

    The module's ``nn.Parameter`` objects keep their identity (optimizers and
    ``state_dict`` see the usual tensors) but their ``.data`` become views of
    ``self.flat``; ``.grad`` become views of ``self.gflat``."""

    def __init__(self, module: torch.nn.Module, device):
        self.params = list(module.parameters())
        self.names = [n for n, _ in module.named_parameters()]
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o = _ru(o + p.numel(), _ALIGN)
        self.numel = o
        self.offsets = offs
        self.flat = torch.zeros(o, dtype=torch.float32, device=device)
        self.gflat = torch.zeros(o, dtype=torch.float32, device=device)
        self.views, self.gviews = [], []
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                v = self.flat[off:off + p.numel()].view_as(p)
                v.copy_(p.data.to(device=device, dtype=torch.float32))
                p.data = v
                self.views.append(v)
                self.gviews.append(self.gflat[off:off + p.numel()].view_as(p))
        self.device = device
        self._ptrs = [v.data_ptr() for v in self.views]
        self._gptrs = [g.data_ptr() for g in self.gviews]
        self.generation = 0
        self.grad_sync = None   # ddp.GradSync attached by data-parallel training
        _FLAT_REGISTRY[:] = [r for r in _FLAT_REGISTRY if r() is not None]
        _FLAT_REGISTRY.append(weakref.ref(self))

    def intact(self) -> bool:
        """Every parameter's storage is still its view of ``flat`` (host-cheap:
        one pointer list compare; runs several times per training step)."""
        f32 = torch.float32
        return [p.data_ptr() for p in self.params] == self._ptrs and all(p.dtype is f32 for p in self.params)

    def version_key(self):
        return (self.generation, sum(p._version for p in self.params))

    def prepare_grads(self):
        """Make every ``p.grad`` (of params that require grad) a view of
        ``gflat`` holding its current accumulated value (0 if it was None)."""
        if all(p.grad is None for p in self.params):
            self.gflat.zero_()   # one memset (the common zero_grad(set_to_none=True) case)
            for p, g in zip(self.params, self.gviews):
                if p.requires_grad:
                    p.grad = g
            return
        for p, g in zip(self.params, self.gviews):
            cur = p.grad
            if cur is None:
                g.zero_()
            elif cur.data_ptr() != g.data_ptr():
                g.copy_(cur)
            if p.requires_grad:
                p.grad = g

    def grads_are_views(self) -> bool:
        grads = [p.grad for p in self.params]
        if any(g is None for g in grads):
            return False
        return [g.data_ptr() for g in grads] == self._gptrs


_FLAT_REGISTRY: list = []

# Optional launch tracer (bench.py): an object with start(info) -> token|None and
# stop(token); info = (phase, layer, kernel key, algorithmic flops, algorithmic bytes).
TRACER = None

# PReLU backward is fused into a layer's dgrad/wgrad loaders when its weight-gradient
# kernel reads the gated operand in at most this many input-channel chunks
FUSE_MAX_CHUNKS = int(os.environ.get("RDN_FUSE_MAX_CHUNKS", "1"))
# weight gradients on a side stream (overlapped with the dgrad chain) and the depth
# of the dYpre ring that decouples the two chains
WGRAD_STREAM = os.environ.get("RDN_WGRAD_STREAM", "1") != "0"
WGRAD_SLOTS = max(2, int(os.environ.get("RDN_WGRAD_SLOTS", "4")))
# bench.py's per-kernel profiling pass serialises the backward (isolated kernel times)
SERIAL_BWD = False
# channel-blocked ("planar") activation buffers: a level-l buffer is [C/cb, P, cb] with
# cb = F_l/2 (one plane per dense-block growth slice), so a conv reading or writing a
# channel slice touches only its planes (include/rdunet_hip.h, *_pl fields)
PLANAR = os.environ.get("RDN_PLANAR", "1") != "0"
# extra elements between two planes (keeps plane starts off power-of-two strides)
PLANE_PAD = int(os.environ.get("RDN_PLANE_PAD", "0"))


def find_flat(params):
    """The FlatParams whose parameter list is exactly ``params`` (same objects,
    same order) with every gradient one of its views, else None."""
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


def _plan(F0: int, cin_img: int, has_t: bool, cout_img: int):
    """Forward-ordered layer list + buffer shapes {name: (level, channels)}."""
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
    return layers, bufs


def _assign_backward(layers):
    """Gradient routing: which slice receives each layer's input gradient and
    whether it is the first (store) or a later (accumulate) contribution, in
    backward (reverse) execution order."""
    written = set()
    # gradient arriving at a layer's output = gradient slice of its dst
    for L in layers:
        L.ddst = None if L.dst is None else Slice("d" + L.dst.buf, L.dst.c0)
    for L in reversed(layers):
        if L.name == "input_block.conv_1":
            L.dsrc = Slice("dIN")
            L.accum = False
            continue
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
class UNetEngine:
    """Buffers and prebuilt launch descriptors for one input shape."""

    def __init__(self, module, B, Hh, Ww, dtype, train: bool):
        if Hh % 8 or Ww % 8:
            raise RuntimeError(f"RDUNet needs H and W divisible by 8 (three 2x down-samplings); got {Hh}x{Ww}")
        F0 = module.base_filters
        if F0 % 16:
            raise RuntimeError(f"base_filters must be a multiple of 16 for the NHWC/MFMA layout; got {F0}")
        self.module = module
        self.B, self.H, self.W = B, Hh, Ww
        self.dtype = dtype
        self.code = H.dtype_code(dtype)
        self.train = train
        self.has_t = module.time_conditioned
        self.cin_img = module.image_channels
        self.cout_img = module.out_channels
        dev = next(module.parameters()).device
        self.device = dev
        self.fp = flat_params(module, dev)
        layers, bufspec = _plan(F0, self.cin_img, self.has_t, self.cout_img)
        _assign_backward(layers)
        self.layers = layers
        self.packs = weight_packs(module, self.fp, layers, dtype)
        self.packs.attach(layers)
        self.P = [B * (Hh >> l) * (Ww >> l) for l in range(4)]
        self.grid = [(B, Hh >> l, Ww >> l) for l in range(4)]
        self.bufs = {}
        self.geo = {}   # buffer name -> (pixel stride ps, plane stride pl); pl = 0: plain NHWC
        F = [F0 << l for l in range(4)]

        def alloc(name, lvl, ch):
            cb = F[lvl] // 2
            if PLANAR and name not in ("IN", "dIN") and not name.startswith("PRE_") and ch % cb == 0 and ch > cb:
                pl = self.P[lvl] * cb + PLANE_PAD
                t = torch.zeros(ch // cb, pl, dtype=dtype, device=dev)
                self.geo[name] = (cb, pl)
            else:
                t = torch.zeros(self.P[lvl], ch, dtype=dtype, device=dev)
                self.geo[name] = (ch, 0)
            self.bufs[name] = t

        for name, (lvl, ch) in bufspec.items():
            if not train and name.startswith("PRE_"):
                continue
            alloc(name, lvl, ch)
        self.named = dict(module.named_parameters())
        self._build_fwd()
        if train:
            for name, (lvl, ch) in bufspec.items():
                if name.startswith("PRE_"):
                    continue
                alloc("d" + name, lvl, ch)
            # weight gradients (wgrad + reduce) run on a side stream, overlapped with
            # the dgrad chain; the per-layer dYpre / PReLU-partial buffers they read
            # form a ring of SLOTS so the dgrad chain can run SLOTS layers ahead
            self.side = torch.cuda.Stream(device=dev) if (dev.type == "cuda" and WGRAD_STREAM) else None
            self.slots = WGRAD_SLOTS if self.side is not None else 1
            self.dyp_elems = max(self.P[self._out_level(L)] * L.cout_pad for L in layers)
            self.dyp = torch.zeros(self.slots, self.dyp_elems, dtype=dtype, device=dev)
            lib = H.lib()
            self.pws_bytes = max(lib.rdn_prelu_bwd_workspace_size(self.code, self.P[self._out_level(L)], L.cout,
                                                                  L.cout_pad) for L in layers)
            self._build_bwd()
        self._build_info()
        self.token = 0

    # ------------------------------------------------------------------
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
                flags |= H.EPI_OUT_NCHW | H.EPI_RESID  # + inputs (Unet_model.py:166)
            else:
                d.out, d.out_ps, d.out_c0, d.out_pl = self._slice(L.dst)
                if L.resid is not None:
                    flags |= H.EPI_RESID
                    d.res, d.res_ps, d.res_c0, d.res_pl = self._slice(L.resid)
                    d.res_climit = L.resid_c
            d.flags = flags
            L.fwd_desc = d

    def _build_bwd(self):
        lib = H.lib()
        ws_need = 0
        part_need = 0
        for b, L in enumerate(reversed(self.layers)):   # backward order -> ring slot
            L.extra["slot"] = b % self.slots
            L.extra["dyp"] = self.dyp[L.extra["slot"]].data_ptr()
        for L in self.layers:
            olvl = self._out_level(L)
            dyp = L.extra["dyp"]
            # 3x3 convs whose output gradient arrives as an NHWC slice run the
            # PReLU backward inside their dgrad / wgrad loaders (gate = saved
            # PReLU input); the output conv (NCHW dy) and the 2x2 convs keep
            # the separate rdn_prelu_bwd pass producing dYpre.
            fused = (L.kind == "c3" and L.ddst is not None) and os.environ.get("RDN_FUSE_PRELU", "1") != "0"
            if fused:  # only when the wgrad re-reads operand A (with the gate) at most FUSE_MAX_CHUNKS times
                n_, h_, w_ = self.grid[L.level]
                probe = H.WgradDesc(dtype=self.code, gather=H.RDN_G_CONV3, n=n_, h=h_, w=w_, hin=h_, win=w_,
                                    mdim=L.cout, ndim=L.cin_pad)
                fused = lib.rdn_wgrad_chunks(C.byref(probe)) <= FUSE_MAX_CHUNKS
            L.extra["fused"] = fused
            pre = self.bufs[L.pre]
            alpha = self.named[L.act + ".weight"]
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
            L.dgrad_desc = d
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
            wg.splits = 0
            splits = lib.rdn_wgrad_splits(C.byref(wg))
            wg.splits = splits
            ws_need = max(ws_need, lib.rdn_wgrad_workspace_size(C.byref(wg)))
            if fused:
                part_need = max(part_need, splits * 2 * wg.mdim * 4)
            L.wgrad_desc = wg
            L.extra["wgrad"] = (splits, wg.mdim, wg.ndim, ndim_real, taps)
            L.extra["grad_w"] = self.fp.gviews[self.fp.names.index(L.name + ".weight")]
            L.extra["grad_b"] = self.fp.gviews[self.fp.names.index(L.name + ".bias")]
            L.extra["grad_a"] = self.fp.gviews[self.fp.names.index(L.act + ".weight")]
            L.extra["olvl"] = olvl
            L.extra["pidx"] = [self.fp.names.index(n) for n in (L.name + ".weight", L.name + ".bias", L.act + ".weight")]
        self.ws = torch.zeros(max(ws_need // 4, 4), dtype=torch.float32, device=self.device)
        pws = max(part_need, self.pws_bytes, 16) // 4
        self.pws = torch.zeros(self.slots, (pws + 3) // 4 * 4, dtype=torch.float32, device=self.device)
        for L in self.layers:
            L.extra["pws"] = self.pws[L.extra["slot"]].data_ptr()
            L.wgrad_desc.ws = self.ws.data_ptr()
            if L.extra["fused"]:
                L.wgrad_desc.part = L.extra["pws"]
        if self.side is not None:   # per layer: dYpre ready (compute stream) / slot free (side stream)
            for L in self.layers:
                L.extra["ev_ready"] = torch.cuda.Event()
                L.extra["ev_done"] = torch.cuda.Event()
            self.ev_begin = torch.cuda.Event()
            self.ev_end = torch.cuda.Event()

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
        d = self._probe_copy(desc, H.ConvDesc, ("gate", "gate_alpha"))
        buf = C.create_string_buffer(128)
        H.check(H.lib().rdn_conv_kernel_name(C.byref(d), buf, 128), "rdn_conv_kernel_name")
        return buf.value.decode()

    def _wgrad_key(self, wg):
        d = self._probe_copy(wg, H.WgradDesc, ("a_gate", "a_gate_alpha", "part"))
        buf = C.create_string_buffer(128)
        H.check(H.lib().rdn_wgrad_kernel_name(C.byref(d), buf, 128), "rdn_wgrad_kernel_name")
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
            info = {"fwd": ("fwd", L.name, self._kernel_key(L.fwd_desc), 2 * macs, fwd_bytes)}
            if self.train:
                # a fused PReLU backward (gate in the loader) also reads the saved
                # PReLU input of the output slice
                gate = Pout * L.cout if L.extra.get("fused") else 0
                dg_bytes = es * (Pout * L.cout + gate + Pin * L.cin * (2 if L.accum else 1) +
                                 (Pin * L.resid_c if L.resid is not None else 0))
                info["dgrad"] = ("dgrad", L.name, self._kernel_key(L.dgrad_desc), 2 * macs, dg_bytes)
                info["wgrad"] = ("wgrad", L.name, self._wgrad_key(L.wgrad_desc), 2 * macs,
                                 es * (Pout * L.cout + gate + Pin * L.cin))
            L.extra["info"] = info

    # ------------------------------------------------------------------
    def forward(self, x: torch.Tensor, t: torch.Tensor | None) -> torch.Tensor:
        lib, st = H.lib(), H.stream_ptr()
        B, Hh, Ww = self.B, self.H, self.W
        self.packs.refresh()
        IN = self.bufs["IN"]
        if self.has_t:
            te = t.to(device=x.device, dtype=torch.float32).expand(B, 1, Hh, Ww)
            H.check(lib.rdn_pack_input(self.code, x.data_ptr(), B, self.cin_img, Hh, Ww, te.data_ptr(),
                                       te.stride(0), te.stride(2), te.stride(3), 1, IN.data_ptr(), 8, st),
                    "pack_input")
        else:
            H.check(lib.rdn_pack_input(self.code, x.data_ptr(), B, self.cin_img, Hh, Ww, None, 0, 0, 0, 0,
                                       IN.data_ptr(), 8, st), "pack_input")
        y = torch.empty(B, self.cout_img, Hh, Ww, dtype=torch.float32, device=x.device)
        last = self.layers[-1].fwd_desc
        last.out_nchw, last.res_nchw = y.data_ptr(), x.data_ptr()
        fwd = lib.rdn_conv_fwd
        tr = TRACER
        for L in self.layers:
            tok = tr.start(L.extra["info"]["fwd"]) if tr is not None else None
            rc = fwd(C.byref(L.fwd_desc), st)
            if tok is not None:
                tr.stop(tok)
            if rc:
                H.check(rc, f"conv_fwd[{L.name}]")
        self.token += 1
        return y

    def backward(self, dy: torch.Tensor, need_dx: bool):
        """Reverse sweep.  Compute stream: PReLU backward (unfused layers) and the
        dgrad chain.  Side stream (when enabled): each layer's wgrad + reduce, which
        only wait for that layer's dYpre (event ``ev_ready``); a layer's unfused
        PReLU backward waits for the side stream to release its ring slot (the
        ``ev_done`` of the layer SLOTS earlier in backward order).  Gradient
        buffers are never aliased (one per activation buffer) and a slice's
        gradient is complete before its producer layer is reached, so the two
        chains share nothing else but these slots."""
        if not self.train:
            raise RuntimeError("engine was built without saved activations (no_grad forward)")
        lib, st = H.lib(), H.stream_ptr()
        self.fp.prepare_grads()
        sync = self.fp.grad_sync
        if sync is not None:
            sync.begin()
        dy = dy.contiguous()
        side = None if SERIAL_BWD else self.side
        if side is not None:
            main = torch.cuda.current_stream()
            sst = side.cuda_stream
            self.ev_begin.record(main)
            side.wait_event(self.ev_begin)   # gradients zeroed / accumulated state ready
        else:
            sst = st
        tr = TRACER
        rev = list(reversed(self.layers))
        for b, L in enumerate(rev):
            info = L.extra["info"]
            olvl = L.extra["olvl"]
            n, h, w = self.grid[olvl]
            P = self.P[olvl]
            pre = self.bufs[L.pre]
            ga, gb = L.extra["grad_a"], L.extra["grad_b"]
            fused = L.extra["fused"]
            dyp, pws = L.extra["dyp"], L.extra["pws"]
            # unfused: the PReLU-backward pass leaves its dalpha/dbias partials in
            # pws for this layer's rdn_wgrad_reduce to sum (no finalize launch)
            if fused:
                rc = 0
            else:
                if side is not None and b >= self.slots:
                    main.wait_event(rev[b - self.slots].extra["ev_done"])
                if L.ddst is None:
                    rc = lib.rdn_prelu_bwd(self.code, P, n, h, w, L.cout, L.cout_pad, None, 0, 0, 0, dy.data_ptr(),
                                           pre.data_ptr(), pre.shape[1], self.named[L.act + ".weight"].data_ptr(),
                                           dyp, None, None, pws, st)
                else:
                    dd_ptr, dd_ps, dd_c0, dd_pl = self._slice(L.ddst)
                    rc = lib.rdn_prelu_bwd(self.code, P, n, h, w, L.cout, L.cout_pad, dd_ptr, dd_ps,
                                           dd_c0, dd_pl, None, pre.data_ptr(), pre.shape[1],
                                           self.named[L.act + ".weight"].data_ptr(), dyp, None, None, pws, st)
            if rc:
                H.check(rc, f"prelu_bwd[{L.name}]")
            if side is not None:
                L.extra["ev_ready"].record(main)
            if L.name != "input_block.conv_1" or need_dx:
                tok = tr.start(info["dgrad"]) if tr is not None else None
                rc = lib.rdn_conv_fwd(C.byref(L.dgrad_desc), st)
                if tok is not None:
                    tr.stop(tok)
                if rc:
                    H.check(rc, f"dgrad[{L.name}]")
            if side is not None:
                side.wait_event(L.extra["ev_ready"])
            tok = tr.start(info["wgrad"], side) if tr is not None else None
            rc = lib.rdn_conv_wgrad(C.byref(L.wgrad_desc), sst)
            if tok is not None:
                tr.stop(tok)
            if rc:
                H.check(rc, f"wgrad[{L.name}]")
            splits, mdim, ndim, ndim_real, taps = L.extra["wgrad"]
            part_splits = 0 if fused else lib.rdn_prelu_bwd_blocks(self.code, P, L.cout_pad)
            rc = lib.rdn_wgrad_reduce(self.ws.data_ptr(), splits, mdim, ndim, ndim_real, taps,
                                      L.extra["grad_w"].data_ptr(), 1, pws, part_splits,
                                      ga.data_ptr(), gb.data_ptr(), sst)
            if rc:
                H.check(rc, f"wgrad_reduce[{L.name}]")
            if side is not None:
                L.extra["ev_done"].record(side)
            if sync is not None:
                sync.params_done(L.extra["pidx"], stream=side)
        if side is not None:
            self.ev_end.record(side)
            main.wait_event(self.ev_end)
        if sync is not None:
            sync.finish()
        if not need_dx:
            return None
        dx = dy.clone()  # global residual: output + inputs (Unet_model.py:166)
        dIN = self.bufs["dIN"]
        H.check(lib.rdn_nhwc_to_nchw(self.code, dIN.data_ptr(), dIN.shape[1], 0, 0, self.B, self.cin_img, self.H, self.W,
                                     dx.data_ptr(), 1, st), "nhwc_to_nchw")
        return dx


class _UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, x, t, anchor):
        y = engine.forward(x, t)
        ctx.engine = engine
        ctx.token = engine.token
        return y

    @staticmethod
    def backward(ctx, dy):
        eng = ctx.engine
        if eng.token != ctx.token:
            raise RuntimeError("RDUNet engine activations were overwritten by a later forward of the same shape "
                               "before this backward ran; call backward before the next forward")
        dx = eng.backward(dy, ctx.needs_input_grad[1])
        return None, dx, None, None


def run_unet(module, x: torch.Tensor, t: torch.Tensor | None) -> torch.Tensor:
    """Entry used by ``RDUNet_T.forward`` / ``RDUNet.forward``."""
    H.require_device(x, *(p for p in [next(module.parameters())]))
    if t is not None:
        H.require_device(t)
    if x.dim() != 4 or x.size(1) != module.image_channels:
        raise RuntimeError(f"expected input [B,{module.image_channels},H,W], got {tuple(x.shape)}")
    x = x.contiguous()
    if x.dtype != torch.float32:
        x = x.float()
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in module.parameters()))
    dtype = module.compute_dtype
    fp = flat_params(module, x.device)
    key = (x.size(0), x.size(2), x.size(3), dtype, bool(need_grad))
    eng = module._rdn_engines.get(key)
    if eng is None:
        eng = UNetEngine(module, x.size(0), x.size(2), x.size(3), dtype, bool(need_grad))
        module._rdn_engines[key] = eng
    if not need_grad:
        with torch.no_grad():
            return eng.forward(x, t)
    anchor = fp.params[0]
    return _UNetFunction.apply(eng, x, t, anchor)
