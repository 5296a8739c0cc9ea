"""conv3_big (csrc/conv3_big.hip): the large-tile bf16 3x3 conv of the level-1..3
forward and input-gradient launches, through the C ABI.

Each case runs twice on the same operands: through the default dispatch (which
must pick conv3_big: rdn_conv_kernel_name says so) and through conv3_halo (a
tile override, desc.bn, bypasses conv3_big).  Both run the same MFMA over the same
k sequence on the same bf16 operands, so the outputs must be bit-identical; both
are also held to torch fp32 math on the CPU at the bf16 budget of
test_gpu_kernels.py (2e-2).  Shapes are the network's (Unet_model.py:72-89 dense
convs, :35-43 up convs, their input gradients), at batch sizes that clear
the kernel's grid rule, including channel-blocked ("planar") operands, the
residual / accumulate epilogues and partial edge tiles.
"""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from vub_image_denoising_amd import _hip as H  # noqa: E402

BF = torch.bfloat16


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _pack(w, cout, cin):
    ck = H.lib().rdn_conv3_chunk(cin, H.RDN_BF16)
    kp = H.lib().rdn_conv3_packed_k(cin, H.RDN_BF16)
    rows = (cout + 127) // 128 * 128
    out = torch.zeros(rows, kp, dtype=BF, device="cuda")
    H.check(H.lib().rdn_pack_weights(H.PACK_CONV_FWD, H.RDN_BF16, w.data_ptr(), cout, cin, 3, 3, 0, cin,
                                     out.data_ptr(), rows, kp, ck, H.stream_ptr()), "pack")
    return out


class Operand:
    """An NHWC bf16 operand of P pixels x C channels, plain ([P][C]) or channel-
    blocked in planes of cb channels ([C/cb][P][cb], include/rdunet_hip.h)."""

    def __init__(self, P, C, cb=0, fill=True):
        self.P, self.C, self.cb = P, C, cb
        if cb:
            self.t = torch.randn(C // cb, P, cb, device="cuda").to(BF) if fill else \
                torch.zeros(C // cb, P, cb, dtype=BF, device="cuda")
        else:
            self.t = torch.randn(P, C, device="cuda").to(BF) if fill else torch.zeros(P, C, dtype=BF, device="cuda")

    @property
    def ps(self):
        return self.cb or self.C

    @property
    def pl(self):
        return self.P * self.cb if self.cb else 0

    def nchw(self, N, Hh, Ww, c0, c):
        full = self.t.permute(1, 0, 2).reshape(self.P, self.C) if self.cb else self.t
        return full[:, c0:c0 + c].float().cpu().reshape(N, Hh, Ww, c).permute(0, 3, 1, 2).contiguous()


CASES = [
    # name, N, H, W, cin (K side), x channels, x c0, x planes, ncols, out channels, out c0, out planes,
    # resid (res channels, c0, climit), gate, accum -- shapes the dispatch rule gives to conv3_big
    ("L2_conv3_fwd_resid", 16, 64, 64, 320, 320, 0, 64, 128, 128, 0, 0, (320, 0, 128), False, False),
    ("L3_conv2_dgrad_accum", 16, 32, 32, 128, 128, 0, 0, 512, 512, 0, 128, None, False, True),
    ("L2_up2_dgrad_planar_out", 16, 64, 64, 128, 128, 0, 0, 384, 384, 0, 128, None, False, False),
    ("L2_up_conv_fwd_slice", 16, 64, 64, 384, 384, 0, 0, 128, 320, 0, 64, None, False, False),
    ("L1_up1_dgrad_bn64", 16, 128, 128, 64, 64, 0, 0, 192, 192, 0, 32, None, False, True),
    ("L2_ragged_fwd_resid", 25, 72, 56, 256, 256, 0, 64, 128, 128, 0, 0, (256, 0, 128), False, False),
    ("L3_conv3_fwd_planar_in", 32, 32, 32, 640, 640, 0, 128, 256, 256, 0, 0, (640, 0, 256), False, False),
    ("L1_conv2_dgrad_ck32_accum", 16, 128, 128, 32, 32, 0, 0, 128, 128, 0, 32, None, False, True),
    ("L1_conv3_dgrad_bn80_resid", 16, 128, 128, 64, 64, 0, 0, 160, 160, 0, 32, (160, 0, 64), False, False),
    ("L1_conv1_dgrad_bn96_accum", 16, 128, 128, 32, 32, 0, 0, 96, 96, 0, 32, None, False, True),
    ("L1_conv2_fwd_bn32_planar", 16, 128, 128, 128, 160, 0, 32, 32, 160, 128, 32, None, False, False),
    ("L1_conv0_fwd_bn32_planar", 16, 128, 128, 64, 160, 0, 32, 32, 160, 64, 32, None, False, False),
    # 4-wave blocks, two per CU (",w4": 64-column items on 32-channel chunks): the
    # level-1 conv_3 forward, a ragged grid of it and the level-1 conv_0 input gradient
    ("L1_conv3_fwd_ck32_w4", 16, 128, 128, 160, 160, 0, 32, 64, 64, 0, 0, (160, 0, 64), False, False),
    ("L1_ragged_fwd_ck32_w4", 29, 72, 120, 160, 160, 0, 32, 64, 64, 0, 0, (160, 0, 64), False, False),
    ("L1_conv0_dgrad_ck32_w4", 16, 128, 128, 32, 32, 0, 0, 64, 160, 0, 32, None, False, True),
]
# gated input gradients are not taken by conv3_big (they stay on conv3_halo)
GATED = ("L3_gated_dgrad", 8, 32, 32, 256, 256, 0, 0, 640, 640, 0, 128, None, True, True)


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)
    H.load_library()


def _run(case, force_halo, ops):
    (name, N, Hh, Ww, cin, xc, xc0, xcb, ncols, oc, oc0, ocb, resid, gate, accum) = case
    x, wp, b, a, out0, pre, res, gt, ga = ops
    out = Operand(N * Hh * Ww, oc, ocb, fill=False)
    out.t.copy_(out0.t)
    fwd = _is_fwd(case)
    flags = (H.EPI_BIAS | H.EPI_PRELU | H.EPI_STORE_PRE) if fwd else 0
    if resid:
        flags |= H.EPI_RESID
    if accum:
        flags |= H.EPI_ACCUM
    d = H.ConvDesc(dtype=H.RDN_BF16, gather=H.RDN_G_CONV3, flags=flags, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cin,
                   x=x.t.data_ptr(), x_ps=x.ps, x_c0=xc0, x_pl=x.pl, wp=wp.data_ptr(), kp=wp.shape[1], ncols=ncols,
                   cout=ncols, bias=b.data_ptr(), alpha=a.data_ptr(), out=out.t.data_ptr(), out_ps=out.ps,
                   out_c0=oc0, out_pl=out.pl)
    if fwd:
        d.pre, d.pre_ps = pre.data_ptr(), ncols
    if resid:
        d.res, d.res_ps, d.res_c0, d.res_pl, d.res_climit = res.t.data_ptr(), res.ps, resid[1], res.pl, resid[2]
    if gate:
        d.gate, d.gate_ps, d.gate_alpha, d.gate_pl = gt.t.data_ptr(), gt.ps, ga.data_ptr(), gt.pl
    if force_halo:
        d.bn = H.lib().rdn_conv3_pick_bn(ncols)
    buf = C.create_string_buffer(128)
    H.check(H.lib().rdn_conv_kernel_name(C.byref(d), buf, 128), "name")
    H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()), name)
    torch.cuda.synchronize()
    return out, buf.value.decode()


def _is_fwd(case):
    return "_fwd" in case[0] and not case[13]


@pytest.mark.parametrize("case", CASES + [GATED], ids=[c[0] for c in CASES + [GATED]])
def test_conv3_big_vs_halo_and_torch(case):
    (name, N, Hh, Ww, cin, xc, xc0, xcb, ncols, oc, oc0, ocb, resid, gate, accum) = case
    P = N * Hh * Ww
    x = Operand(P, xc, xcb)
    w = (torch.randn(ncols, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).contiguous()
    wp = _pack(w, ncols, cin)
    b = torch.randn(ncols, device="cuda") * 0.1
    a = torch.rand(ncols, device="cuda") * 0.5
    out0 = Operand(P, oc, ocb)
    pre = torch.zeros(P, ncols, dtype=BF, device="cuda")
    res = Operand(P, resid[0], 0) if resid else None
    gt = Operand(P, cin, 0) if gate else None
    ga = torch.rand(cin, device="cuda") * 0.5 if gate else None
    ops = (x, wp, b, a, out0, pre, res, gt, ga)
    y_big, k_big = _run(case, False, ops)
    pre_big = pre.clone()
    y_halo, k_halo = _run(case, True, ops)
    print(f"{name}: default -> {k_big}; override -> {k_halo}")
    assert k_big.startswith("conv3_halo_kernel" if gate else "conv3_big_kernel"), k_big
    assert (",w4>" in k_big) == name.endswith("_w4"), k_big
    assert k_halo.startswith("conv3_halo_kernel"), k_halo
    # torch fp32 reference on the bf16 operands
    xs = x.nchw(N, Hh, Ww, xc0, cin)
    if gate:
        g = gt.nchw(N, Hh, Ww, 0, cin)
        xs = torch.where(g > 0, xs, ga.cpu().view(1, -1, 1, 1) * xs).to(BF).float()
    wr = w.cpu().to(BF).float()
    fwd = _is_fwd(case)
    core = F.conv2d(xs, wr, b.cpu() if fwd else None, padding=1)
    ref = F.prelu(core, a.cpu()) if fwd else core
    if resid:
        rr = res.nchw(N, Hh, Ww, resid[1], ncols).clone()
        rr[:, resid[2]:] = 0
        ref = ref + rr
    if accum:
        ref = ref + out0.nchw(N, Hh, Ww, oc0, ncols)
    got = y_big.nchw(N, Hh, Ww, oc0, ncols)
    e = _rel(got, ref)
    same = torch.equal(y_big.t, y_halo.t)
    ndiff = (y_big.t != y_halo.t).sum().item()
    print(f"{name}: rel err vs torch {e:.2e}; bit-identical to conv3_halo: {same} ({ndiff} differing)")
    assert e < 2e-2
    if fwd:
        assert _rel(pre_big[:, :ncols].float().cpu().reshape(N, Hh, Ww, ncols).permute(0, 3, 1, 2), core) < 2e-2
    # channels outside [oc0, oc0 + ncols) untouched
    if oc > ncols:
        full0 = out0.nchw(N, Hh, Ww, 0, oc)
        fullb = y_big.nchw(N, Hh, Ww, 0, oc)
        keep = torch.ones(oc, dtype=torch.bool)
        keep[oc0:oc0 + ncols] = False
        assert torch.equal(full0[:, keep], fullb[:, keep])
    assert same, f"{ndiff} elements differ from conv3_halo"
