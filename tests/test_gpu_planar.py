"""Channel-blocked ("planar") operands (include/rdunet_hip.h, *_pl fields): every
kernel that reads or writes an activation slice gives BIT-IDENTICAL results for
the plain NHWC layout [P, C] and the planar layout [C/cb, P, cb] of the same
values -- the layout changes addresses only, never the arithmetic or its order.

Shapes are the network's dense-block slices (Unet_model.py:81-89: conv_k reads
channels [0, C+k*i) of the block buffer and writes [C+k*i, C+(k+1)*i); conv_3
adds the residual [0, C)) at small spatial sizes, in both compute dtypes, on the
bf16 weight-stationary kernel (<= 96 input channels), the halo kernel, the rows
and halo weight-gradient kernels and the 2x2 gather/scatter GEMMs.
"""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

from vub_image_denoising_amd import _hip as H  # noqa: E402


def planar(x, cb):
    """[P, C] -> [C/cb, P, cb] (same values)."""
    P, Cc = x.shape
    return x.view(P, Cc // cb, cb).permute(1, 0, 2).contiguous()


def unplanar(x):
    n, P, cb = x.shape
    return x.permute(1, 0, 2).reshape(P, n * cb)


def geo(t, planar_):
    """(pointer, ps, pl) of a plain [P, C] or planar [n, P, cb] buffer."""
    if planar_:
        return t.data_ptr(), t.shape[2], t.shape[1] * t.shape[2]
    return t.data_ptr(), t.shape[1], 0


def _pack(mode, w, d0, d1, kh, kw, pad0, pad1, rows, kp, dt):
    ck = 0
    if kh == 3 and mode in (H.PACK_CONV_FWD, H.PACK_CONV_DGRAD):
        kside = pad1 if mode == H.PACK_CONV_FWD else pad0
        ck = H.lib().rdn_conv3_chunk(kside, H.dtype_code(dt))
        kp = H.lib().rdn_conv3_packed_k(kside, H.dtype_code(dt))
    rows = (rows + 127) // 128 * 128
    kp = (kp + 63) // 64 * 64
    out = torch.zeros(rows, kp, dtype=dt, device="cuda")
    H.check(H.lib().rdn_pack_weights(mode, H.dtype_code(dt), w.data_ptr(), d0, d1, kh, kw, pad0, pad1, out.data_ptr(),
                                     rows, kp, ck, H.stream_ptr()), "pack")
    return out


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)
    H.load_library()


DTS = [torch.float32, torch.bfloat16]


# (C, k): block width C (cb = C/2), conv_k of the dense block
@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("Cb,k", [(32, 0), (32, 1), (32, 2), (32, 3), (64, 2), (64, 3), (128, 1)])
def test_dense_conv_fwd_planar(dt, Cb, k):
    cb = Cb // 2
    D = Cb + 3 * cb
    N, Hh, Ww = 2, 16, 32
    P = N * Hh * Ww
    cin = Cb + k * cb
    cout = Cb if k == 3 else cb
    buf = torch.randn(P, D, device="cuda").to(dt)
    nxt = torch.randn(P, D, device="cuda").to(dt)       # conv_3 writes the next block's buffer
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).contiguous()
    b = torch.randn(cout, device="cuda") * 0.1
    a = torch.rand(cout, device="cuda") * 0.5
    wp = _pack(H.PACK_CONV_FWD, w, cout, cin, 3, 3, 0, cin, cout, 9 * cin, dt)
    outs = []
    for pl in (False, True):
        x = planar(buf, cb) if pl else buf.clone()
        o = planar(nxt, cb) if pl else nxt.clone()
        pre = torch.zeros(P, cout, dtype=dt, device="cuda")
        d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_CONV3, flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_STORE_PRE,
                       n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cin, wp=wp.data_ptr(), kp=wp.shape[1], ncols=cout,
                       cout=cout, bias=b.data_ptr(), alpha=a.data_ptr(), pre=pre.data_ptr(), pre_ps=cout)
        d.x, d.x_ps, d.x_pl = geo(x, pl)
        if k == 3:   # out_3 + x into the next buffer's channels [0, C)
            d.out, d.out_ps, d.out_pl = geo(o, pl)
            d.res, d.res_ps, d.res_pl = geo(x, pl)
            d.res_climit = Cb
            d.flags |= H.EPI_RESID
            dst = o
        else:        # dense growth slice of the same buffer
            d.out, d.out_ps, d.out_pl = geo(x, pl)
            d.out_c0 = cin
            dst = x
        H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()))
        torch.cuda.synchronize()
        outs.append(((unplanar(dst) if pl else dst).cpu(), pre.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("Cb,k", [(32, 0), (32, 3), (64, 1), (128, 3)])
def test_dense_dgrad_wgrad_planar(dt, Cb, k):
    """Input gradient (gated: PReLU backward fused into the loader, accumulate into
    the gradient slice, + residual gradient for conv_3) and weight gradient (gated
    A slice + fused dalpha/dbias partials) of one dense conv, plain vs planar."""
    cb = Cb // 2
    D = Cb + 3 * cb
    N, Hh, Ww = 2, 16, 32
    P = N * Hh * Ww
    cin = Cb + k * cb
    cout = Cb if k == 3 else cb
    code = H.dtype_code(dt)
    lib = H.lib()
    dB = torch.randn(P, D, device="cuda").to(dt)          # gradient buffer of the block
    dN = torch.randn(P, D, device="cuda").to(dt)          # gradient of the next buffer (conv_3's dst)
    X = torch.randn(P, D, device="cuda").to(dt)
    pre = torch.randn(P, cout, device="cuda").to(dt)
    a = torch.rand(cout, device="cuda")
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).contiguous()
    wpd = _pack(H.PACK_CONV_DGRAD, w, cout, cin, 3, 3, cout, 0, cin, 9 * cout, dt)
    res = []
    for pl in (False, True):
        gB = planar(dB, cb) if pl else dB.clone()
        gN = planar(dN, cb) if pl else dN.clone()
        Xb = planar(X, cb) if pl else X.clone()
        src_g, src_c0 = (gN, 0) if k == 3 else (gB, cin)   # gradient arriving at the conv's output
        d = H.ConvDesc(dtype=code, gather=H.RDN_G_CONV3, flags=H.EPI_ACCUM, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cout,
                       wp=wpd.data_ptr(), kp=wpd.shape[1], ncols=cin, cout=cin)
        d.x, d.x_ps, d.x_pl = geo(src_g, pl)
        d.x_c0 = src_c0
        d.gate, d.gate_ps, d.gate_alpha = pre.data_ptr(), cout, a.data_ptr()
        d.out, d.out_ps, d.out_pl = geo(gB, pl)
        if k == 3:
            d.flags |= H.EPI_RESID
            d.res, d.res_ps, d.res_pl = geo(gN, pl)
            d.res_climit = Cb
        H.check(lib.rdn_conv_fwd(C.byref(d), H.stream_ptr()), "dgrad")
        wd = H.WgradDesc(dtype=code, gather=H.RDN_G_CONV3, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, mdim=cout, ndim=cin)
        wd.a, wd.a_ps, wd.a_pl = geo(src_g, pl)
        wd.a_c0 = src_c0
        wd.b, wd.b_ps, wd.b_pl = geo(Xb, pl)
        splits = lib.rdn_wgrad_splits(C.byref(wd))
        ws = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(wd)) // 4, device="cuda")
        part = torch.zeros(splits * 2 * cout, device="cuda")
        wd.ws, wd.splits = ws.data_ptr(), splits
        wd.a_gate, wd.a_gate_ps, wd.a_gate_alpha, wd.part = pre.data_ptr(), cout, a.data_ptr(), part.data_ptr()
        H.check(lib.rdn_conv_wgrad(C.byref(wd), H.stream_ptr()), "wgrad")
        torch.cuda.synchronize()
        res.append(((unplanar(gB) if pl else gB).cpu(), ws.cpu(), part.cpu()))
    for u, v in zip(res[0], res[1]):
        assert torch.equal(u, v)


@pytest.mark.parametrize("dt", DTS)
def test_down_up_planar(dt):
    """down_l reads the skip half [0, F) of CAT_l; up_l's ConvTranspose2d scatters
    into [F, 3F) of CAT_l; their input and weight gradients, plain vs planar."""
    F0 = 32
    cb = F0 // 2
    N, Hh, Ww = 2, 16, 16
    P0, P1 = N * Hh * Ww, N * Hh * Ww // 4
    code = H.dtype_code(dt)
    lib = H.lib()
    cat = torch.randn(P0, 3 * F0, device="cuda").to(dt)
    low = torch.randn(P1, 2 * F0, device="cuda").to(dt)           # U_{l+1}: 2F channels, cb' = F
    wd_ = torch.randn(2 * F0, F0, 2, 2, device="cuda") * 0.1      # Conv2d(F -> 2F, k2 s2)
    wu = torch.randn(2 * F0, 2 * F0, 2, 2, device="cuda") * 0.1   # ConvTranspose2d(2F -> 2F)
    b1, a1 = torch.randn(2 * F0, device="cuda") * 0.1, torch.rand(2 * F0, device="cuda")
    wpd = _pack(H.PACK_CONV_FWD, wd_, 2 * F0, F0, 2, 2, 0, F0, 2 * F0, 4 * F0, dt)
    wpu = _pack(H.PACK_GEMM_T, wu, 2 * F0, 2 * F0, 2, 2, 2 * F0, 0, 8 * F0, 2 * F0, dt)
    res = []
    for pl in (False, True):
        c = planar(cat, cb) if pl else cat.clone()
        u = planar(low, F0) if pl else low.clone()
        out = torch.zeros(P1, 2 * F0, dtype=dt, device="cuda")
        d = H.ConvDesc(dtype=code, gather=H.RDN_G_S2, flags=H.EPI_BIAS | H.EPI_PRELU, n=N, h=Hh // 2, w=Ww // 2,
                       hin=Hh, win=Ww, cin=F0, wp=wpd.data_ptr(), kp=wpd.shape[1], ncols=2 * F0, cout=2 * F0,
                       bias=b1.data_ptr(), alpha=a1.data_ptr(), out=out.data_ptr(), out_ps=2 * F0)
        d.x, d.x_ps, d.x_pl = geo(c, pl)
        H.check(lib.rdn_conv_fwd(C.byref(d), H.stream_ptr()), "down")
        d2 = H.ConvDesc(dtype=code, gather=H.RDN_G_PIX, flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_SCATTER2, n=N,
                        h=Hh // 2, w=Ww // 2, hin=Hh // 2, win=Ww // 2, cin=2 * F0, wp=wpu.data_ptr(),
                        kp=wpu.shape[1], ncols=8 * F0, cout=2 * F0, bias=b1.data_ptr(), alpha=a1.data_ptr())
        d2.x, d2.x_ps, d2.x_pl = geo(u, pl)
        d2.out, d2.out_ps, d2.out_pl = geo(c, pl)
        d2.out_c0 = F0
        H.check(lib.rdn_conv_fwd(C.byref(d2), H.stream_ptr()), "up")
        # weight gradients: down (B = CAT skip slice, gathered s2) and up (A = U buffer)
        dyp = torch.randn(P1, 2 * F0, device="cuda", generator=torch.Generator("cuda").manual_seed(3)).to(dt)
        w1 = H.WgradDesc(dtype=code, gather=H.RDN_G_S2, n=N, h=Hh // 2, w=Ww // 2, hin=Hh, win=Ww, a=dyp.data_ptr(),
                         a_ps=2 * F0, mdim=2 * F0, ndim=F0)
        w1.b, w1.b_ps, w1.b_pl = geo(c, pl)
        ws1 = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(w1)) // 4, device="cuda")
        w1.ws, w1.splits = ws1.data_ptr(), lib.rdn_wgrad_splits(C.byref(w1))
        H.check(lib.rdn_conv_wgrad(C.byref(w1), H.stream_ptr()), "wgrad down")
        dyh = torch.randn(P0, 2 * F0, device="cuda", generator=torch.Generator("cuda").manual_seed(4)).to(dt)
        w2 = H.WgradDesc(dtype=code, gather=H.RDN_G_S2, n=N, h=Hh // 2, w=Ww // 2, hin=Hh, win=Ww, mdim=2 * F0,
                         b=dyh.data_ptr(), b_ps=2 * F0, ndim=2 * F0)
        w2.a, w2.a_ps, w2.a_pl = geo(u, pl)
        ws2 = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(w2)) // 4, device="cuda")
        w2.ws, w2.splits = ws2.data_ptr(), lib.rdn_wgrad_splits(C.byref(w2))
        H.check(lib.rdn_conv_wgrad(C.byref(w2), H.stream_ptr()), "wgrad up")
        torch.cuda.synchronize()
        res.append((out.cpu(), (unplanar(c) if pl else c).cpu(), ws1.cpu(), ws2.cpu()))
    for u_, v_ in zip(res[0], res[1]):
        assert torch.equal(u_, v_)


@pytest.mark.parametrize("dt", DTS)
def test_prelu_bwd_and_converters_planar(dt):
    N, Hh, Ww, Cc, cb = 2, 8, 16, 80, 16
    P = N * Hh * Ww
    code = H.dtype_code(dt)
    lib = H.lib()
    dy = torch.randn(P, Cc, device="cuda").to(dt)
    pre = torch.randn(P, 16, device="cuda").to(dt)
    a = torch.rand(16, device="cuda")
    img = torch.randn(N, 48, Hh, Ww, device="cuda")
    res = []
    for pl in (False, True):
        g = planar(dy, cb) if pl else dy.clone()
        gp, ps, pls = geo(g, pl)
        dyp = torch.zeros(P, 16, dtype=dt, device="cuda")
        ws = torch.zeros(lib.rdn_prelu_bwd_workspace_size(code, P, 16, 16) // 4, device="cuda")
        da, db = torch.zeros(16, device="cuda"), torch.zeros(16, device="cuda")
        H.check(lib.rdn_prelu_bwd(code, P, N, Hh, Ww, 16, 16, gp, ps, 48, pls, None, pre.data_ptr(), 16, a.data_ptr(),
                                  dyp.data_ptr(), da.data_ptr(), db.data_ptr(), ws.data_ptr(), H.stream_ptr()))
        # NCHW fp32 -> channels [32, 80) of the buffer (accumulating), and back
        H.check(lib.rdn_nchw_to_nhwc(code, img.data_ptr(), N, 48, Hh, Ww, gp, ps, 32, pls, 1, H.stream_ptr()))
        back = torch.zeros(N, 48, Hh, Ww, device="cuda")
        H.check(lib.rdn_nhwc_to_nchw(code, gp, ps, 32, pls, N, 48, Hh, Ww, back.data_ptr(), 0, H.stream_ptr()))
        torch.cuda.synchronize()
        res.append((dyp.cpu(), da.cpu(), db.cpu(), (unplanar(g) if pl else g).cpu(), back.cpu()))
    for u, v in zip(res[0], res[1]):
        assert torch.equal(u, v)
    # the accumulate path really added the image
    ref = dy[:, 32:].float().cpu() + img.cpu().permute(0, 2, 3, 1).reshape(P, 48)
    assert torch.allclose(res[0][3][:, 32:].float(), ref.to(dt).float(), atol=0, rtol=0) or dt == torch.bfloat16
