"""Per-kernel parity of librdunet_hip on the GPU, through the C ABI, against
torch fp32 math on the CPU (the same aten ops the reference runs).

fp32 mode: rel-L2 <= 1e-4 (exact-fp32 MFMA, different summation order).
bf16 mode: inputs rounded to bf16 on both sides, fp32 accumulation: rel-L2 <= 2e-2.
"""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from vub_image_denoising_amd import _hip as H  # noqa: E402


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _tol(dt):
    return 1e-4 if dt == torch.float32 else 2e-2


def _nchw(buf, N, H_, W_, c0, c):
    return buf[:, c0:c0 + c].float().cpu().reshape(N, H_, W_, c).permute(0, 3, 1, 2).contiguous()


def _pack(mode, w, d0, d1, kh, kw, pad0, pad1, rows, kp, dt):
    """3x3 modes use the chunked K layout of the halo kernel (rdn_conv3_chunk)."""
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


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,Hh,Ww,Cs_in,ci0,cin,cout,Cs_out,co0", [
    (2, 16, 16, 80, 0, 48, 16, 80, 48),   # dense conv_1 of a 32-ch block: channel slice in/out
    (1, 8, 24, 32, 0, 32, 32, 32, 0),
    (2, 16, 16, 80, 0, 80, 32, 112, 80),  # whole-row chunk (bf16 CK=80), conv_3 of level 0
    (1, 10, 20, 96, 0, 96, 32, 128, 96),  # CK=96, ragged tiles
    (2, 8, 8, 160, 0, 160, 64, 160, 96),
    (1, 16, 16, 8, 0, 8, 32, 32, 0),      # input conv (8 padded channels)
    (3, 4, 4, 640, 0, 640, 256, 256, 0),  # deepest conv_3 shape, BN=128 with 2 N tiles
])
def test_conv3x3_fwd_prelu(dt, N, Hh, Ww, Cs_in, ci0, cin, cout, Cs_out, co0):
    P = N * Hh * Ww
    x = torch.randn(P, Cs_in, device="cuda").to(dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).contiguous()
    b = torch.randn(cout, device="cuda") * 0.1
    a = torch.rand(cout, device="cuda") * 0.5
    wp = _pack(H.PACK_CONV_FWD, w, cout, cin, 3, 3, 0, cin, cout, 9 * cin, dt)
    out = torch.zeros(P, Cs_out, dtype=dt, device="cuda")
    pre = torch.zeros(P, cout, dtype=dt, device="cuda")
    d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_CONV3,
                   flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_STORE_PRE, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cin,
                   x=x.data_ptr(), x_ps=Cs_in, x_c0=ci0, wp=wp.data_ptr(), kp=wp.shape[1], ncols=cout, cout=cout,
                   bias=b.data_ptr(), alpha=a.data_ptr(), out=out.data_ptr(), out_ps=Cs_out, out_c0=co0,
                   pre=pre.data_ptr(), pre_ps=cout)
    H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()))
    torch.cuda.synchronize()
    xs = _nchw(x, N, Hh, Ww, ci0, cin)
    wr = w.cpu().to(dt).float() if dt != torch.float32 else w.cpu()
    ref_pre = F.conv2d(xs, wr, b.cpu(), padding=1)
    ref = F.prelu(ref_pre, a.cpu())
    assert _rel(_nchw(pre, N, Hh, Ww, 0, cout), ref_pre) < _tol(dt)
    assert _rel(_nchw(out, N, Hh, Ww, co0, cout), ref) < _tol(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_resid_accum_nchw(dt):
    N, Hh, Ww, cin, cout = 2, 8, 16, 32, 16
    P = N * Hh * Ww
    x = torch.randn(P, cin, device="cuda").to(dt)
    res = torch.randn(P, 48, device="cuda").to(dt)
    w = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    b = torch.randn(cout, device="cuda") * 0.1
    a = torch.rand(cout, device="cuda")
    wp = _pack(H.PACK_CONV_FWD, w, cout, cin, 3, 3, 0, cin, cout, 9 * cin, dt)
    out0 = torch.randn(P, 24, device="cuda").to(dt)
    out = out0.clone()
    d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_CONV3,
                   flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_RESID | H.EPI_ACCUM, n=N, h=Hh, w=Ww, hin=Hh, win=Ww,
                   cin=cin, x=x.data_ptr(), x_ps=cin, x_c0=0, wp=wp.data_ptr(), kp=wp.shape[1], ncols=cout, cout=cout,
                   bias=b.data_ptr(), alpha=a.data_ptr(), out=out.data_ptr(), out_ps=24, out_c0=8,
                   res=res.data_ptr(), res_ps=48, res_c0=8, res_climit=10)
    H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()))
    # NCHW fp32 output with NCHW residual (the output block + inputs)
    y = torch.zeros(N, cout, Hh, Ww, device="cuda")
    rn = torch.randn(N, cout, Hh, Ww, device="cuda")
    d2 = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_CONV3,
                    flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_RESID | H.EPI_OUT_NCHW, n=N, h=Hh, w=Ww, hin=Hh, win=Ww,
                    cin=cin, x=x.data_ptr(), x_ps=cin, x_c0=0, wp=wp.data_ptr(), kp=wp.shape[1], ncols=cout,
                    cout=cout, bias=b.data_ptr(), alpha=a.data_ptr(), out_nchw=y.data_ptr(), res_nchw=rn.data_ptr())
    H.check(H.lib().rdn_conv_fwd(C.byref(d2), H.stream_ptr()))
    torch.cuda.synchronize()
    xs = _nchw(x, N, Hh, Ww, 0, cin)
    wr = w.cpu().to(dt).float()
    core = F.prelu(F.conv2d(xs, wr, b.cpu(), padding=1), a.cpu())
    radd = _nchw(res, N, Hh, Ww, 8, cout).clone()
    radd[:, 10:] = 0
    ref = core + radd + _nchw(out0, N, Hh, Ww, 8, cout)
    assert _rel(_nchw(out, N, Hh, Ww, 8, cout), ref) < _tol(dt)
    assert torch.equal(out[:, :8].cpu(), out0[:, :8].cpu())  # untouched channels
    assert _rel(y, core + rn.cpu()) < _tol(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_down_and_up_fwd(dt):
    N, Hh, Ww, C0, C1 = 2, 16, 16, 32, 64
    P0, P1 = N * Hh * Ww, N * Hh * Ww // 4
    # Conv2d(k2,s2) reading a channel slice of a [P0, 96] concat buffer
    cat = torch.randn(P0, 96, device="cuda").to(dt)
    w = torch.randn(C1, C0, 2, 2, device="cuda") * 0.1
    b = torch.randn(C1, device="cuda") * 0.1
    a = torch.rand(C1, device="cuda")
    wp = _pack(H.PACK_CONV_FWD, w, C1, C0, 2, 2, 0, C0, C1, 4 * C0, dt)
    out = torch.zeros(P1, 160, dtype=dt, device="cuda")
    d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_S2, flags=H.EPI_BIAS | H.EPI_PRELU, n=N, h=Hh // 2,
                   w=Ww // 2, hin=Hh, win=Ww, cin=C0, x=cat.data_ptr(), x_ps=96, x_c0=0, wp=wp.data_ptr(),
                   kp=wp.shape[1], ncols=C1, cout=C1, bias=b.data_ptr(), alpha=a.data_ptr(), out=out.data_ptr(),
                   out_ps=160, out_c0=0)
    H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()))
    # ConvTranspose2d(k2,s2) C1->C1 from a [P1, 64] buffer scattered into cat[:, 32:96]
    u = torch.randn(P1, C1, device="cuda").to(dt)
    wt = torch.randn(C1, C1, 2, 2, device="cuda") * 0.1
    bt = torch.randn(C1, device="cuda") * 0.1
    at = torch.rand(C1, device="cuda")
    wpt = _pack(H.PACK_GEMM_T, wt, C1, C1, 2, 2, C1, 0, 4 * C1, C1, dt)
    cat2 = cat.clone()
    pre = torch.zeros(P0, C1, dtype=dt, device="cuda")
    d2 = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_PIX,
                    flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_SCATTER2 | H.EPI_STORE_PRE, n=N, h=Hh // 2, w=Ww // 2,
                    hin=Hh // 2, win=Ww // 2, cin=C1, x=u.data_ptr(), x_ps=C1, x_c0=0, wp=wpt.data_ptr(),
                    kp=wpt.shape[1], ncols=4 * C1, cout=C1, bias=bt.data_ptr(), alpha=at.data_ptr(),
                    out=cat2.data_ptr(), out_ps=96, out_c0=32, pre=pre.data_ptr(), pre_ps=C1)
    H.check(H.lib().rdn_conv_fwd(C.byref(d2), H.stream_ptr()))
    torch.cuda.synchronize()
    ref = F.prelu(F.conv2d(_nchw(cat, N, Hh, Ww, 0, C0), w.cpu().to(dt).float(), b.cpu(), stride=2), a.cpu())
    assert _rel(_nchw(out, N, Hh // 2, Ww // 2, 0, C1), ref) < _tol(dt)
    ref_pre = F.conv_transpose2d(_nchw(u, N, Hh // 2, Ww // 2, 0, C1), wt.cpu().to(dt).float(), bt.cpu(), stride=2)
    assert _rel(_nchw(pre, N, Hh, Ww, 0, C1), ref_pre) < _tol(dt)
    assert _rel(_nchw(cat2, N, Hh, Ww, 32, C1), F.prelu(ref_pre, at.cpu())) < _tol(dt)
    assert torch.equal(cat2[:, :32].cpu(), cat[:, :32].cpu())


def _wgrad(dt, gather, N, h, w, hin, win, A, a_ps, a_c0, mdim, B, b_ps, b_c0, ndim, ndim_real, taps, splits=0):
    d = H.WgradDesc(dtype=H.dtype_code(dt), gather=gather, n=N, h=h, w=w, hin=hin, win=win, a=A.data_ptr(), a_ps=a_ps,
                    a_c0=a_c0, mdim=mdim, b=B.data_ptr(), b_ps=b_ps, b_c0=b_c0, ndim=ndim, splits=splits)
    lib = H.lib()
    ns = lib.rdn_wgrad_splits(C.byref(d))
    d.splits = ns
    ws = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(d)) // 4, device="cuda")
    d.ws = ws.data_ptr()
    H.check(lib.rdn_conv_wgrad(C.byref(d), H.stream_ptr()))
    g = torch.zeros(mdim * ndim_real * taps, device="cuda")
    H.check(lib.rdn_wgrad_reduce(ws.data_ptr(), ns, mdim, ndim, ndim_real, taps, g.data_ptr(), 0, None, 0, None, None,
                                 H.stream_ptr()))
    torch.cuda.synchronize()
    return g


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,Hh,Ww,cin,Cs,cout,cpad", [
    (2, 16, 16, 48, 80, 16, 16),
    (1, 8, 8, 160, 160, 64, 64),
    (2, 16, 16, 32, 32, 3, 8),      # output conv: 3 real rows, zero-padded dY
    (1, 32, 32, 640, 640, 256, 256),
])
def test_conv3x3_backward(dt, N, Hh, Ww, cin, Cs, cout, cpad):
    """dgrad (as a conv with rotated/transposed packed weights) and wgrad vs autograd."""
    P = N * Hh * Ww
    x = torch.randn(P, Cs, device="cuda").to(dt)
    dyp = torch.zeros(P, cpad, device="cuda")
    dyp[:, :cout] = torch.randn(P, cout, device="cuda")
    dyp = dyp.to(dt)
    w = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    # dgrad -> store into a [P, Cs] buffer
    wpd = _pack(H.PACK_CONV_DGRAD, w, cout, cin, 3, 3, cpad, 0, cin, 9 * cpad, dt)
    dx = torch.zeros(P, Cs, dtype=dt, device="cuda")
    d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_CONV3, flags=0, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cpad,
                   x=dyp.data_ptr(), x_ps=cpad, x_c0=0, wp=wpd.data_ptr(), kp=wpd.shape[1], ncols=cin, cout=cin,
                   out=dx.data_ptr(), out_ps=Cs, out_c0=0)
    H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()))
    g = _wgrad(dt, H.RDN_G_CONV3, N, Hh, Ww, Hh, Ww, dyp, cpad, 0, cout, x, Cs, 0, cin, cin, 9)
    xs = _nchw(x, N, Hh, Ww, 0, cin).requires_grad_(True)
    wr = w.cpu().to(dt).float().requires_grad_(True)
    y = F.conv2d(xs, wr, padding=1)
    y.backward(_nchw(dyp, N, Hh, Ww, 0, cout))
    assert _rel(_nchw(dx, N, Hh, Ww, 0, cin), xs.grad) < _tol(dt)
    assert _rel(g.view(cout, cin, 3, 3), wr.grad) < _tol(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_down_up_backward(dt):
    N, Hh, Ww, C0, C1 = 2, 16, 16, 32, 64
    h, w_ = Hh // 2, Ww // 2
    P0, P1 = N * Hh * Ww, N * h * w_
    lib = H.lib()
    # ---- down: Conv2d(C0->C1, k2 s2) input = cat[:, 0:32] of width 96
    cat = torch.randn(P0, 96, device="cuda").to(dt)
    dy = torch.randn(P1, C1, device="cuda").to(dt)
    w = torch.randn(C1, C0, 2, 2, device="cuda") * 0.1
    wpd = _pack(H.PACK_GEMM_T, w, C1, C0, 2, 2, C1, 0, 4 * C0, C1, dt)
    dcat0 = torch.randn(P0, 96, device="cuda").to(dt)
    dcat = dcat0.clone()
    d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_PIX, flags=H.EPI_SCATTER2 | H.EPI_ACCUM, n=N, h=h, w=w_,
                   hin=h, win=w_, cin=C1, x=dy.data_ptr(), x_ps=C1, x_c0=0, wp=wpd.data_ptr(), kp=wpd.shape[1],
                   ncols=4 * C0, cout=C0, out=dcat.data_ptr(), out_ps=96, out_c0=0)
    H.check(lib.rdn_conv_fwd(C.byref(d), H.stream_ptr()))
    g = _wgrad(dt, H.RDN_G_S2, N, h, w_, Hh, Ww, dy, C1, 0, C1, cat, 96, 0, C0, C0, 4)
    xs = _nchw(cat, N, Hh, Ww, 0, C0).requires_grad_(True)
    wr = w.cpu().to(dt).float().requires_grad_(True)
    F.conv2d(xs, wr, stride=2).backward(_nchw(dy, N, h, w_, 0, C1))
    assert _rel(_nchw(dcat, N, Hh, Ww, 0, C0), xs.grad + _nchw(dcat0, N, Hh, Ww, 0, C0)) < _tol(dt)
    assert _rel(g.view(C1, C0, 2, 2), wr.grad) < _tol(dt)
    # ---- up: ConvTranspose2d(C1->C1, k2 s2); input u [P1, C1], dY hi-res [P0, C1]
    u = torch.randn(P1, C1, device="cuda").to(dt)
    dyh = torch.randn(P0, C1, device="cuda").to(dt)
    wt = torch.randn(C1, C1, 2, 2, device="cuda") * 0.1
    wpu = _pack(H.PACK_CONV_FWD, wt, C1, C1, 2, 2, 0, C1, C1, 4 * C1, dt)
    du = torch.zeros(P1, C1, dtype=dt, device="cuda")
    d = H.ConvDesc(dtype=H.dtype_code(dt), gather=H.RDN_G_S2, flags=0, n=N, h=h, w=w_, hin=Hh, win=Ww, cin=C1,
                   x=dyh.data_ptr(), x_ps=C1, x_c0=0, wp=wpu.data_ptr(), kp=wpu.shape[1], ncols=C1, cout=C1,
                   out=du.data_ptr(), out_ps=C1, out_c0=0)
    H.check(lib.rdn_conv_fwd(C.byref(d), H.stream_ptr()))
    gt = _wgrad(dt, H.RDN_G_S2, N, h, w_, Hh, Ww, u, C1, 0, C1, dyh, C1, 0, C1, C1, 4)
    us = _nchw(u, N, h, w_, 0, C1).requires_grad_(True)
    wtr = wt.cpu().to(dt).float().requires_grad_(True)
    F.conv_transpose2d(us, wtr, stride=2).backward(_nchw(dyh, N, Hh, Ww, 0, C1))
    assert _rel(_nchw(du, N, h, w_, 0, C1), us.grad) < _tol(dt)
    assert _rel(gt.view(C1, C1, 2, 2), wtr.grad) < _tol(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C_,cpad,nchw", [(16, 16, False), (64, 64, False), (3, 8, True)])
def test_prelu_bwd(dt, C_, cpad, nchw):
    N, Hh, Ww = 2, 8, 16
    P = N * Hh * Ww
    pre = torch.randn(P, cpad, device="cuda").to(dt)
    pre[::7, 0] = 0  # exact zeros take the negative branch (aten: mask = x > 0)
    a = torch.rand(C_, device="cuda")
    if nchw:
        dyn = torch.randn(N, C_, Hh, Ww, device="cuda")
        dy_args = (None, 0, 0, dyn.data_ptr())
        dyr = dyn.cpu()
    else:
        dyb = torch.randn(P, 80, device="cuda").to(dt)
        dy_args = (dyb.data_ptr(), 80, 16, None)
        dyr = _nchw(dyb, N, Hh, Ww, 16, C_)
    dyp = torch.full((P, cpad), 7.0, dtype=dt, device="cuda")
    da = torch.full((C_,), 0.5, device="cuda")   # accumulates into existing gradients
    db = torch.full((C_,), -0.25, device="cuda")
    ws = torch.zeros(H.lib().rdn_prelu_bwd_workspace_size(H.dtype_code(dt), P, C_, cpad) // 4, device="cuda")
    H.check(H.lib().rdn_prelu_bwd(H.dtype_code(dt), P, N, Hh, Ww, C_, cpad, *dy_args[:3], 0, dy_args[3], pre.data_ptr(), cpad,
                                  a.data_ptr(), dyp.data_ptr(), da.data_ptr(), db.data_ptr(), ws.data_ptr(),
                                  H.stream_ptr()))
    torch.cuda.synchronize()
    x = _nchw(pre, N, Hh, Ww, 0, C_).requires_grad_(True)
    ar = a.cpu().requires_grad_(True)
    y = F.prelu(x, ar)
    y.backward(dyr)
    assert _rel(_nchw(dyp, N, Hh, Ww, 0, C_), x.grad) < _tol(dt)
    assert torch.all(dyp[:, C_:].float() == 0)
    assert _rel(da - 0.5, ar.grad) < _tol(dt)
    assert _rel(db + 0.25, x.grad.sum((0, 2, 3))) < _tol(dt)


def test_charbonnier_clip_adam_combine():
    lib = H.lib()
    p = torch.randn(2, 3, 16, 16, device="cuda")
    t = torch.randn(2, 3, 16, 16, device="cuda")
    from vub_image_denoising_amd import functional as Fn
    pr = p.clone().requires_grad_(True)
    loss = Fn.combined_loss(pr, t, mse_weight=0.3, charbonnier_weight=0.7)
    loss.backward()
    pc = p.cpu().requires_grad_(True)
    tc = t.cpu()
    ref = 0.3 * torch.mean((pc - tc) ** 2) + 0.7 * torch.mean(torch.sqrt((pc - tc) ** 2 + 1e-6))
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    assert _rel(pr.grad, pc.grad) < 1e-5
    # grad-norm + clip on a flat buffer
    g = torch.randn(10007, device="cuda")
    ws = torch.zeros(lib.rdn_reduce_workspace_size(g.numel()) // 4, device="cuda")
    out = torch.zeros(2, device="cuda")
    pp = torch.nn.Parameter(torch.zeros(10007))
    pp.grad = g.cpu().clone()
    H.check(lib.rdn_sqnorm(g.data_ptr(), g.numel(), 1.0, ws.data_ptr(), out.data_ptr(), H.stream_ptr()))
    H.check(lib.rdn_clip_scale(g.data_ptr(), g.numel(), out[1:].data_ptr(), H.stream_ptr()))
    tot = torch.nn.utils.clip_grad_norm_([pp], 1.0)
    torch.cuda.synchronize()
    assert abs(out[0].item() - tot.item()) < 1e-5 * tot.item()
    assert _rel(g, pp.grad) < 1e-5
    # AdamW step vs torch.optim.AdamW (CPU) for 3 steps
    n = 4096
    p0 = torch.randn(n)
    pg = p0.clone().cuda()
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    pt = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([pt], lr=1e-3, weight_decay=1e-2)
    for step in range(1, 4):
        gr = torch.randn(n)
        pt.grad = gr.clone()
        opt.step()
        gg = gr.cuda()
        H.check(lib.rdn_adam_step(pg.data_ptr(), gg.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8,
                                  1e-2, 1, step, None, 1.0, H.stream_ptr()))
    assert _rel(pg, pt.detach()) < 1e-6
    # sampling combine
    x = torch.randn(4096, device="cuda")
    f1, f2, y = torch.randn(4096, device="cuda"), torch.randn(4096, device="cuda"), torch.randn(4096, device="cuda")
    xr = x.cpu() - ((1 - 0.75) * f1.cpu() + 0.75 * y.cpu()) + ((1 - 0.5) * f2.cpu() + 0.5 * y.cpu())
    Fn.sampling_combine(x, f1, f2, y, 0.75, 0.5)
    assert _rel(x, xr) < 1e-6


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_prelu_gate_matches_separate_pass(dt):
    """dgrad/wgrad with the PReLU-backward gate (dY, saved PReLU input) equal the
    unfused rdn_prelu_bwd -> dYpre -> dgrad/wgrad pipeline; the dalpha/dbias
    partials summed in rdn_wgrad_reduce match rdn_prelu_bwd's."""
    lib = H.lib()
    N, Hh, Ww, cin, Cs, cout, Cd = 2, 16, 32, 48, 80, 16, 80
    P = N * Hh * Ww
    code = H.dtype_code(dt)
    st = H.stream_ptr()
    x = torch.randn(P, Cs, device="cuda").to(dt)            # conv input (dense buffer)
    dyb = torch.randn(P, Cd, device="cuda").to(dt)          # gradient buffer, slice [48, 64)
    pre = torch.randn(P, cout, device="cuda").to(dt)
    pre[::5] = 0
    a = torch.rand(cout, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    wpd = _pack(H.PACK_CONV_DGRAD, w, cout, cin, 3, 3, cout, 0, cin, 9 * cout, dt)
    # unfused
    dyp = torch.zeros(P, cout, dtype=dt, device="cuda")
    da1, db1 = torch.zeros(cout, device="cuda"), torch.zeros(cout, device="cuda")
    pws = torch.zeros(lib.rdn_prelu_bwd_workspace_size(code, P, cout, cout) // 4 + 4096, device="cuda")
    H.check(lib.rdn_prelu_bwd(code, P, N, Hh, Ww, cout, cout, dyb.data_ptr(), Cd, 48, 0, None, pre.data_ptr(), cout,
                              a.data_ptr(), dyp.data_ptr(), da1.data_ptr(), db1.data_ptr(), pws.data_ptr(), st))

    def dgrad(xp, xps, xc0, gate):
        out = torch.zeros(P, Cs, dtype=dt, device="cuda")
        d = H.ConvDesc(dtype=code, gather=H.RDN_G_CONV3, flags=0, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cout, x=xp,
                       x_ps=xps, x_c0=xc0, wp=wpd.data_ptr(), kp=wpd.shape[1], ncols=cin, cout=cin,
                       out=out.data_ptr(), out_ps=Cs, out_c0=0)
        if gate:
            d.gate, d.gate_ps, d.gate_alpha = pre.data_ptr(), cout, a.data_ptr()
        H.check(lib.rdn_conv_fwd(C.byref(d), st))
        return out

    def wgrad(ap, aps, ac0, gate, da, db):
        wd = H.WgradDesc(dtype=code, gather=H.RDN_G_CONV3, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, a=ap, a_ps=aps, a_c0=ac0,
                         mdim=cout, b=x.data_ptr(), b_ps=Cs, b_c0=0, ndim=cin)
        ns = lib.rdn_wgrad_splits(C.byref(wd))
        wd.splits = ns
        ws = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(wd)) // 4, device="cuda")
        part = torch.zeros(ns * 2 * cout, device="cuda")
        wd.ws = ws.data_ptr()
        if gate:
            wd.a_gate, wd.a_gate_ps, wd.a_gate_alpha, wd.part = pre.data_ptr(), cout, a.data_ptr(), part.data_ptr()
        g = torch.zeros(cout * cin * 9, device="cuda")
        H.check(lib.rdn_conv_wgrad(C.byref(wd), st))
        H.check(lib.rdn_wgrad_reduce(ws.data_ptr(), ns, cout, cin, cin, 9, g.data_ptr(), 0,
                                     part.data_ptr() if gate else None, 0, da.data_ptr() if gate else None,
                                     db.data_ptr() if gate else None, st))
        return g

    o1 = dgrad(dyp.data_ptr(), cout, 0, False)
    g1 = wgrad(dyp.data_ptr(), cout, 0, False, None, None)
    da2, db2 = torch.zeros(cout, device="cuda"), torch.zeros(cout, device="cuda")
    o2 = dgrad(dyb.data_ptr(), Cd, 48, True)
    g2 = wgrad(dyb.data_ptr(), Cd, 48, True, da2, db2)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.equal(g1, g2)
    assert _rel(da2, da1) < 1e-5 and _rel(db2, db1) < 1e-5
    # unfused path as the engine runs it: rdn_prelu_bwd leaves its partials, the
    # layer's rdn_wgrad_reduce sums them (part_splits = rdn_prelu_bwd_blocks)
    pws2 = torch.zeros_like(pws)
    H.check(lib.rdn_prelu_bwd(code, P, N, Hh, Ww, cout, cout, dyb.data_ptr(), Cd, 48, 0, None, pre.data_ptr(), cout,
                              a.data_ptr(), dyp.data_ptr(), None, None, pws2.data_ptr(), st))
    nb = lib.rdn_prelu_bwd_blocks(code, P, cout)
    da3, db3 = torch.zeros(cout, device="cuda"), torch.zeros(cout, device="cuda")
    wd = H.WgradDesc(dtype=code, gather=H.RDN_G_CONV3, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, a=dyp.data_ptr(), a_ps=cout,
                     a_c0=0, mdim=cout, b=x.data_ptr(), b_ps=Cs, b_c0=0, ndim=cin)
    ns = lib.rdn_wgrad_splits(C.byref(wd))
    wd.splits = ns
    ws = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(wd)) // 4, device="cuda")
    wd.ws = ws.data_ptr()
    g3 = torch.zeros(cout * cin * 9, device="cuda")
    H.check(lib.rdn_conv_wgrad(C.byref(wd), st))
    H.check(lib.rdn_wgrad_reduce(ws.data_ptr(), ns, cout, cin, cin, 9, g3.data_ptr(), 0, pws2.data_ptr(), nb,
                                 da3.data_ptr(), db3.data_ptr(), st))
    torch.cuda.synchronize()
    assert torch.equal(g3, g1)
    assert _rel(da3, da1) < 1e-5 and _rel(db3, db1) < 1e-5


@pytest.mark.parametrize("cin,cout,Cs_in,gate,accum", [
    (80, 32, 80, False, False),   # level-0 conv_3 (CK=80, BN=32), residual epilogue
    (32, 80, 32, True, True),     # its input gradient: gated dY, accumulate, BN=80 (2 epilogue passes)
    (16, 64, 48, True, False),    # conv_2 dgrad slice of a wider gradient buffer
    (96, 32, 96, False, False),   # up_0.conv (CK=96, one block per CU)
    (8, 32, 8, False, False),     # input conv
])
@pytest.mark.parametrize("full", [False, True])
def test_conv3_ws_matches_halo(cin, cout, Cs_in, gate, accum, full):
    """The weight-stationary persistent kernel (default for bf16 single-chunk,
    <= 96-column layers) against the K-streaming halo kernel (forced with an
    explicit bn) on a multi-tile ragged image: every tile, flag and the gate
    must give bitwise-identical results (same MFMA k order, same epilogue).
    full: whole 8 x 16 tiles, where conv3_ws runs its accumulator epilogue
    (round 5: swapped MFMA operands, stores from the registers)."""
    dt, code, lib, st = torch.bfloat16, H.RDN_BF16, H.lib(), H.stream_ptr()
    N, Hh, Ww = (4, 64, 128) if full else (6, 120, 136)   # 256 / 810 tiles: several per persistent block
    P = N * Hh * Ww
    x = torch.randn(P, Cs_in, device="cuda").to(dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).contiguous()
    b = torch.randn(cout, device="cuda") * 0.1
    a = torch.rand(cout, device="cuda") * 0.5
    ga = torch.rand(cin, device="cuda")
    pre_in = torch.randn(P, cin, device="cuda").to(dt)
    pre_in[::3] = 0
    res = torch.randn(P, cout, device="cuda").to(dt)
    wp = _pack(H.PACK_CONV_FWD, w, cout, cin, 3, 3, 0, cin, cout, 9 * cin, dt)
    init = torch.randn(P, cout, device="cuda").to(dt)
    outs = []
    for bn in (0, 16):
        out, pre = init.clone(), torch.zeros(P, cout, dtype=dt, device="cuda")
        flags = H.EPI_ACCUM if accum else (H.EPI_BIAS | H.EPI_PRELU | H.EPI_STORE_PRE | H.EPI_RESID)
        d = H.ConvDesc(dtype=code, gather=H.RDN_G_CONV3, flags=flags, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cin,
                       x=x.data_ptr(), x_ps=Cs_in, x_c0=Cs_in - cin, wp=wp.data_ptr(), kp=wp.shape[1], ncols=cout,
                       cout=cout, bias=b.data_ptr(), alpha=a.data_ptr(), out=out.data_ptr(), out_ps=cout, out_c0=0,
                       pre=pre.data_ptr(), pre_ps=cout, res=res.data_ptr(), res_ps=cout, res_c0=0, res_climit=cout,
                       bn=bn)
        if gate:
            d.gate, d.gate_ps, d.gate_alpha = pre_in.data_ptr(), cin, ga.data_ptr()
        if bn == 0:
            name = C.create_string_buffer(128)
            H.check(lib.rdn_conv_kernel_name(C.byref(d), name, 128))
            if name.value.decode().startswith("conv3_ws_kernel"):   # (else conv3_wsd: full 96-channel tiles)
                assert name.value.decode().endswith(",ae>") == full, name.value
        H.check(lib.rdn_conv_fwd(C.byref(d), st))
        outs.append((out, pre))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    # and against torch on one image
    xs = _nchw(x, N, Hh, Ww, Cs_in - cin, cin)[:1]
    if gate:
        ps = _nchw(pre_in, N, Hh, Ww, 0, cin)[:1]
        xs = torch.where(ps > 0, xs, ga.cpu().view(1, -1, 1, 1) * xs).to(dt).float()
    ref = F.conv2d(xs, w.cpu().to(dt).float(), None if accum else b.cpu(), padding=1)
    if accum:
        ref = ref + _nchw(init, N, Hh, Ww, 0, cout)[:1]
    else:
        ref = F.prelu(ref, a.cpu()) + _nchw(res, N, Hh, Ww, 0, cout)[:1]
    assert _rel(_nchw(outs[0][0], N, Hh, Ww, 0, cout)[:1], ref) < 2e-2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3_halo_bn_choice_bit_exact(dt):
    """The halo kernel's BN (columns per block; grid-aware choice in pick_bn) only
    changes which block computes a column: outputs are bit-identical for every BN,
    on a level-3-like shape (128 output channels, 8x16 tiles)."""
    N, Hh, Ww, cin, cout = 2, 16, 32, 256, 128
    code = H.dtype_code(dt)
    x = torch.randn(N * Hh * Ww, cin, device="cuda").to(dt)
    w = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    b = torch.randn(cout, device="cuda") * 0.1
    a = torch.full((cout,), 0.25, device="cuda")
    wp = _pack(H.PACK_CONV_FWD, w, cout, cin, 3, 3, 0, cin, cout, 9 * cin, dt)
    outs = []
    for bn in (128, 64, 32):
        out = torch.zeros(N * Hh * Ww, cout, dtype=dt, device="cuda")
        pre = torch.zeros_like(out)
        d = H.ConvDesc(dtype=code, gather=H.RDN_G_CONV3, flags=H.EPI_BIAS | H.EPI_PRELU | H.EPI_STORE_PRE,
                       n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cin, x=x.data_ptr(), x_ps=cin, x_c0=0,
                       wp=wp.data_ptr(), kp=wp.shape[1], ncols=cout, cout=cout, bias=b.data_ptr(),
                       alpha=a.data_ptr(), out=out.data_ptr(), out_ps=cout, out_c0=0, pre=pre.data_ptr(),
                       pre_ps=cout, bn=bn)
        H.check(H.lib().rdn_conv_fwd(C.byref(d), H.stream_ptr()), f"conv bn={bn}")
        torch.cuda.synchronize()
        outs.append((out.clone(), pre.clone()))
    for o, p in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(p, outs[0][1])
    wr = w.cpu().to(dt).float() if dt != torch.float32 else w.cpu()
    ref = F.conv2d(x.float().cpu().reshape(N, Hh, Ww, cin).permute(0, 3, 1, 2), wr, b.cpu(), padding=1)
    got = outs[0][1].float().cpu().reshape(N, Hh, Ww, cout).permute(0, 3, 1, 2)
    assert _rel(got, ref) < _tol(dt)
