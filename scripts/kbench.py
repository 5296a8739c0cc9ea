"""Micro-benchmark of single conv launches (the network's real shapes at B=16,
256x256) for one or more builds of librdunet_hip, interleaved in ONE process
(MI355X_MICROARCH / cdna_hip_programming rule 24).

  python scripts/kbench.py [lib1.so lib2.so ...]
"""
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from vub_image_denoising_amd import _hip as H  # noqa: E402


def load(path):
    lib = C.CDLL(path)
    for name, (res, args) in H.SIGNATURES.items():
        fn = getattr(lib, name, None)   # older variant builds may lack newer entry points
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


# (name, N, H, W, buf_in, cin, cout_cols, kind) kind: fwd (bias+prelu+pre) | dgrad (store)
SHAPES = [
    ("L0 conv_0 32->16", 16, 256, 256, 80, 32, 16, "fwd"),
    ("L0 conv_1 48->16", 16, 256, 256, 80, 48, 16, "fwd"),
    ("L0 conv_2 64->16", 16, 256, 256, 80, 64, 16, "fwd"),
    ("L0 conv_3 80->32", 16, 256, 256, 80, 80, 32, "fwd"),
    ("L1 conv_0 64->32", 16, 128, 128, 160, 64, 32, "fwd"),
    ("L1 conv_1 96->32", 16, 128, 128, 160, 96, 32, "fwd"),
    ("L0 dgrad1 16->48", 16, 256, 256, 16, 16, 48, "dgrad"),
    ("L0 dgrad2 16->64", 16, 256, 256, 16, 16, 64, "dgrad"),
    ("L0 up0 dgrad 32->96", 16, 256, 256, 32, 32, 96, "dgrad"),
    ("L1 dgrad0 32->64", 16, 128, 128, 32, 32, 64, "dgrad"),
    ("L0 dgrad3 32->80", 16, 256, 256, 32, 32, 80, "dgrad"),
    ("L1 conv_3 160->64", 16, 128, 128, 160, 160, 64, "fwd"),
    ("L1 dgrad3 64->160", 16, 128, 128, 64, 64, 160, "dgrad"),
    ("L2 conv_0 128->64", 16, 64, 64, 320, 128, 64, "fwd"),
    ("L2 conv_2 256->64", 16, 64, 64, 320, 256, 64, "fwd"),
    ("L2 conv_0 128->64 B32", 32, 64, 64, 320, 128, 64, "fwd"),
    ("L2 conv_3 320->128", 16, 64, 64, 320, 320, 128, "fwd"),
    ("L2 dgrad3 128->320", 16, 64, 64, 128, 128, 320, "dgrad"),
    ("L3 conv_3 640->256", 16, 32, 32, 640, 640, 256, "fwd"),
    ("L3 dgrad3 256->640", 16, 32, 32, 256, 256, 640, "dgrad"),
]


def setup(lib, shp, dt):
    name, N, Hh, Ww, cs, cin, cols, kind = shp
    code = H.dtype_code(dt)
    P = N * Hh * Ww
    x = torch.randn(P, cs, device="cuda").to(dt)
    w = torch.randn(cols, cin, 3, 3, device="cuda") * 0.05
    ck = lib.rdn_conv3_chunk(cin, code)
    kp = lib.rdn_conv3_packed_k(cin, code)
    rows = (cols + 127) // 128 * 128
    wp = torch.zeros(rows, kp, dtype=dt, device="cuda")
    H.check(lib.rdn_pack_weights(H.PACK_CONV_FWD, code, w.data_ptr(), cols, cin, 3, 3, 0, cin, wp.data_ptr(), rows, kp,
                                 ck, torch.cuda.current_stream().cuda_stream))
    b = torch.zeros(cols, device="cuda")
    a = torch.full((cols,), 0.25, device="cuda")
    out = torch.zeros(P, cols, dtype=dt, device="cuda")
    pre = torch.zeros(P, cols, dtype=dt, device="cuda")
    flags = (H.EPI_BIAS | H.EPI_PRELU | H.EPI_STORE_PRE) if kind == "fwd" else 0
    d = H.ConvDesc(dtype=code, gather=H.RDN_G_CONV3, flags=flags, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, cin=cin,
                   x=x.data_ptr(), x_ps=cs, x_c0=0, wp=wp.data_ptr(), kp=kp, ncols=cols, cout=cols,
                   bias=b.data_ptr(), alpha=a.data_ptr(), out=out.data_ptr(), out_ps=cols, out_c0=0,
                   pre=pre.data_ptr(), pre_ps=cols, bn=int(os.environ.get("KB_BN", "0")))
    flops = 2.0 * P * cols * 9 * cin
    es = 2 if dt == torch.bfloat16 else 4
    byts = es * P * (cin + cols * (2 if kind == "fwd" else 1))
    return d, (x, w, wp, b, a, out, pre), flops, byts


# weight gradients: (name, N, H, W, a_ps, mdim, b_ps, ndim)
WSHAPES = [
    ("L0 wgrad conv_0 16x32", 16, 256, 256, 16, 16, 80, 32),
    ("L0 wgrad conv_1 16x48", 16, 256, 256, 16, 16, 80, 48),
    ("L0 wgrad conv_3 32x80", 16, 256, 256, 32, 32, 80, 80),
    ("L0 wgrad up0 32x96", 16, 256, 256, 32, 32, 96, 96),
    ("L1 wgrad conv_0 32x64", 16, 128, 128, 32, 32, 160, 64),
    ("L1 wgrad conv_3 64x160", 16, 128, 128, 64, 64, 160, 160),
    ("L2 wgrad conv_3 128x320", 16, 64, 64, 128, 128, 320, 320),
    ("L3 wgrad conv_3 256x640", 16, 32, 32, 256, 256, 640, 640),
]


def wsetup(lib, shp, dt):
    name, N, Hh, Ww, aps, md, bps, nd = shp
    code = H.dtype_code(dt)
    P = N * Hh * Ww
    a = torch.randn(P, aps, device="cuda").to(dt)
    b = torch.randn(P, bps, device="cuda").to(dt)
    wd = H.WgradDesc(dtype=code, gather=H.RDN_G_CONV3, n=N, h=Hh, w=Ww, hin=Hh, win=Ww, a=a.data_ptr(), a_ps=aps,
                     a_c0=0, mdim=md, b=b.data_ptr(), b_ps=bps, b_c0=0, ndim=nd)
    ns = int(os.environ.get("KB_SPLITS", "0")) or lib.rdn_wgrad_splits(C.byref(wd))
    wd.splits = ns
    ws = torch.zeros(lib.rdn_wgrad_workspace_size(C.byref(wd)) // 4 + 64, device="cuda")
    wd.ws = ws.data_ptr()
    g = torch.zeros(md * nd * 9, device="cuda")
    flops = 2.0 * P * md * 9 * nd
    byts = 2 * P * (md + nd)
    return wd, (a, b, ws, g), flops, byts, ns


def wbench(L, libs, dt, st, reps):
    only = os.environ.get("KB_ONLY", "")
    for shp in WSHAPES:
        if only and only not in shp[0]:
            continue
        setups = [wsetup(lib, shp, dt) for lib in L]
        tw = [[] for _ in L]
        tr = [[] for _ in L]
        for rnd in range(3):
            for i, lib in enumerate(L):
                wd, (a, b, ws, g), _, _, ns = setups[i]
                md, nd = shp[5], shp[7]
                red = lambda: lib.rdn_wgrad_reduce(ws.data_ptr(), ns, md, nd, nd, 9, g.data_ptr(), 0, None, 0, None, None, st)
                for _ in range(2):
                    lib.rdn_conv_wgrad(C.byref(wd), st)
                    red()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                for _ in range(reps):
                    rc = lib.rdn_conv_wgrad(C.byref(wd), st)
                e[1].record()
                for _ in range(reps):
                    rc2 = red()
                e[2].record()
                torch.cuda.synchronize()
                assert rc == 0 and rc2 == 0, lib.rdn_last_error()
                tw[i].append(e[0].elapsed_time(e[1]) / reps)
                tr[i].append(e[1].elapsed_time(e[2]) / reps)
        res = []
        for i in range(len(L)):
            t, r = min(tw[i]), min(tr[i])
            fl, by = setups[i][2], setups[i][3]
            res.append(f"{t * 1e3:6.1f}+{r * 1e3:5.1f}us {fl / t / 1e9:4.0f}TF {by / t / 1e6:5.0f}GB s{setups[i][4]}")
        print(f"{shp[0]:24s} " + " ".join(f"{x:>34s}" for x in res), flush=True)


def main():
    libs = sys.argv[1:] or [H.LIB_PATH]
    L = [load(p) for p in libs]
    dt = torch.bfloat16 if os.environ.get("KB_DT", "bf16") == "bf16" else torch.float32
    st = torch.cuda.current_stream().cuda_stream
    reps = int(os.environ.get("KB_REPS", "20"))
    print(f"{'shape':24s} " + " ".join(f"{os.path.basename(p)[:22]:>24s}" for p in libs))
    if os.environ.get("KB_WGRAD", "1") != "0":
        wbench(L, libs, dt, st, reps)
    only = os.environ.get("KB_ONLY", "")
    if os.environ.get("KB_CONV", "1") == "0":
        return
    for shp in SHAPES:
        if only and only not in shp[0]:
            continue
        res = []
        setups = [setup(lib, shp, dt) for lib in L]
        times = [[] for _ in L]
        for rnd in range(3):
            for i, lib in enumerate(L):
                d = setups[i][0]
                for _ in range(2):
                    lib.rdn_conv_fwd(C.byref(d), st)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    rc = lib.rdn_conv_fwd(C.byref(d), st)
                e.record()
                torch.cuda.synchronize()
                assert rc == 0, lib.rdn_last_error()
                times[i].append(s.elapsed_time(e) / reps)
        for i in range(len(L)):
            t = min(times[i])
            fl, by = setups[i][2], setups[i][3]
            res.append(f"{t * 1e3:7.1f}us {fl / t / 1e9:6.0f}TF {by / t / 1e6:5.0f}GB")
        print(f"{shp[0]:24s} " + " ".join(f"{r:>24s}" for r in res), flush=True)


if __name__ == "__main__":
    main()
