"""3x3 weight-gradient launches (rdn_conv_wgrad, the train step's multi-chunk shapes at
B16 256^2, bf16, plain NHWC operands) timed for several builds of the library,
interleaved in one process -- e.g. the diagnostic builds of wgrad3_glds.hip
(scripts/build_variants.sh with -DWG_DIAG_*) that remove one part of the work.

    python scripts/wg_kbench.py build/variants/lib_base.so build/variants/lib_nomfma.so ...
"""
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from vub_image_denoising_amd import _hip as H  # noqa: E402

# (name, n, h, w, mdim = dY channels, ndim = input channels)
SHAPES = [
    ("L1 conv_1 96->32", 16, 128, 128, 32, 96),
    ("L1 conv_2 128->32", 16, 128, 128, 32, 128),
    ("L1 conv_3 160->64", 16, 128, 128, 64, 160),
    ("L2 conv_0 128->64", 16, 64, 64, 64, 128),
    ("L2 conv_2 256->64", 16, 64, 64, 64, 256),
    ("L2 conv_3 320->128", 16, 64, 64, 128, 320),
    ("L3 conv_3 640->256", 16, 32, 32, 256, 640),
]


def load(path):
    lib = C.CDLL(path)
    for name, (res, args) in H.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:] if p.endswith(".so")]
    out = sys.argv[-1] if sys.argv[-1].endswith(".json") else None
    st = torch.cuda.current_stream().cuda_stream
    rows = []
    for name, n, h, w, m, nd in SHAPES:
        P = n * h * w
        a = (torch.randn(P, m, device="cuda") * 0.1).bfloat16()
        b = (torch.randn(P, nd, device="cuda") * 0.1).bfloat16()
        d = H.WgradDesc(dtype=H.RDN_BF16, gather=H.RDN_G_CONV3, n=n, h=h, w=w, hin=h, win=w,
                        a=a.data_ptr(), a_ps=m, a_c0=0, mdim=m, b=b.data_ptr(), b_ps=nd, b_c0=0, ndim=nd)
        lib0 = libs[0][1]
        ws = torch.zeros(lib0.rdn_wgrad_workspace_size(C.byref(d)) // 4 + 16, device="cuda")
        d.ws = ws.data_ptr()
        flops = 2.0 * P * m * 9 * nd
        r = {"shape": name, "splits": lib0.rdn_wgrad_splits(C.byref(d))}
        buf = C.create_string_buffer(128)
        lib0.rdn_wgrad_kernel_name(C.byref(d), buf, 128)
        r["kernel"] = buf.value.decode()
        for rep in range(3):
            for lname, lib in libs:
                H.check(lib.rdn_conv_wgrad(C.byref(d), st), "wgrad")
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    lib.rdn_conv_wgrad(C.byref(d), st)
                e.record()
                torch.cuda.synchronize()
                us = 1e3 * s.elapsed_time(e) / 20
                r[lname] = min(r.get(lname, 1e9), round(us, 2))
        for lname, _ in libs:
            r[lname + "_tfs"] = round(flops / (r[lname] * 1e-6) / 1e12, 1)
        # the reduced weight gradient of every build against the first one's
        grads = []
        for lname, lib in libs:
            g = torch.zeros(m * nd * 9, device="cuda")
            H.check(lib.rdn_conv_wgrad(C.byref(d), st), "wgrad")
            H.check(lib.rdn_wgrad_reduce(d.ws, lib.rdn_wgrad_splits(C.byref(d)), m, nd, nd, 9, g.data_ptr(), 0, None, 0,
                                         None, None, st), "reduce")
            torch.cuda.synchronize()
            grads.append(g)
        r["bit_identical"] = all(torch.equal(grads[0], g) for g in grads[1:])
        rows.append(r)
        print(json.dumps(r), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
