"""Fused level-0 dgrad + wgrad launches (rdn_conv_dgrad_wgrad, conv3_dw.hip) of the
train step (B16 256^2 bf16, the network's own descriptors) timed for several builds
of the library, interleaved in one process -- e.g. the diagnostic builds of
conv3_dw.hip (scripts/build_variants.sh with -DDW_DIAG_*) that remove one part of the
work, or a tuning variant.

    python scripts/dw_kbench.py build/variants/lib_a.so build/variants/lib_b.so ... [out.json]

DW_SHAPE=<substring of the kernel name> keeps one shape, DW_NOTREE=1 drops the in-tree
library (for PMC passes, where same-named kernels of two libraries cannot be told apart).
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def load(path):
    from vub_image_denoising_amd import _hip as H
    lib = C.CDLL(path)
    for name, (res, args) in H.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def main():
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import _hip as H
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
    paths = [p for p in sys.argv[1:] if p.endswith(".so")]
    out = sys.argv[-1] if sys.argv[-1].endswith(".json") else None
    res_out = out
    libs = [] if os.environ.get("DW_NOTREE") else [("tree", H.lib())]
    libs += [(os.path.basename(p)[:-3], load(p)) for p in paths]
    shape = os.environ.get("DW_SHAPE", "")   # kernel-name filter (e.g. "80,32")
    batch = int(os.environ.get("DW_BATCH", "16"))
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = DiffusionModel(vm.RDUNet_T(base_filters=32), timesteps=20).to(dev)
    m.unet.set_compute_dtype("bf16")
    x = torch.rand(batch, 3, 256, 256, device=dev) * 2 - 1
    opt = torch.optim.SGD(m.parameters(), lr=0.0)
    train_step_device(m, x, x + 0.1, opt, 'uniform', 1.0)
    torch.cuda.synchronize()
    eng = m.unet._rdn_engines[(batch, 256, 256, torch.bfloat16, True)][0]
    st = H.stream_ptr()
    rows, seen = [], set()
    for L in eng.layers:
        if not L.extra.get("dw"):
            continue
        k = L.extra["info"]["dw"][2]
        if k in seen or shape not in k:
            continue
        seen.add(k)
        r = {"layer": L.name, "kernel": k}
        for rep in range(3):
            for lname, lib in libs:
                for _ in range(2):
                    H.check(lib.rdn_conv_dgrad_wgrad(C.byref(L.dgrad_desc), C.byref(L.wgrad_desc), st), lname)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    lib.rdn_conv_dgrad_wgrad(C.byref(L.dgrad_desc), C.byref(L.wgrad_desc), st)
                e.record()
                torch.cuda.synchronize()
                us = 1e3 * s.elapsed_time(e) / 20
                r[lname] = min(r.get(lname, 1e9), round(us, 2))
                if hasattr(lib, "rdn_dw_stamps") and rep == 2:   # (-DDW_STAMPS build: phase cycles per tile)
                    import numpy as np
                    n = 512 * 8 * 8
                    buf = np.zeros(n, dtype=np.uint64)
                    lib.rdn_dw_stamps.restype = C.c_int
                    lib.rdn_dw_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), n)
                    a = buf.reshape(512, 8, 8).astype(np.float64)
                    nb = int((a[:, :, 6] > 0).any(axis=1).sum())
                    out = {}
                    for role, ws in (("D", slice(0, 4)), ("W", slice(4, 8))):
                        blk = a[:nb, ws, :]
                        tiles = blk[:, :, 6].sum()
                        out[role] = [round(float(blk[:, :, q].sum() / max(tiles, 1)), 1) for q in range(5)]
                    r[lname + "_phases"] = out   # cycles per tile: gate/store, load issue, MFMA, epilogue, barrier
        rows.append(r)
        print(json.dumps(r), flush=True)
    if res_out:
        with open(res_out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
