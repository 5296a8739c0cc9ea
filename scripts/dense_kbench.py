"""The fused level-0 forward (rdn_dense3_fwd, conv3_dense.hip) of the train step's
level-0 DenoisingBlock descriptors, timed for several builds of the library in one
process (e.g. its -DDN_DIAG_* diagnostic builds, which remove one part of the work).

    python scripts/dense_kbench.py build/variants/lib_a.so ... [B] [l1]

(l1: the level-1 launch, conv3_dense1.hip, and its -DDN1_DIAG_* builds)
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import _hip as H
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
    paths = [p for p in sys.argv[1:] if p.endswith(".so")]
    batch = int(next((a for a in sys.argv[1:] if a.isdigit()), "16"))
    libs = [("tree", H.lib())]
    for p in paths:
        lib = C.CDLL(p)
        for name, (res, args) in H.SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is not None:
                fn.restype, fn.argtypes = res, args
        libs.append((os.path.basename(p)[:-3], lib))
    torch.manual_seed(0)
    m = DiffusionModel(vm.RDUNet_T(base_filters=32), timesteps=20).cuda()
    m.unet.set_compute_dtype("bf16")
    x = torch.rand(batch, 3, 256, 256, device="cuda") * 2 - 1
    opt = torch.optim.SGD(m.parameters(), lr=0.0)
    train_step_device(m, x, x + 0.1, opt, "uniform", 1.0)
    torch.cuda.synchronize()
    eng = m.unet._rdn_engines[(batch, 256, 256, torch.bfloat16, True)][0]
    lvl = 1 if "l1" in sys.argv[1:] else 0
    desc = next((L.extra["dense3"] for L in eng.layers if "dense3" in L.extra and L.level == lvl), None)
    if desc is None:
        raise SystemExit("no dense3 descriptor on the engine")
    st = H.stream_ptr()
    res = {}
    for rep in range(3):
        for name, lib in libs:
            for _ in range(2):
                H.check(lib.rdn_dense3_fwd(C.byref(desc), st), name)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                lib.rdn_dense3_fwd(C.byref(desc), st)
            e.record()
            torch.cuda.synchronize()
            us = 1e3 * s.elapsed_time(e) / 20
            res[name] = min(res.get(name, 1e9), round(us, 2))
    print(json.dumps({"batch": batch, "level": lvl, **res}))


if __name__ == "__main__":
    main()
