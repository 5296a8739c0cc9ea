"""Per-layer timing of conv3_big against conv3_halo on the network's own level-1..3
launch descriptors (train step, bf16, B16 and B32), same process, interleaved."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main(batch):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import _hip as H
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = DiffusionModel(vm.RDUNet_T(base_filters=32), timesteps=20).to(dev)
    m.unet.set_compute_dtype("bf16")
    x = torch.rand(batch, 3, 256, 256, device=dev) * 2 - 1
    opt = torch.optim.SGD(m.parameters(), lr=0.0)
    train_step_device(m, x, x + 0.1, opt, 'uniform', 1.0)
    torch.cuda.synchronize()
    eng = m.unet._rdn_engines[(batch, 256, 256, torch.bfloat16, True)][0]
    lib, st = H.lib(), H.stream_ptr()
    rows = []

    def timed(desc, reps=20):
        for _ in range(3):
            H.check(lib.rdn_conv_fwd(C.byref(desc), st))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            H.check(lib.rdn_conv_fwd(C.byref(desc), st))
        e.record()
        torch.cuda.synchronize()
        return 1e3 * s.elapsed_time(e) / reps

    def name(desc):
        b = C.create_string_buffer(128)
        H.check(lib.rdn_conv_kernel_name(C.byref(desc), b, 128))
        return b.value.decode()

    for L in eng.layers:
        for phase, desc in (("fwd", L.fwd_desc), ("dgrad", L.dgrad_desc)):
            if desc is None or L.kind != "c3":
                continue
            k = name(desc)
            if not k.startswith("conv3_big"):
                continue
            flops = L.extra["info"]["fwd"][3]
            d2 = H.ConvDesc.from_buffer_copy(desc)
            d2.bn = lib.rdn_conv3_pick_bn(d2.ncols)
            tb, th = [], []
            for _ in range(2):   # interleaved
                tb.append(timed(desc))
                th.append(timed(d2))
            r = {"layer": L.name, "phase": phase, "big": k, "big_us": round(min(tb), 2), "halo": name(d2),
                 "halo_us": round(min(th), 2), "big_tflops": round(flops / (min(tb) * 1e-6) / 1e12, 1)}
            rows.append(r)
            print(json.dumps(r), flush=True)
    return rows


if __name__ == "__main__":
    out = {b: main(b) for b in (16, 32)}
    json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/big_plans.json", "w"), indent=0)
