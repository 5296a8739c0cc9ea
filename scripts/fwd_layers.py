"""Per-launch times of a forward-only pass (engine.TRACER events, eager): config 1's
RDUNet(64) on 1 x 3 x 64^2 fp32 by default, or RDUNet_T / other shapes.

  python scripts/fwd_layers.py [rdunet64|rdunet128|t32] [n] [size] [fp32|bf16] [out.json]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import engine as E
    a = sys.argv[1:]
    which = a[0] if a else "rdunet64"
    n = int(a[1]) if len(a) > 1 else 1
    size = int(a[2]) if len(a) > 2 else 64
    dt = a[3] if len(a) > 3 else "fp32"
    torch.manual_seed(0)
    if which == "t32":
        m = vm.RDUNet_T(base_filters=32)
    else:
        m = vm.RDUNet(channels=3, base_filters=64 if which == "rdunet64" else 128)
    m = m.cuda().eval()
    m.set_compute_dtype(dt)
    x = torch.randn(n, 3, size, size, device="cuda")
    args = (x, torch.rand(n, 1, 1, 1, device="cuda")) if which == "t32" else (x,)
    with torch.no_grad():
        for _ in range(3):
            m(*args)
        torch.cuda.synchronize()
        tr = bench.EventTracer()
        E.TRACER = tr
        m(*args)
        E.TRACER = None
        rows = sorted(tr.per_layer(), key=lambda r: -r["us"])
    tot = sum(r["us"] for r in rows)
    print(json.dumps({"model": which, "n": n, "size": size, "dtype": dt, "sum_us": round(tot, 1), "launches": len(rows)}))
    for r in rows:
        print(json.dumps(r))
    if len(a) > 4:
        json.dump(rows, open(a[4], "w"), indent=0)


if __name__ == "__main__":
    main()
