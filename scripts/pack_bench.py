"""Time the train step's batched weight repack (rdn_pack_weights_batched) of an
RDUNet_T(32) bf16 model: HIP events around 20 forced refreshes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vub_image_denoising_amd as vm  # noqa: E402


def main():
    m = vm.RDUNet_T(base_filters=32).cuda()
    m.set_compute_dtype("bf16")
    with torch.no_grad():
        m(torch.rand(1, 3, 64, 64, device="cuda"), torch.full((1, 1, 1, 1), 0.5, device="cuda"))
    packs = m._rdn_packs[torch.bfloat16]
    for _ in range(3):
        packs.key = None
        packs.refresh()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        packs.key = None
        packs.refresh()
    e.record()
    torch.cuda.synchronize()
    print(json.dumps({"packs": len(packs.items), "us_per_repack": round(1e3 * s.elapsed_time(e) / 20, 2)}))


if __name__ == "__main__":
    main()
