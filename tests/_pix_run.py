"""Child of tests/test_gpu_pix.py: one bf16 RDUNet_T forward + backward (the 2x2
convs' forward and input-gradient launches) under the RDN_PIX setting of its
environment; saves the output, every parameter gradient and the input gradient."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out, B, Hh, Ww):
    import vub_image_denoising_amd as vm
    torch.manual_seed(0)
    m = vm.RDUNet_T(base_filters=32).cuda()
    m.set_compute_dtype("bf16")
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(B, 3, Hh, Ww, generator=g) * 2 - 1).cuda().requires_grad_(True)
    t = torch.rand(B, 1, 1, 1, generator=g).cuda()
    w = torch.randn(B, 3, Hh, Ww, generator=g).cuda()
    y = m(x, t)
    (y * w).mean().backward()
    eng = [e for pool in m._rdn_engines.values() for e in pool if e.train][0]
    keys = sorted({v[2] for L in eng.layers for k, v in L.extra["info"].items() if isinstance(v, tuple)})
    res = {"y": y.detach().float().cpu().numpy(), "dx": x.grad.float().cpu().numpy()}
    res.update({"g_" + n: p.grad.float().cpu().numpy() for n, p in m.named_parameters()})
    np.savez(out, keys=np.array(keys), **res)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
