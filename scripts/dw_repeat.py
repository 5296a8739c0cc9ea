import sys, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_gpu_dw import _grads, _rel
import vub_image_denoising_amd.engine as E
for fuse in (True, False):
    ref = None
    for rep in range(4):
        y, g, n = _grads(fuse, 2, 256)
        if ref is None:
            ref = g; continue
        diff = {k: _rel(g[k], ref[k]) for k in g if not torch.equal(g[k], ref[k])}
        print("fuse", fuse, "rep", rep, "non-identical tensors:", len(diff), sorted(diff.items(), key=lambda x: -x[1])[:4], flush=True)
