"""Config 5's mixed patch stream (BASELINE.json configs[4]: real-noise training at
patch sizes 128 and 256; the reference's SIDD loader hard-codes 256,
dataset_creation/SIDD_dataset.py:56,63-66): ONE RDUNet_T(32) trained on batches that
alternate 128x128 and 256x256, produced by the GPU loaders (synth.load_data_gpu with
patch_size=(128, 256) -> MixedPatchLoader over two PatchPools) and run through
train_graph.TrainStepGraphs (one captured step per shape, sharing the parameters,
gradient buffer and Adam state).

Each step is checked against the CPU oracle's train step (oracle/rdunet_ref.py
train_step, diffusion_RDUnet.py:76-115) at that step's shape, from the GPU's
parameters just before it: fp32 loss <= 1e-6 relative, every clipped gradient tensor
<= 1e-3 rel-L2 (the budget of test_gpu_fullsize.py: two fp32 rounding paths, each up
to 6e-4 from fp64 per tensor) -- or, on a step where a tensor exceeds
that, every tensor <= 2e-3 against the fp64 oracle (below) --, the flat gradient <= 3e-4 (at batch 2
the gradient averages 2 images, not 16: measured 1e-5..1e-4).  The
AdamW update applied inside the replay is checked against torch.optim.AdamW's update
of the same parameters with the same (GPU) gradient (<= 1e-5 relative on the deltas),
so the Adam state carried across the two captured graphs is checked too."""
import itertools
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import rdunet_ref as R  # noqa: E402
from oracle.weights import make_params  # noqa: E402


def _images(n=2, h=384, w=512, seed=3):
    """Smooth procedural RGB textures (uint8 HWC)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    out = []
    for _ in range(n):
        img = np.zeros((h, w, 3))
        for c in range(3):
            for _ in range(4):
                fy, fx, ph = rng.uniform(0.005, 0.05), rng.uniform(0.005, 0.05), rng.uniform(0, 6.3)
                img[:, :, c] += rng.uniform(20, 50) * np.sin(fy * yy + fx * xx + ph)
        out.append(np.clip(img + 128, 0, 255).astype(np.uint8))
    return out


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_mixed_128_256_stream_train_graphs_vs_oracle():
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel
    from vub_image_denoising_amd.optim import FusedAdamW
    from vub_image_denoising_amd.synth import MixedPatchLoader, load_data_gpu
    from vub_image_denoising_amd.train_graph import TrainStepGraphs
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
    tr, va = load_data_gpu(None, batch_size=2, validation_split=0.2, images=_images(), patch_size=(128, 256), seed=3)
    assert isinstance(tr, MixedPatchLoader) and isinstance(va, MixedPatchLoader)
    assert [ld.pool.patch_size for ld in tr.loaders] == [128, 256]
    params = {k: torch.from_numpy(v) for k, v in make_params(R.param_shapes(32), 21).items()}
    model = DiffusionModel(vm.RDUNet_T(base_filters=32), timesteps=20)
    model.unet.load_state_dict(params)
    model = model.cuda()
    lr, wd = 1e-4, 1e-4
    opt = FusedAdamW(model.parameters(), lr=lr, weight_decay=wd)
    # reference AdamW (torch.optim on the CPU) fed the gradients the replay used
    ref_p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    ref_opt = torch.optim.AdamW(list(ref_p.values()), lr=lr, weight_decay=wd)
    graphs = TrainStepGraphs(model, opt, 'uniform', 1.0, t_input=True)
    g = torch.Generator().manual_seed(8)
    shapes = []
    for noisy, clean in itertools.islice(iter(tr), 4):
        B, S = clean.size(0), clean.size(-1)
        shapes.append(S)
        t = torch.randint(0, 21, (B,), generator=g)
        before = {n[5:]: p.detach().cpu().clone() for n, p in model.named_parameters()}
        for k, v in ref_p.items():     # the oracle step starts from the GPU's parameters
            with torch.no_grad():
                v.copy_(before[k])
        loss = graphs(clean, noisy, t.cuda().float()).item()
        torch.cuda.synchronize()
        got_g = {n[5:]: p.grad.detach().cpu() for n, p in model.named_parameters()}
        after = {n[5:]: p.detach().cpu() for n, p in model.named_parameters()}
        ref_loss, _, ref_g, _ = R.train_step(before, clean.cpu(), noisy.cpu(), t, 20, clip_value=1.0)
        lrel = abs(loss - float(ref_loss)) / abs(float(ref_loss))
        worst = max((_rel(got_g[k], ref_g[k]), k) for k in ref_g)
        num = sum(float(((got_g[k].double() - ref_g[k].double()) ** 2).sum()) for k in ref_g)
        den = sum(float((ref_g[k].double() ** 2).sum()) for k in ref_g)
        flat = math.sqrt(num / den)
        for k, v in ref_p.items():
            v.grad = got_g[k].clone()
        ref_opt.step()
        dnum = sum(float((((after[k] - before[k]) - (ref_p[k].detach() - before[k])).double() ** 2).sum())
                   for k in ref_p)
        dden = sum(float(((ref_p[k].detach() - before[k]).double() ** 2).sum()) for k in ref_p)
        drel = math.sqrt(dnum / dden)
        print(f"{B}x{S}^2: loss {loss:.7f} oracle {float(ref_loss):.7f} (rel {lrel:.1e}), flat grad {flat:.1e}, "
              f"worst {worst[1]} {worst[0]:.1e}, AdamW delta {drel:.1e}")
        assert lrel <= 1e-6
        assert flat <= 3e-4
        if worst[0] > 1e-3:
            # A PReLU-slope gradient (sum of pre*dY over the negative pixels) can cancel to
            # a small norm where fp32 summation order alone moves it by ~1e-3: the
            # reference's own fp32 gradients reach 6e-4 from fp64 on block_2_0.* (SURVEY.md
            # section 7), and two independent fp32 paths (GPU, oracle) each that far from
            # fp64 can sit 1.2e-3 apart -- what round 5 saw (1.73e-3 on
            # block_2_0.actv_0.weight).  So such a step is judged against the fp64 oracle
            # instead, per tensor at SURVEY section 7's bound: <= 2e-3 rel-L2 (a fixed cap,
            # not a multiple of the fp32 oracle's own error)
            _, _, g64, _ = R.train_step({k: v.double() for k, v in before.items()}, clean.cpu().double(),
                                        noisy.cpu().double(), t, 20, clip_value=1.0)
            for k in ref_g:
                e_gpu = _rel(got_g[k], g64[k])
                assert e_gpu <= 2e-3, (k, e_gpu, _rel(ref_g[k], g64[k]))
        assert drel <= 1e-5
    assert shapes == [128, 256, 128, 256]
    assert graphs.captures == 2 and len(graphs.graphs) == 2
    engines = [k for k in model.unet._rdn_engines if k[-1]]
    assert {k[1] for k in engines} == {128, 256}
