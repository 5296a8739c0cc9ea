"""Config 2 at full size: the 256x256 train step (diffusion_RDUnet.py:76-115) at the
benched batch 16 and at north_star's batch 32, against the CPU oracle.

Oracle cost: the reference's loss is the mean over the whole batch, so its
gradient is the mean of per-image gradients; the oracle runs image by image
(fp32, ~1.3 GB each instead of ~40 GB for the batch) and clips the mean
(clip_grad_norm_ semantics, :113).  An fp64 oracle at this size costs minutes
(measured 7 s per image on 8 cores), so the fp32 GPU path is held to the fp32
oracle with a stated budget instead:

* loss: <= 1e-6 relative (both sides fp32; the loss is one reduction);
* every gradient tensor: rel-L2 <= 1e-3, the whole flat gradient <= 1e-4.
  Budget: SURVEY.md §8c measured the reference's own fp32 gradients at up to
  6e-4 from fp64 (64x64, B=2); the GPU's fp32 MFMA is exact fp32 (only the
  summation order differs), so two fp32 results differ by their two rounding
  paths: <= 2 x 6e-4 ~ 1e-3 per tensor.  Measured on MI355X: loss 4e-9 / 2e-8,
  worst tensor 6e-5 / 4e-5, flat 7e-6 / 4e-6 (B16 / B32);
* bf16 (the benched arithmetic) against the same fp32 oracle: loss <= 5e-3
  relative, gradient rel-L2 <= 6e-2 per tensor and <= 3e-2 for the whole flat
  gradient.  Budget: bf16 keeps 8 significant bits (unit roundoff 2^-9 = 2e-3);
  every layer rounds its activations once in forward and its gradients once in
  backward, ~70 layers deep: sqrt(2*70) * 2e-3 ~ 2.4e-2 for a typical tensor,
  2.5x margin for the worst one.  The network output carries ~2.5e-3 relative
  error on values of magnitude ~1, and the loss is the mean
  Charbonnier residual of ~0.13, so a bias of ~3e-4 absolute (2.5e-3 relative)
  is expected: 2x margin.  Measured on MI355X: loss 2.1e-3 / 2.2e-3, flat 7.1e-3 /
  7.2e-3, worst tensor 1.9e-2 / 2.0e-2 (B16 / B32).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import rdunet_ref as R  # noqa: E402
from oracle.weights import make_params  # noqa: E402

T_STEPS = 20
_CACHE = {}


def _inputs(batch, size=256, seed=77):
    g = torch.Generator().manual_seed(seed + batch)
    clean = torch.rand(batch, 3, size, size, generator=g) * 2 - 1
    noisy = clean + (25 / 255 * 2) * torch.randn(batch, 3, size, size, generator=g)
    t = torch.randint(0, T_STEPS + 1, (batch,), generator=g)
    return clean, noisy, t


def _params():
    return {k: torch.from_numpy(v) for k, v in make_params(R.param_shapes(32), 5).items()}


def _oracle(batch):
    """fp32 oracle, image by image: mean loss, clipped mean gradient."""
    if batch in _CACHE:
        return _CACHE[batch]
    import os
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
    clean, noisy, t = _inputs(batch)
    params = _params()
    loss, gsum = 0.0, None
    for b in range(batch):
        lb, _, gb, _ = R.train_step(params, clean[b:b + 1], noisy[b:b + 1], t[b:b + 1], T_STEPS, clip_value=math.inf)
        loss += float(lb)
        gsum = gb if gsum is None else {k: gsum[k] + gb[k] for k in gb}
    g = {k: v / batch for k, v in gsum.items()}
    total, clipped = R.clip_grad_norm(list(g.values()), 1.0)
    _CACHE[batch] = (loss / batch, dict(zip(g.keys(), clipped)), float(total))
    return _CACHE[batch]


def _gpu(batch, dtype):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
    model = DiffusionModel(vm.RDUNet_T(base_filters=32), timesteps=T_STEPS)
    model.unet.load_state_dict(_params())
    model = model.cuda()
    model.unet.set_compute_dtype(dtype)
    clean, noisy, t = _inputs(batch)

    class _Z:
        def zero_grad(self, set_to_none=True):
            for p in model.parameters():
                p.grad = None
    loss = train_step_device(model, clean.cuda(), noisy.cuda(), _Z(), clip_value=1.0, t=t.cuda()).item()
    grads = {n[5:]: p.grad.detach().cpu() for n, p in model.named_parameters()}
    del model
    torch.cuda.empty_cache()
    return loss, grads


def _compare(batch, dtype, loss_tol, tensor_tol, flat_tol):
    ref_loss, ref_g, ref_norm = _oracle(batch)
    loss, g = _gpu(batch, dtype)
    lrel = abs(loss - ref_loss) / abs(ref_loss)
    worst, worst_n, num, den = 0.0, "", 0.0, 0.0
    for n, r in ref_g.items():
        d = (g[n].double() - r.double())
        e = (d.norm() / r.double().norm().clamp_min(1e-30)).item()
        num += float((d ** 2).sum())
        den += float((r.double() ** 2).sum())
        if e > worst:
            worst, worst_n = e, n
    flat = math.sqrt(num / den)
    print(f"B={batch} {dtype}: loss {loss:.7f} oracle {ref_loss:.7f} (rel {lrel:.2e}); grad-norm {ref_norm:.4f}; "
          f"flat grad rel {flat:.2e}; worst tensor {worst_n} {worst:.2e}")
    assert lrel <= loss_tol
    assert flat <= flat_tol
    assert worst <= tensor_tol, (worst_n, worst)


@pytest.mark.parametrize("batch", [16, 32])
def test_train_step_256_fp32_vs_oracle(batch):
    _compare(batch, "fp32", 1e-6, 1e-3, 1e-4)


@pytest.mark.parametrize("batch", [16, 32])
def test_train_step_256_bf16_vs_oracle(batch):
    _compare(batch, "bf16", 5e-3, 6e-2, 3e-2)
