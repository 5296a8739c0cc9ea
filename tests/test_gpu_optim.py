"""FusedAdam / FusedAdamW (vub_image_denoising_amd/optim.py) against torch.optim.Adam /
AdamW (the reference's optimizers: diffusion_RDUnet.py:264-276, main_diffusion_RDUnet.py:230)
over several steps, and a checkpoint save / load_state_dict / resume round trip that
continues bit-identically (diffusion_RDUnet.py:170-193)."""
import io

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model_with_grads(seed=0, bf=16):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
    torch.manual_seed(seed)
    model = DiffusionModel(vm.RDUNet_T(base_filters=bf), timesteps=20).cuda()
    g = torch.Generator().manual_seed(seed + 1)
    clean = (torch.rand(2, 3, 32, 32, generator=g) * 2 - 1).cuda()
    noisy = clean + 0.1 * torch.randn(2, 3, 32, 32, generator=g).cuda()

    class _Z:
        def zero_grad(self, set_to_none=True):
            for p in model.parameters():
                p.grad = None
    train_step_device(model, clean, noisy, _Z(), clip_value=1.0, t=torch.tensor([3, 11]).cuda())
    return model


def _set_grads(model, step):
    """Deterministic per-step gradients written into the flat gradient views."""
    g = torch.Generator(device="cuda").manual_seed(100 + step)
    for p in model.parameters():
        p.grad.copy_(torch.randn(p.shape, generator=g, device="cuda") * 1e-2)


@pytest.mark.parametrize("kind", ["adam", "adamw"])
def test_fused_adam_matches_torch(kind):
    from vub_image_denoising_amd.optim import FusedAdam, FusedAdamW
    model = _model_with_grads()
    ref = [p.detach().clone().requires_grad_(True) for p in model.parameters()]
    if kind == "adam":   # the main_*/`--optimizer_choice adam` swap, L2 weight decay
        fo = FusedAdam(model.parameters(), lr=2e-3, betas=(0.9, 0.999), weight_decay=1e-2)
        to = torch.optim.Adam(ref, lr=2e-3, betas=(0.9, 0.999), weight_decay=1e-2, foreach=False)
    else:
        fo = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
        to = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-4, foreach=False)
    for step in range(5):
        _set_grads(model, step)
        for p, r in zip(model.parameters(), ref):
            r.grad = p.grad.detach().clone()
        fo.step()
        to.step()
    worst = 0.0
    for p, r in zip(model.parameters(), ref):
        err = ((p.detach() - r.detach()).norm() / r.detach().norm().clamp_min(1e-12)).item()
        worst = max(worst, err)
    print(f"{kind}: worst per-tensor rel err after 5 steps {worst:.2e}")
    assert worst < 1e-6   # scalars rounded to fp32 from torch's doubles: ulp-level differences only
    # state in torch's per-parameter format
    st = fo.state_dict()["state"][0]
    assert int(st["step"]) == 5 and st["exp_avg"].shape == next(model.parameters()).shape
    p0 = next(model.parameters())
    for key in ("exp_avg", "exp_avg_sq"):
        a_, b_ = fo.state[p0][key].double(), to.state[ref[0]][key].double()
        e = ((a_ - b_).norm() / b_.norm()).item()
        print(f"{kind}: {key} rel err {e:.2e}")
        assert e < 1e-6


@pytest.mark.parametrize("bind_first", [False, True])
def test_fused_adam_resume_bit_identical(bind_first):
    """Save after 3 steps, load into a fresh optimizer (bound or not yet bound to
    its flat buffer), then one more step on both: identical parameters."""
    from vub_image_denoising_amd.optim import FusedAdamW
    m1 = _model_with_grads(seed=4)
    o1 = FusedAdamW(m1.parameters(), lr=1e-3, weight_decay=1e-4)
    for step in range(3):
        _set_grads(m1, step)
        o1.step()
    buf = io.BytesIO()
    torch.save({"model_state_dict": m1.state_dict(), "optimizer_state_dict": o1.state_dict()}, buf)
    buf.seek(0)
    ck = torch.load(buf, map_location="cuda", weights_only=True)
    m2 = _model_with_grads(seed=9)   # different weights and moments before the load
    o2 = FusedAdamW(m2.parameters(), lr=1e-3, weight_decay=1e-4)
    if bind_first:
        _set_grads(m2, 7)
        o2.step()
    m2.load_state_dict(ck["model_state_dict"])
    o2.load_state_dict(ck["optimizer_state_dict"])
    assert o2._step == 3 if bind_first else True
    _set_grads(m1, 3)
    _set_grads(m2, 3)
    o1.step()
    o2.step()
    assert o2._step == 4
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), n
    for a, b in zip(o1.state_dict()["state"].values(), o2.state_dict()["state"].values()):
        assert torch.equal(a["exp_avg"], b["exp_avg"]) and torch.equal(a["exp_avg_sq"], b["exp_avg_sq"])
