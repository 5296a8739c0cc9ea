"""Data-parallel training through the real network on the GPU: two ranks (gloo
over the one GPU of the box; the 8-GPU RCCL run is the driver's), each training on
half of a batch with ddp.GradSync attached (bucketed all-reduce on a side stream,
overlapped with the fused backward), must end with the clipped gradient the single
process computes on the whole batch: images are
independent and the loss is a mean over equal halves."""
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


# (dtype, base filters, image size, bucket MB).  The bf16 case runs the fused level-0
# dgrad+wgrad kernel (conv3_dw: F0=32 level-0 shapes), whose weight-gradient reduce
# runs on the COMPUTE stream while the other layers' reduce on the side stream:
# 50-KB buckets put bucket boundaries on fused layers, so an all-reduce ordered
# after only one of the two streams would read unreduced gradients
CASES = [("fp32", 16, 32, 0.5), ("bf16", 32, 64, 0.05)]


def _setup(dtype="fp32", bf=16, size=32, seed=41):
    from oracle.weights import make_params
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel
    model = DiffusionModel(vm.RDUNet_T(base_filters=bf), timesteps=20)
    sd = model.state_dict()
    p = make_params({k[5:]: tuple(v.shape) for k, v in sd.items()}, seed)
    model.load_state_dict({"unet." + k: torch.from_numpy(v) for k, v in p.items()})
    g = torch.Generator().manual_seed(5)
    clean = torch.rand(4, 3, size, size, generator=g) * 2 - 1
    noisy = clean + 0.2 * torch.randn(4, 3, size, size, generator=g)
    t = torch.tensor([3, 11, 17, 20])
    model = model.cuda()
    model.unet.set_compute_dtype(dtype)
    return model, clean.cuda(), noisy.cuda(), t.cuda()


def _rank(rank, world, init_file, q, case):
    try:
        dtype, bf, size, bucket_mb = case
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
        from vub_image_denoising_amd.ddp import GradSync
        from vub_image_denoising_amd.diffusion_RDUnet import train_step_device
        model, clean, noisy, t = _setup(dtype, bf, size)
        opt = torch.optim.SGD(model.parameters(), lr=0.0)
        sl = slice(2 * rank, 2 * rank + 2)
        train_step_device(model, clean[sl], noisy[sl], opt, clip_value=1.0, t=t[sl])  # builds the flat buffer
        model.unet._rdn_flat.grad_sync = GradSync(model.unet._rdn_flat, bucket_mb=bucket_mb)
        train_step_device(model, clean[sl], noisy[sl], opt, clip_value=1.0, t=t[sl])
        torch.cuda.synchronize()
        q.put((rank, model.unet._rdn_flat.gflat.cpu().numpy(), len(model.unet._rdn_flat.grad_sync.buckets)))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put((rank, repr(e), 0))


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_ddp_two_ranks_match_single_process(tmp_path, case):
    from vub_image_denoising_amd.diffusion_RDUnet import train_step_device
    model, clean, noisy, t = _setup(*case[:3])
    opt = torch.optim.SGD(model.parameters(), lr=0.0)
    train_step_device(model, clean, noisy, opt, clip_value=1.0, t=t)
    torch.cuda.synchronize()
    ref = model.unet._rdn_flat.gflat.cpu().numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, str(tmp_path / "rdv"), q, case)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, g, nb = q.get(timeout=110)
        assert not isinstance(g, str), g
        res[r] = (g, nb)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[0][1] > 1, "several buckets (launched during the backward)"
    assert np.array_equal(res[0][0], res[1][0]), "ranks hold the same averaged gradient"
    err = np.linalg.norm(res[0][0] - ref) / np.linalg.norm(ref)
    worst = max(np.linalg.norm(res[0][0][lo:hi] - ref[lo:hi]) / max(np.linalg.norm(ref[lo:hi]), 1e-30)
                for lo, hi in _param_ranges(model))
    print(f"{case[0]}: {res[0][1]} buckets, flat rel err {err:.2e}, worst tensor {worst:.2e}")
    # fp32: summation order only.  bf16: the split-K weight-gradient partials of a
    # half batch sum in another order (fp32), the bf16 activations are per image
    # and identical -- a bucket reduced before its gradients were final would be off
    # by O(1) in some tensor
    assert err < (1e-5 if case[0] == "fp32" else 1e-3), err
    assert worst < (1e-4 if case[0] == "fp32" else 1e-2), worst


def _param_ranges(model):
    fp = model.unet._rdn_flat
    return [(o, o + p.numel()) for p, o in zip(fp.params, fp.offsets)]


def _rank_accum(rank, world, init_file, q):
    try:
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
        from vub_image_denoising_amd.ddp import GradSync
        from vub_image_denoising_amd.diffusion_RDUnet import train_step_device
        model, clean, noisy, t = _setup("fp32", 16, 32)
        opt = torch.optim.SGD(model.parameters(), lr=0.0)
        sl = slice(2 * rank, 2 * rank + 2)
        train_step_device(model, clean[sl], noisy[sl], opt, clip_value=1.0, t=t[sl])  # builds the flat buffer
        model.unet._rdn_flat.grad_sync = GradSync(model.unet._rdn_flat, bucket_mb=0.5)
        train_step_device(model, clean[sl], noisy[sl], opt, clip_value=1.0, t=t[sl], clip=False)
        train_step_device(model, clean[sl], noisy[sl], opt, clip_value=1.0, t=t.flip(0)[sl], zero_grad=False)
        torch.cuda.synchronize()
        q.put((rank, torch.cat([p.grad.flatten() for p in model.parameters()]).cpu().numpy()))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put((rank, repr(e)))


def test_ddp_accumulate_then_clip(tmp_path):
    """zero_grad=False with clip=True (advisor r04): the gradients held from the
    previous call are already averaged, so the 1/world factor must not be folded
    into this clip -- two ranks equal one process accumulating the same two
    half-batch-per-rank steps, then clipping."""
    from vub_image_denoising_amd.diffusion_RDUnet import train_step_device
    model, clean, noisy, t = _setup("fp32", 16, 32)
    opt = torch.optim.SGD(model.parameters(), lr=0.0)
    train_step_device(model, clean, noisy, opt, clip_value=1.0, t=t, clip=False)
    train_step_device(model, clean, noisy, opt, clip_value=1.0, t=t.flip(0), zero_grad=False)
    torch.cuda.synchronize()
    ref = torch.cat([p.grad.flatten() for p in model.parameters()]).cpu().numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_accum, args=(r, 2, str(tmp_path / "rdv"), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, g = q.get(timeout=110)
        assert not isinstance(g, str), g
        res[r] = g
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert np.array_equal(res[0], res[1])
    err = np.linalg.norm(res[0] - ref) / np.linalg.norm(ref)
    assert err < 1e-5, err
