"""Split-K forward of the small-grid 3x3 convs (rdn_conv_fwd_splitk, csrc/conv3_halo.hip;
engine.SPLITK): a batch-1 forward's deep levels (UNet/RDUNet_model.py:157-186, config 1's
RDUNet(64) on 1 x 3 x 64^2) walk the input channels in slices on separate blocks and one
launch sums the slices in slice order and applies the conv epilogue.

Only the fp32 summation order changes against the single-pass launch (the slices are
summed chunk-group by chunk-group instead of in one running accumulator), so:
* fp32: the network output within rel-L2 1e-5 of the unsplit build (summation-order
  noise ~1e-7 per conv, 44 convs deep) and within the config-1 oracle bound (1e-3) of
  the CPU oracle on the same weights;
* bf16: within rel-L2 1e-2 of the unsplit build (a 1-ulp flip of a bf16 activation
  after a differently-ordered fp32 sum, propagated);
* RDUNet_T's forward-only path (the samplers' engine) at batch 1: the output within
  rel-L2 1e-5 of the unsplit build; train engines never split.  (The train step keeps
  the single-pass launches: at batch 1 its gradients are sums over a few thousand pixels
  with random signs, so one PReLU input within the fp32 noise (~1e-6) of 0 whose gate
  flips under the reordered sum moves its layer's weight gradient by ~1/sqrt(P) and
  everything upstream with it -- measured on a 64^2 image with split train engines:
  forward states equal to 4e-6, one gate flipped, gradients 3.4e-3 from the fp64
  oracle against 7e-7 unsplit; with no flip (48 x 80) 5e-7.)
* deterministic: two split runs bit-identical.
The split path must actually be taken (engine layers carry `splitk`)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(model_fn, x, split, dtype="fp32", t=None, train=False, seed=0):
    from vub_image_denoising_amd import engine as E
    old = E.SPLITK
    E.SPLITK = split
    try:
        torch.manual_seed(seed)
        m = model_fn().cuda()
        m.set_compute_dtype(dtype)
        state = None
        if train:
            y = m(x, t) if t is not None else m(x)
            eng = [e for pool in m._rdn_engines.values() for e in pool if e.train][0]
            state = {k: v.detach().float().clone() for k, v in eng.bufs.items()}   # what backward reads
            w = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).cuda()
            (y * w).mean().backward()
            grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        else:
            m.eval()
            with torch.no_grad():
                y = m(x, t) if t is not None else m(x)
            grads = None
        nsplit = sum("splitk" in L.extra for pool in m._rdn_engines.values() for eng in pool for L in eng.layers)
        m.fwd_state = state
        return y.detach().clone(), grads, nsplit, m
    finally:
        E.SPLITK = old


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def test_rdunet64_batch1_fp32_split_vs_unsplit_and_oracle():
    import vub_image_denoising_amd as vm
    from oracle import rdunet_ref as R
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(1)).cuda()
    mk = lambda: vm.RDUNet(channels=3, base_filters=64)   # noqa: E731
    ys, _, ns, m = _run(mk, x, True)
    yu, _, nu, _ = _run(mk, x, False)
    ys2, _, _, _ = _run(mk, x, True)
    print(f"split layers {ns}, unsplit {nu}; rel {_rel(ys, yu):.2e}")
    assert ns >= 8 and nu == 0
    assert torch.equal(ys, ys2)
    assert _rel(ys, yu) < 1e-5
    params = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    with torch.no_grad():
        yr = R.rdunet_forward(params, x.cpu())
    r = _rel(ys.cpu(), yr)
    print(f"vs oracle rel {r:.2e}")
    assert r < 1e-3


def test_rdunet64_batch1_bf16_split_vs_unsplit():
    import vub_image_denoising_amd as vm
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(2)).cuda()
    mk = lambda: vm.RDUNet(channels=3, base_filters=64)   # noqa: E731
    ys, _, ns, _ = _run(mk, x, True, "bf16")
    yu, _, _, _ = _run(mk, x, False, "bf16")
    print(f"bf16 split layers {ns}; rel {_rel(ys, yu):.2e}")
    assert ns >= 4
    assert _rel(ys, yu) < 1e-2


@pytest.mark.parametrize("hw", [(64, 64), (48, 80)])
def test_rdunet_t_batch1_forward_split_train_unsplit(hw):
    import vub_image_denoising_amd as vm
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(1, 3, *hw, generator=g) * 2 - 1).cuda()
    t = torch.rand(1, 1, 1, 1, generator=g).cuda()
    mk = lambda: vm.RDUNet_T(base_filters=32)   # noqa: E731
    ys, _, ns, _ = _run(mk, x, True, "fp32", t=t)
    yu, _, _, _ = _run(mk, x, False, "fp32", t=t)
    _, gs, ntrain, _ = _run(mk, x, True, "fp32", t=t, train=True)
    print(f"RDUNet_T {hw}: forward split layers {ns}, train-engine split layers {ntrain}; rel {_rel(ys, yu):.2e}")
    assert ns >= 1 and ntrain == 0
    assert _rel(ys, yu) < 1e-5
    assert all(np.isfinite(v.cpu().numpy()).all() for v in gs.values())


def test_split_forward_repeatable_eager_and_replayed():
    """The split forwards share one slab workspace per engine: repeated forwards of one
    engine, eager and graph-replayed, are bit-identical, and a forward of a different input
    in between leaves nothing behind.  (An in-launch combine of the slabs -- the last slice
    block of a tile sums them after a ticket add -- was tried in r06 and measured slower:
    config 1's graph forward 1.22 -> 2.07 ms, one block reading up to 32 slabs serially.)"""
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import engine as E
    assert E.SPLITK
    torch.manual_seed(0)
    m = vm.RDUNet(channels=3, base_filters=64).cuda().eval()
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(7)).cuda()
    x2 = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(8)).cuda()
    with torch.no_grad():
        y0 = m(x).clone()
        y2 = m(x2).clone()
        ys = [m(x).clone() for _ in range(3)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        xs = x2.clone()
        with torch.cuda.stream(s):
            m(xs)
            with torch.cuda.graph(g, stream=s):
                yg = m(xs)
        torch.cuda.current_stream().wait_stream(s)
        reps = []
        for inp in (x, x2, x):
            xs.copy_(inp)
            g.replay()
            reps.append(yg.clone())
        torch.cuda.synchronize()
    nsplit = sum("splitk" in L.extra for pool in m._rdn_engines.values() for eng in pool for L in eng.layers)
    assert nsplit >= 8
    for y in ys:
        assert torch.equal(y, y0)
    assert not torch.equal(y2, y0)
    assert torch.equal(reps[0], y0) and torch.equal(reps[2], y0) and torch.equal(reps[1], y2)
