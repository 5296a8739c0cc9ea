"""dYpre / partial / slab slots of the weight-gradient stream (engine.py, round 4):
one slot per layer while their buffers fit RDN_SLOT_BUDGET of the free device
memory, else the 6-slot ring (the dgrad chain then waits for the side stream where
it reuses a slot).  Scheduling only: the gradients are bit-identical either way, and
the choice is made once per engine pool (its engines share the slot buffers)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(budget, B=2, S=256, seed=0):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import engine as E
    old = E.SLOT_BUDGET
    E.SLOT_BUDGET = budget
    try:
        torch.manual_seed(seed)
        m = vm.RDUNet_T(base_filters=32).cuda()
        m.set_compute_dtype("bf16")
        g = torch.Generator().manual_seed(seed + 1)
        x = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).cuda()
        t = torch.rand(B, 1, 1, 1, generator=g).cuda()
        w = torch.randn(B, 3, S, S, generator=g).cuda()
        grads = []
        for _ in range(2):   # one forward, one backward: engine 0 serves both
            m.zero_grad(set_to_none=True)
            y = m(x, t)
            (y * w).mean().backward()
            grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
        # two forwards alive before their backwards (x and its mirror image): the pool's
        # second engine holds the second graph's activations, and both backwards run
        # on the ONE set of backward scratch (slots, partials, slabs) the pool shares
        m.zero_grad(set_to_none=True)
        y1, y2 = m(x, t), m(x.flip(-1), t)
        (y1 * w).mean().backward()
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
        m.zero_grad(set_to_none=True)
        (y2 * w).mean().backward()
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
        pools = [pool for pool in m._rdn_engines.values() if any(eng.train for eng in pool)]
        assert len(pools) == 1 and len(pools[0]) >= 2, [len(p) for p in pools]
        assert all(eng.scratch is pools[0][0].scratch for eng in pools[0]), "one scratch dict per pool"
        slots = {eng.slots for pool in m._rdn_engines.values() for eng in pool if eng.train}
        nlayers = {len(eng.layers) for pool in m._rdn_engines.values() for eng in pool if eng.train}
        return grads, slots, nlayers
    finally:
        E.SLOT_BUDGET = old


def test_slot_budget_ring_bit_identical():
    """The ring (budget 0) and one slot per layer give bit-identical gradients, also
    with two live graphs on two pooled engines sharing the pool's scratch; the
    second graph's gradient (mirrored input) differs from the first's, so a backward
    that read the other engine's buffers would show."""
    g_all, s_all, n_all = _grads(1e9)
    g_ring, s_ring, _ = _grads(0.0)
    assert s_all == n_all and s_ring == {6}, (s_all, s_ring, n_all)
    assert len(g_all) == len(g_ring) == 4
    for a, b in zip(g_all, g_ring):
        for n in a:
            assert torch.equal(a[n], b[n]), n
    for n in g_ring[0]:   # the live-graph backward of x equals the sequential one
        assert torch.equal(g_ring[2][n], g_ring[0][n]), n
    assert any(not torch.equal(g_ring[3][n], g_ring[2][n]) for n in g_ring[2])


def _grads_batch(batch, B=2, S=256, seed=0):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import engine as E
    old = E.REDUCE_BATCH
    E.REDUCE_BATCH = batch
    try:
        torch.manual_seed(seed)
        m = vm.RDUNet_T(base_filters=32).cuda()
        m.set_compute_dtype("bf16")
        g = torch.Generator().manual_seed(seed + 1)
        x = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).cuda()
        t = torch.rand(B, 1, 1, 1, generator=g).cuda()
        w = torch.randn(B, 3, S, S, generator=g).cuda()
        (m(x, t) * w).mean().backward()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    finally:
        E.REDUCE_BATCH = old


def test_reduce_batch_bit_identical():
    """The fused layers' split-K reduces batched into one launch per run of fused
    layers (rdn_wgrad_reduce_batch) against one launch per layer: same per-block
    work and summation order, so every gradient is bit-identical."""
    g1, g0 = _grads_batch(True), _grads_batch(False)
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n
