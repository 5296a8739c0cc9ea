"""PReLU backward fused into the input-gradient epilogue of the layer's last
consumer (rdn_conv_desc.gout: conv_k+1 finishes dense slice out_k, Unet_model.py:
81-87; up_l.conv finishes up_l.conv_t's output, :43) against the separate
rdn_prelu_bwd pass it replaces (aten _prelu_kernel_backward + conv bias gradient).

fp32: the epilogue gates the same fp32 value the separate pass would have read back,
so every dYpre -- hence every conv weight gradient and every activation gradient --
is bit-identical; the PReLU-slope and conv-bias gradients differ only in how the
pixel sum is cut into partials (per 8x16 / 16x16 tile instead of per pass block):
rel-L2 <= 1e-5.  bf16: the gate multiplies the fp32 sum instead of its bf16
rounding (slope branch: one bf16 rounding fewer), so gradients agree to bf16
rounding noise: rel-L2 <= 1e-2 per tensor (the full-size oracle tests bound the
absolute error of the default path).  bf16 also runs the gate-out epilogue of the
fused dgrad+wgrad kernel (conv3_dw ",go", round 4): up_0.conv finishing up_0.conv_t
and the level-1 conv_0s finishing the layer that feeds their block (its residual
reader, the block's conv_3, adds its share earlier in backward order; a finished
conv_3 also gets its plain dY stored, RDN_EPI_GOUT_KEEP, for its own residual)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def DW_PREGATED():
    from vub_image_denoising_amd import engine as E
    return E.DW_PREGATED


_LAST_DW = {}


def _dw_keys(S):
    return _LAST_DW.get(S, [])


def _grads(gate_out, dtype, B, S, F0=32, seed=0):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import engine as E
    old = E.GATE_OUT
    E.GATE_OUT = gate_out   # (on by default since round 4: engine.py has the step A/B)
    try:
        torch.manual_seed(seed)
        m = vm.RDUNet_T(base_filters=F0).cuda()
        m.set_compute_dtype(dtype)
        g = torch.Generator().manual_seed(seed + 1)
        x = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).cuda()
        t = torch.rand(B, 1, 1, 1, generator=g).cuda()
        w = torch.randn(B, 3, S, S, generator=g).cuda()
        y = m(x, t)
        (y * w).mean().backward()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        keys = []
        _LAST_DW[S] = []
        for pool in m._rdn_engines.values():
            for eng in pool:
                for L in eng.layers:
                    if "dw" in L.extra.get("info", {}):
                        _LAST_DW.setdefault(S, []).append((L.name, L.extra["info"]["dw"][2]))
                    if L.extra.get("gates") is not None:
                        info = L.extra["info"]
                        keys.append((L.name, L.extra["gates"].name, info["dw"][2] if "dw" in info else info["dgrad"][2]))
        return y.detach().clone(), grads, keys
    finally:
        E.GATE_OUT = old


@pytest.mark.parametrize("B,S", [(2, 256), (2, 64)])
def test_gate_out_fp32_bit_identical_dypre(B, S):
    y0, g0, k0 = _grads(False, "fp32", B, S)
    y1, g1, k1 = _grads(True, "fp32", B, S)
    assert not k0
    # every dense slice out_0..2 at levels 2/3 (out_1..2 at level 1) and every
    # up_l.conv_t output is finished by an epilogue
    assert len(k1) >= 16, k1
    assert torch.equal(y0, y1)
    for n in g0:
        if ".conv" in n and n.endswith(".weight"):
            assert torch.equal(g1[n], g0[n]), (n, _rel(g1[n], g0[n]))
    worst = max(_rel(g1[n], g0[n]) for n in g0)
    assert worst <= 1e-5, sorted(((_rel(g1[n], g0[n]), n) for n in g0), reverse=True)[:5]


@pytest.mark.parametrize("B,S", [(16, 256), (2, 256), (2, 64), (1, 32)])
def test_gate_out_bf16_matches_separate(B, S):
    y0, g0, k0 = _grads(False, "bf16", B, S)
    y1, g1, k1 = _grads(True, "bf16", B, S)
    assert not k0
    assert torch.equal(y0, y1)
    worst = max(_rel(g1[n], g0[n]) for n in g0)
    assert worst <= 1e-2, sorted(((_rel(g1[n], g0[n]), n) for n in g0), reverse=True)[:5]
    if S >= 64:   # (64^2: the 8x8 level-3 grids keep the separate pass: no full 8x16 tiles;
        # bf16: level-1 conv_1 / conv_2 run as the fused gated dgrad+wgrad (conv3_dw
        # column halves), which finishes no other layer -- 14 finishers at 64^2)
        assert len(k1) >= 14, k1
    if S >= 64:   # the fused dgrad+wgrad finishers (conv3_dw ",go"): up_0.conv finishes
        # up_0.conv_t; a level-1 block's conv_0 finishes the layer feeding the block
        # (encoder block_1_1 <- block_1_0.conv_3; decoder block_1_2 <- up_1.conv,
        # block_1_3 <- block_1_2.conv_3; block_1_0's input is down_0's, a 2x2 conv: not here;
        # since round 5 the finished conv_3s run the pre-gated fused dgrad+wgrad, ",pregated")
        fin = {(j, k) for j, k, key in k1 if key.startswith("conv3_dw") and ",go" in key}
        assert fin == {("up_0.conv", "up_0.conv_t"), ("block_1_1.conv_0", "block_1_0.conv_3"),
                       ("block_1_2.conv_0", "up_1.conv"), ("block_1_3.conv_0", "block_1_2.conv_3")}, k1
        if DW_PREGATED():   # the finished level-1 conv_3s read the dYpre these epilogues write
            pre = {L for L, key in _dw_keys(S) if key.endswith(",pregated>")}
            assert {"block_1_0.conv_3", "block_1_2.conv_3"} <= pre, pre
    if B == 16:   # the train step's shape: conv3_big serves the level-1 and up-conv finishers
        assert any("conv3_big" in k and ",go" in k for _, _, k in k1), k1
        assert any("conv3_halo" in k for _, _, k in k1), k1
