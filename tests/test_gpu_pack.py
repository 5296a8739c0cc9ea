"""The batched weight repack of the train step (rdn_pack_weights_batched: every pack of
the model in one launch, one thread per 16-byte unit) against the per-element pack kernel
(rdn_pack_weights) for every pack of a real network -- 3x3 forward (chunked K) and
input-gradient (rotated, transposed) packs, the 2x2 down conv and ConvTranspose GEMM
packs -- in bf16 and fp32: the same values, so the packs must be bit-identical."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from vub_image_denoising_amd import _hip as H  # noqa: E402


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_batched_pack_equals_single_packs(dtype):
    import vub_image_denoising_amd as vm
    torch.manual_seed(3)
    m = vm.RDUNet_T(base_filters=32).cuda()
    m.set_compute_dtype(dtype)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.1)
        m(torch.rand(1, 3, 64, 64, device="cuda") * 2 - 1, torch.full((1, 1, 1, 1), 0.5, device="cuda"))
    torch.cuda.synchronize()
    packs = m._rdn_packs[torch.bfloat16 if dtype == "bf16" else torch.float32]
    code = packs.code
    modes = set()
    for (mode, w, d0, d1, kh, kw, pad0, pad1, out, rows, kp, ck) in packs.items:
        ref = torch.full_like(out, 7.0)   # (every element is written)
        H.check(H.lib().rdn_pack_weights(mode, code, w.data_ptr(), d0, d1, kh, kw, pad0, pad1, ref.data_ptr(), rows, kp,
                                         ck, H.stream_ptr()), "pack")
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int16 if out.element_size() == 2 else torch.int32),
                           ref.view(torch.int16 if ref.element_size() == 2 else torch.int32)), (mode, d0, d1, kh, ck)
        modes.add((mode, ck > 0))
    assert {(H.PACK_CONV_FWD, True), (H.PACK_CONV_DGRAD, True), (H.PACK_GEMM_T, False), (H.PACK_CONV_FWD, False)} <= modes
