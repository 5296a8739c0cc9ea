"""The batched weight repack (one launch after every optimizer step, engine.WeightPacks)
against the single-pack entry point rdn_pack_weights, item by item, bit-exact: both
gather the same fp32 weight (Unet_model.py conv weights, OIHW / IOHW) into the GEMM
operand layout and round it once."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_batched_pack_equals_single_packs(dtype):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import _hip as H
    torch.manual_seed(0)
    unet = vm.RDUNet_T(base_filters=32).cuda()
    unet.set_compute_dtype("bf16" if dtype == torch.bfloat16 else "fp32")
    x = torch.randn(1, 3, 32, 32, device="cuda")
    with torch.no_grad():
        unet(x, torch.full((1, 1, 1, 1), 0.5, device="cuda"))     # builds and fills the packs
    packs = unet._rdn_packs[dtype]
    lib = H.lib()
    code = H.dtype_code(dtype)
    st = H.stream_ptr()
    assert len(packs.items) > 100
    for (mode, w, d0, d1, kh, kw, pad0, pad1, out, rows, kp, ck) in packs.items:
        ref = torch.full_like(out, float("nan"))
        H.check(lib.rdn_pack_weights(mode, code, w.data_ptr(), d0, d1, kh, kw, pad0, pad1, ref.data_ptr(), rows, kp,
                                     ck, st), "rdn_pack_weights")
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int16 if dtype == torch.bfloat16 else torch.int32),
                           ref.view(torch.int16 if dtype == torch.bfloat16 else torch.int32)), (mode, d0, d1, kh, ck)
