"""hipGraph capture of one network forward (sampling.ForwardGraph): the plain
RDUNet (UNet/RDUNet_model.py:157-186) and RDUNet_T with a t map, replayed, equal
their eager forwards bit for bit (same launches, same order), and a replay after an
in-place weight change repacks first."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_forward_graph_plain_rdunet(dtype):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.sampling import ForwardGraph
    torch.manual_seed(3)
    m = vm.RDUNet(channels=3, base_filters=32).cuda().eval().set_compute_dtype(dtype)
    x = torch.rand(1, 3, 64, 64, device="cuda") * 2 - 1
    with torch.no_grad():
        ref = m(x).clone()
        g = ForwardGraph(m, tuple(x.shape))
        assert torch.equal(g(x), ref)
        x2 = torch.rand_like(x)
        assert torch.equal(g(x2), m(x2))
        m.output_block.conv_2.weight.mul_(0.5)   # (in-place: the engine repacks before the next replay)
        m.mark_weights_dirty()
        assert torch.equal(g(x), m(x))


def test_forward_graph_rdunet_t():
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.sampling import ForwardGraph
    torch.manual_seed(4)
    m = vm.RDUNet_T(base_filters=16).cuda().eval()
    x = torch.rand(2, 3, 32, 32, device="cuda") * 2 - 1
    t = torch.tensor([0.25, 0.75], device="cuda").view(2, 1, 1, 1)
    with torch.no_grad():
        g = ForwardGraph(m, tuple(x.shape), t=t)
        assert torch.equal(g(x), m(x, t))
