"""rdn_image_metrics (csrc/metrics.hip) on the GPU against the CPU oracle
(oracle/metrics_ref.py: scikit-image 0.22 PSNR / SSIM restated, pinned in
tests/test_metrics_cpu.py).  Tolerance: the kernel sums the 7x7 window in fp32
directly where scipy's uniform_filter keeps running sums; both round the window
means to fp32, so the cropped-mean SSIM agrees to ~1e-6 -- the test allows 2e-5
absolute on SSIM and 1e-4 dB on PSNR (float64 sums on both sides)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import metrics_ref as M  # noqa: E402


def _pair(rng, shape, noise=0.1, clip=True):
    a = rng.uniform(-1, 1, shape).astype(np.float32)
    # smooth structure so SSIM is far from 0 and from 1
    a = (a + np.roll(a, 1, -1) + np.roll(a, 1, -2)) / 3
    b = a + noise * rng.standard_normal(shape).astype(np.float32)
    if clip:
        b = np.clip(b, -1, 1)
    return a.astype(np.float32), b.astype(np.float32)


# (incl. several column tiles, and the 64-block SIDD batch of bench.py's metrics leg)
@pytest.mark.parametrize("shape", [(1, 1, 7, 7), (2, 3, 13, 70), (3, 3, 64, 64), (4, 3, 256, 256), (1, 2, 45, 130),
                                   (1, 3, 7, 8), (2, 3, 40, 520), (5, 3, 100, 248), (64, 3, 256, 256)])
def test_image_metrics_match_oracle(shape):
    from vub_image_denoising_amd.metrics import image_metrics
    rng = np.random.default_rng(shape[2] * 1000 + shape[3])
    a, b = _pair(rng, shape)
    psnr, ssim = image_metrics(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), 2.0)
    rp, rs = M.batch_metrics(a, b, 2.0)
    np.testing.assert_allclose(psnr.cpu().numpy(), rp, rtol=0, atol=1e-4)
    np.testing.assert_allclose(ssim.cpu().numpy(), rs, rtol=0, atol=2e-5)


def test_identical_and_edge_cases():
    from vub_image_denoising_amd.metrics import image_metrics, peak_signal_noise_ratio, structural_similarity
    rng = np.random.default_rng(3)
    a, b = _pair(rng, (2, 3, 32, 40))
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    psnr, ssim = image_metrics(ta, ta, 2.0)
    assert torch.isinf(psnr).all() and torch.allclose(ssim, torch.ones_like(ssim), atol=1e-6)
    # skimage-named single-image wrappers: HWC with channel_axis=-1 as evaluate_SIDD.py:63-64
    hwc_a, hwc_b = ta[1].permute(1, 2, 0), tb[1].permute(1, 2, 0)
    assert structural_similarity(hwc_a, hwc_b, data_range=2, channel_axis=-1) == pytest.approx(
        M.ssim(a[1].transpose(1, 2, 0), b[1].transpose(1, 2, 0), 2.0, channel_axis=-1), abs=2e-5)
    assert peak_signal_noise_ratio(hwc_a, hwc_b, data_range=2) == pytest.approx(M.psnr(a[1], b[1], 2.0), abs=1e-4)
    with pytest.raises(ValueError):
        image_metrics(ta[:, :, :6], tb[:, :, :6], 2.0)      # smaller than the 7x7 window
    with pytest.raises(RuntimeError):
        image_metrics(torch.from_numpy(a), torch.from_numpy(b), 2.0)   # CPU tensors: no fallback


def test_evaluate_model_end_to_end(tmp_path):
    """evaluate_SIDD.evaluate_model over a synthetic .mat: its averages equal the
    oracle's metrics of the same denoised blocks."""
    import scipy.io
    from torch.utils.data import DataLoader
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel
    from vub_image_denoising_amd.evaluate_SIDD import SIDDMatDataset, evaluate_model
    rng = np.random.default_rng(7)
    gt = rng.integers(0, 256, (2, 3, 32, 32, 3), dtype=np.uint8)
    noisy = np.clip(gt.astype(np.int32) + rng.integers(-20, 21, gt.shape), 0, 255).astype(np.uint8)
    scipy.io.savemat(tmp_path / "n.mat", {"ValidationNoisyBlocksSrgb": noisy})
    scipy.io.savemat(tmp_path / "g.mat", {"ValidationGtBlocksSrgb": gt})
    ds = SIDDMatDataset(str(tmp_path / "n.mat"), str(tmp_path / "g.mat"))
    torch.manual_seed(0)
    model = DiffusionModel(vm.RDUNet_T(base_filters=16), timesteps=4).cuda()
    outs = []
    orig = model.improved_sampling

    def sampler(x):
        y = orig(x)
        outs.append(y.clone())
        return y

    p, s, t_ms, samples = evaluate_model(model, DataLoader(ds, batch_size=4), "cuda", sampler=sampler)
    den = torch.cat(outs).cpu().numpy()
    ref_gt = np.stack([ds[i][1].numpy() for i in range(len(ds))])
    rp, rs = M.batch_metrics(ref_gt, den, 2.0)
    assert p == pytest.approx(float(np.mean(rp)), abs=1e-4)
    assert s == pytest.approx(float(np.mean(rs)), abs=2e-5)
    assert t_ms > 0 and len(samples) == 0   # 6 blocks: none in the reference's sample range 11..14
