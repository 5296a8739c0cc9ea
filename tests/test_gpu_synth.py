"""rdn_synth_batch (csrc/synth.hip) on the GPU against the CPU oracle
(oracle/synth_ref.py, itself pinned to Pillow and to the reference's noise lines in
tests/test_synth_cpu.py).

* given float64 noise (the reference's np.random.normal draws): bit-exact outputs;
* device noise stream: the oracle's numpy restatement of the same counter hash +
  Box-Muller; double-precision log/cos of the GPU and of libm may differ in the
  last ulp, so an element may land one uint8 step apart at a truncation boundary:
  <= 1e-4 of the elements, never more than one step (2/255 in [-1, 1]);
* paired (SIDD) pools; the GpuLoader / load_data_gpu front-end end to end.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import synth_ref as S  # noqa: E402


def _pool(rng, shapes, C=3, P=64, paired=False):
    from vub_image_denoising_amd.synth import PatchPool
    imgs = [rng.integers(0, 256, (h, w, C), dtype=np.uint8) for h, w in shapes]
    noisy = [rng.integers(0, 256, (h, w, C), dtype=np.uint8) for h, w in shapes] if paired else None
    return PatchPool(imgs, P, "cuda", noisy_images=noisy), imgs, noisy


def _items(pool, rng, n, sigmas=(15.0, 25.0, 50.0)):
    from vub_image_denoising_amd.synth import ITEM_DTYPE
    items = np.zeros(n, ITEM_DTYPE)
    params = []
    for k in range(n):
        p = int(rng.integers(0, len(pool)))
        flip = bool(k % 2)
        angle = None if k % 3 == 0 else float(rng.uniform(-10, 10))
        sigma = sigmas[k % len(sigmas)]
        seed = int(rng.integers(0, 2 ** 63))
        pool.encode(p, sigma, flip, angle, seed, items[k])
        params.append((p, flip, angle, sigma, seed))
    return items, params


def _patch(pool, imgs, p):
    k, top, left = pool.patches[p]
    P = pool.patch_size
    return imgs[k][top:top + P, left:left + P]


@pytest.mark.parametrize("C", [3, 1])
def test_synth_given_noise_bit_exact(C):
    from vub_image_denoising_amd.synth import synth_batch
    rng = np.random.default_rng(C)
    pool, imgs, _ = _pool(rng, [(200, 260), (64, 64), (130, 70)], C=C)
    items, params = _items(pool, rng, 9)
    P = pool.patch_size
    noise = rng.normal(size=(9, P, P, C)) * np.array([s for _, _, _, s, _ in params])[:, None, None, None]
    noisy, clean = synth_batch(pool, items, torch.from_numpy(noise).cuda())
    torch.cuda.synchronize()
    for k, (p, flip, angle, sigma, seed) in enumerate(params):
        rn, rc = S.synth_item(_patch(pool, imgs, p), flip, angle, noise[k])
        assert np.array_equal(clean[k].cpu().numpy(), rc), k
        assert np.array_equal(noisy[k].cpu().numpy(), rn), k


def test_synth_device_noise_matches_restatement():
    from vub_image_denoising_amd.synth import synth_batch
    rng = np.random.default_rng(7)
    pool, imgs, _ = _pool(rng, [(256, 256), (300, 200)], P=96)
    items, params = _items(pool, rng, 8)
    noisy, clean = synth_batch(pool, items)
    torch.cuda.synchronize()
    P, C = pool.patch_size, pool.channels
    diff_total, n_total = 0, 0
    for k, (p, flip, angle, sigma, seed) in enumerate(params):
        z = sigma * S.device_normal(seed, P * P * C).reshape(P, P, C)
        rn, rc = S.synth_item(_patch(pool, imgs, p), flip, angle, z)
        assert np.array_equal(clean[k].cpu().numpy(), rc), k
        d = np.abs(noisy[k].cpu().numpy() - rn)
        assert d.max() <= 2.0 / 255 + 1e-6, k
        diff_total += int((d > 0).sum())
        n_total += d.size
    assert diff_total <= 1e-4 * n_total, diff_total
    # noise statistics on unclipped mid-range pixels: std ~ sigma/255*2 in [-1, 1]
    resid = (noisy - clean)[clean.abs() < 0.5]
    assert abs(resid.mean().item()) < 0.01


def test_synth_paired_pool():
    from vub_image_denoising_amd.synth import synth_batch
    rng = np.random.default_rng(9)
    pool, imgs, noisy_imgs = _pool(rng, [(130, 200)], P=64, paired=True)
    items, params = _items(pool, rng, 5)
    noisy, clean = synth_batch(pool, items)
    torch.cuda.synchronize()
    for k, (p, flip, angle, sigma, seed) in enumerate(params):
        rn, rc = S.synth_item(_patch(pool, imgs, p), flip, angle, noisy_u8=_patch(pool, noisy_imgs, p))
        assert np.array_equal(clean[k].cpu().numpy(), rc) and np.array_equal(noisy[k].cpu().numpy(), rn), k


def test_load_data_gpu_end_to_end(tmp_path):
    """load_data_gpu on an image folder: split sizes, device batches, and without
    augmentation the clean side equals the CPU loader's clean item for that index."""
    from PIL import Image
    from vub_image_denoising_amd.data_loader import CustomDataset
    from vub_image_denoising_amd.synth import load_data_gpu
    rng = np.random.default_rng(11)
    for k in range(3):
        Image.fromarray(rng.integers(0, 256, (140, 260, 3), dtype=np.uint8)).save(tmp_path / f"{k}.png")
    tr, va = load_data_gpu(str(tmp_path), batch_size=4, validation_split=0.25, use_rgb=True, patch_size=128,
                           train_noise_levels=[25])
    assert len(tr.dataset) + len(va.dataset) == 6
    cpu = CustomDataset(str(tmp_path), use_rgb=True, noise_levels=[25], patch_size=128)
    seen = 0
    for noisy, clean in tr:
        assert noisy.is_cuda and noisy.shape[1:] == (3, 128, 128)
        seen += noisy.shape[0]
    assert seen == len(tr.dataset)
    idx = va.indices[0]
    noisy, clean = next(iter(va))
    assert torch.equal(clean[0].cpu(), cpu[idx][1])
    trs, vas = load_data_gpu(str(tmp_path), batch_size=2, augment=True, use_rgb=True, patch_size=128)
    n, c = next(iter(trs))
    assert n.shape == (2, 3, 128, 128) and float(c.min()) >= -1 and float(c.max()) <= 1
