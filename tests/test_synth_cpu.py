"""CPU checks of the data-synthesis path:

* the oracle's rotation (oracle/synth_ref.py) against Pillow's own Image.rotate —
  the call torchvision 0.18's RandomRotation(10) makes on PIL images
  (data_loader.py:43) — bit for bit;
* the oracle's whole item against the reference pipeline run literally with PIL +
  numpy: custom_dataset.py:84-86 noise, F.hflip / F.rotate on PIL images, ToTensor
  + Normalize restated (torchvision is not installed);
* the host-side item encoding of vub_image_denoising_amd.synth (affine
  coefficients, struct layout);
* the CPU DataLoaders (load_data / load_sidd_data) on small image folders."""
import ctypes
import os

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import synth_ref as S


@pytest.mark.parametrize("P", [16, 64, 256])
@pytest.mark.parametrize("mode", ["RGB", "L"])
def test_rotation_matches_pillow(P, mode):
    rng = np.random.default_rng(P)
    C = 3 if mode == "RGB" else 1
    img = rng.integers(0, 256, (P, P, C), dtype=np.uint8)
    pil = Image.fromarray(img if C == 3 else img[:, :, 0], mode)
    for ang in (-10.0, -9.97, -7.3, -0.4, -1e-3, 0.3, 2.5, 5.5, 9.99, 10.0):
        ref = np.array(pil.rotate(ang, Image.NEAREST, expand=False, center=None, fillcolor=0))
        if C == 1:
            ref = ref[:, :, None]
        assert np.array_equal(S.rotate_nearest(img, ang), ref), (P, mode, ang)


def _reference_item(patch, noise, flip, angle):
    """dataset_creation/custom_dataset.py:80-95 with data_loader.py:41-46's transform,
    run with the libraries the reference uses (PIL, numpy)."""
    gt_patch = Image.fromarray(patch)
    noisy_patch = np.array(gt_patch, dtype=np.float32)
    noisy_patch += noise
    noisy_patch = np.clip(noisy_patch, 0, 255).astype(np.uint8)
    noisy_patch = Image.fromarray(noisy_patch)
    out = []
    for im in (gt_patch, noisy_patch):
        if flip:
            im = im.transpose(Image.FLIP_LEFT_RIGHT)                      # F.hflip
        if angle is not None:
            im = im.rotate(angle, Image.NEAREST, False, None, fillcolor=0)  # F.rotate
        t = torch.from_numpy(np.array(im)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)  # ToTensor
        out.append(t.sub_(0.5).div_(0.5).numpy())                          # Normalize
    return out[1], out[0]


def test_oracle_item_matches_reference_pipeline():
    rng = np.random.default_rng(1)
    for flip in (False, True):
        for angle in (None, -6.25, 8.0):
            patch = rng.integers(0, 256, (48, 48, 3), dtype=np.uint8)
            noise = rng.normal(scale=25, size=patch.shape)
            rn, rc = _reference_item(patch, noise, flip, angle)
            on, oc = S.synth_item(patch, flip, angle, noise)
            assert np.array_equal(on, rn) and np.array_equal(oc, rc), (flip, angle)


def test_device_noise_stream_statistics():
    z = S.device_normal(12345, 1 << 18)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert not np.array_equal(z[:100], S.device_normal(12346, 100))


def test_host_item_encoding():
    from vub_image_denoising_amd import _hip as H
    from vub_image_denoising_amd import synth
    assert synth.ITEM_DTYPE.itemsize == ctypes.sizeof(H.SynthItem) == 64
    for name, _ in H.SynthItem._fields_:
        assert synth.ITEM_DTYPE.fields[name][1] == getattr(H.SynthItem, name).offset, name
    for ang in (-10.0, -3.3, 0.7, 9.5):
        assert synth.rotate_coeffs(ang, 256, 256) == S.rotate_coeffs(ang, 256, 256)
    assert synth.rotate_coeffs(0.0, 256, 256) is None


def _write_images(folder, sizes, rng, prefix=""):
    os.makedirs(folder, exist_ok=True)
    arrs = []
    for k, (h, w) in enumerate(sizes):
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        Image.fromarray(a).save(os.path.join(folder, f"{prefix}{k:03d}.png"))
        arrs.append(a)
    return arrs


def test_cpu_load_data_patches_and_noise_levels(tmp_path):
    """data_loader.py:7-79 / custom_dataset.py:44-100: non-overlapping patches x noise
    levels, (noisy, clean) in [-1, 1], the clean item equal to the crop."""
    from vub_image_denoising_amd.data_loader import CustomDataset, load_data
    rng = np.random.default_rng(2)
    arrs = _write_images(tmp_path / "imgs", [(300, 520), (256, 256)], rng)
    ds = CustomDataset(str(tmp_path / "imgs"), use_rgb=True)
    assert len(ds.patch_pairs) == 2 + 1 and len(ds) == 3 * 3
    noisy, clean = ds[4]                                  # patch 1, sigma 25
    assert noisy.shape == clean.shape == (3, 256, 256)
    ref = torch.from_numpy(S.to_unit(arrs[0][:256, 256:512]))
    assert torch.equal(clean, ref)
    assert 0.05 < (noisy - clean).std().item() < 0.3
    tr, va = load_data(str(tmp_path / "imgs"), batch_size=2, num_workers=0, validation_split=0.34, use_rgb=True)
    assert len(tr.dataset) + len(va.dataset) == 9
    n, c = next(iter(tr))
    assert n.shape == (2, 3, 256, 256) and c.min() >= -1 and c.max() <= 1


def test_cpu_load_sidd_data(tmp_path):
    """SIDD_dataset.py:10-168: Scene_Instances.txt -> Data/<scene>/{NOISY,GT} pairs,
    non-overlapping 256x256 patches, no synthetic noise."""
    from vub_image_denoising_amd.data_loader import CustomSIDD_Dataset, load_sidd_data
    rng = np.random.default_rng(3)
    root = tmp_path / "SIDD"
    scenes = ["0001_001_S6_00100_00060_3200_L", "0002_001_S6_00100_00020_3200_N"]
    (root / "Data").mkdir(parents=True)
    (root / "Scene_Instances.txt").write_text("\n".join(scenes) + "\n")
    gts = {}
    for s in scenes:
        d = root / "Data" / s
        gt = _write_images(d, [(300, 512)], rng, prefix="GT_SRGB_")[0]
        _write_images(d, [(300, 512)], rng, prefix="NOISY_SRGB_")
        gts[s] = gt
    ds = CustomSIDD_Dataset(str(root), use_rgb=True)
    assert len(ds) == 4
    noisy, gt = ds[1]
    assert torch.equal(gt, torch.from_numpy(S.to_unit(gts[scenes[0]][:256, 256:512])))
    tr, va = load_sidd_data(str(root), batch_size=2, num_workers=0, validation_split=0.5, use_rgb=True)
    assert len(tr.dataset) == 2 and len(va.dataset) == 2


def test_mixed_patch_loader_alternates():
    """Config 5's stream: batches taken from each patch-size loader in turn until all
    are exhausted (synth.MixedPatchLoader)."""
    from vub_image_denoising_amd.synth import MixedPatchLoader

    class L:
        def __init__(self, tag, n):
            self.tag, self.n, self.batch_size, self.dataset = tag, n, 2, list(range(2 * n))

        def __len__(self):
            return self.n

        def __iter__(self):
            return iter([(self.tag, i) for i in range(self.n)])

    m = MixedPatchLoader([L(128, 3), L(256, 1)])
    assert len(m) == 4 and len(m.dataset) == 8
    assert list(m) == [(128, 0), (256, 0), (128, 1), (128, 2)]
