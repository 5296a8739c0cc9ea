"""Config 5's mixed patch sizes (synth.load_data_gpu / load_sidd_data_gpu with
patch_size=(128, 256)): the train / validation split is made once, over cells of
the largest patch grid, so no validation patch of one size shares a pixel with a
training patch of another (advisor r04: the per-size index splits leaked ~80 % of
the 128-pixel validation patches into the 256-pixel training stream).  The loaders
are only built here (no GPU: nothing is synthesised)."""
import numpy as np

from vub_image_denoising_amd.synth import load_data_gpu


def _images():
    rng = np.random.default_rng(0)
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in ((640, 896), (512, 512), (384, 768))]


def _rects(loader):
    pool, L = loader.pool, len(loader.levels)
    out = set()
    for i in loader.indices:
        k, top, left = pool.patches[i // L]
        out.add((k, top, left, pool.patch_size))
    return out


def _overlap(a, b):
    (k1, t1, l1, p1), (k2, t2, l2, p2) = a, b
    return k1 == k2 and t1 < t2 + p2 and t2 < t1 + p1 and l1 < l2 + p2 and l2 < l1 + p1


def test_mixed_sizes_split_without_overlap():
    tr, va = load_data_gpu(None, batch_size=2, validation_split=0.25, images=_images(), patch_size=(128, 256),
                           seed=3, device="cpu")
    tr_r = set().union(*(_rects(ld) for ld in tr.loaders))
    va_r = set().union(*(_rects(ld) for ld in va.loaders))
    assert tr_r and va_r
    assert not any(_overlap(a, b) for a in va_r for b in tr_r)
    # every patch of both grids is used exactly once (no subset: dataset_percentage 1.0)
    for t_ld, v_ld in zip(tr.loaders, va.loaders):
        n = len(t_ld.pool) * len(t_ld.levels)
        assert sorted(t_ld.indices + v_ld.indices) == list(range(n))
    # roughly the requested fraction of cells goes to validation
    frac = len(va.loaders[1].indices) / (len(va.loaders[1].indices) + len(tr.loaders[1].indices))
    assert 0.1 < frac < 0.45, frac


def test_single_size_split_unchanged():
    """One patch size keeps the reference's item-level split (data_loader.py:63-74)."""
    tr, va = load_data_gpu(None, batch_size=2, validation_split=0.25, images=_images(), patch_size=256, seed=3,
                           device="cpu")
    n = len(tr.pool) * 3
    assert len(tr.indices) == int(0.75 * n) and len(tr.indices) + len(va.indices) == n
