"""The CPU-oracle PSNR@sigma=25 fixture (tests/golden/psnr_sigma25_oracle.json, made by
tests/golden/make_psnr_oracle.py) is consistent with the generator it names: same
protocol configuration, every seed present once, and the data each seed's PSNR was
measured on regenerates bit for bit here (the noisy-input PSNR of the held-out sets)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import make_psnr_oracle as MK  # noqa: E402
import psnr_parity as PP  # noqa: E402


def test_fixture_matches_generator():
    import argparse
    fx = json.load(open(os.path.join(REPO, "tests", "golden", "psnr_sigma25_oracle.json")))
    assert fx["config"] == MK.CFG
    seeds = [r["seed"] for r in fx["runs"]]
    assert seeds == [MK.SEED0 + MK.SEED_STRIDE * i for i in range(len(seeds))] and len(seeds) >= 130
    gain = np.mean([r["oracle"] - r["noisy"] for r in fx["runs"]])
    assert gain > 3.0, gain     # a model that denoises (north_star PSNR protocol)
    for r in fx["runs"][:: len(seeds) // 3]:
        a = argparse.Namespace(**dict(MK.CFG, seed=r["seed"]))
        data = PP.make_data(a)
        assert abs(PP.psnr_per_image(data[2], data[3]) - r["noisy"]) < 1e-9
        n256, c256 = MK.eval_256(r["seed"])
        assert abs(PP.psnr_per_image(n256, c256) - r["noisy_256"]) < 1e-9
