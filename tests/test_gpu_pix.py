"""The streaming register-weight GEMM of the 2x2 / stride-2 convolutions (csrc/
conv_pix.hip; Unet_model.py:26-30, 36-42), bf16 -- where it runs: the level-0 down
conv's input gradient (a per-pixel GEMM scattered to 2x2).

It multiplies the same bf16 operands in the same k order with the same MFMA as the
conv_gemm_kernel path it replaces (operands swapped, D = W x^T), so the whole train
step -- output, input gradient and all 207 parameter gradients -- must be bit-identical
to a run with RDN_PIX=0 (the switch is read when the library loads: two child
processes).  Shapes: the train step's 256^2 at B2, and a 48 x 80 image whose 2x2 grids
end in partial 32-pixel groups."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _child(tmp_path, pix, B, Hh, Ww):
    out = str(tmp_path / f"pix{pix}_{B}_{Hh}_{Ww}.npz")
    env = dict(os.environ, RDN_PIX=str(pix))
    subprocess.run([sys.executable, os.path.join(HERE, "_pix_run.py"), out, str(B), str(Hh), str(Ww)],
                   env=env, check=True, timeout=150)
    return np.load(out)


@pytest.mark.parametrize("shape", [(2, 256, 256), (3, 48, 80)])
def test_pix_kernel_bit_identical_to_gemm(tmp_path, shape):
    a = _child(tmp_path, 1, *shape)
    b = _child(tmp_path, 0, *shape)
    ka, kb = [str(k) for k in a["keys"]], [str(k) for k in b["keys"]]
    used = [k for k in ka if k.startswith("conv_pix_kernel")]
    print(f"{shape}: conv_pix instantiations {used}")
    assert used and not any(k.startswith("conv_pix_kernel") for k in kb)
    bad = [n for n in a.files if n != "keys" and not np.array_equal(a[n], b[n])]
    worst = {n: float(np.abs(a[n] - b[n]).max() / (np.abs(b[n]).max() + 1e-30)) for n in bad[:5]}
    assert not bad, f"{len(bad)} tensors differ, e.g. {worst}"
