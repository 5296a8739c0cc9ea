"""The CPU oracle (oracle/rdunet_ref.py) against the reference's own outputs
(tests/golden/golden_rdunet.npz, made by importing the reference)."""
import numpy as np
import torch

from oracle import rdunet_ref as R
from oracle.weights import make_params


def _params(shapes, seed, prefix=""):
    p = make_params(shapes, seed)
    return {prefix + k: torch.from_numpy(v) for k, v in p.items()}


def _rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def test_param_names_match_reference(golden):
    names = [str(n) for n in golden["ts_names"]]
    shapes = R.param_shapes(16, 4, 3)
    assert names == ["unet." + k for k in shapes.keys()]
    assert len(names) == 207


def test_param_count_f32():
    assert sum(int(np.prod(s)) for s in R.param_shapes(32).values()) == 10_407_142


def test_fwd_rdunet_t16_scalar_t(golden):
    p = _params(R.param_shapes(16), int(golden["fwd16_seed"]))
    with torch.no_grad():
        y = R.rdunet_t_forward(p, torch.from_numpy(golden["fwd16_x"]), torch.from_numpy(golden["fwd16_t"]))
    assert _rel(y.numpy(), golden["fwd16_y"]) < 1e-5


def test_fwd_rdunet_t32_map_t(golden):
    p = _params(R.param_shapes(32), int(golden["fwd32_seed"]))
    with torch.no_grad():
        y = R.rdunet_t_forward(p, torch.from_numpy(golden["fwd32_x"]), torch.from_numpy(golden["fwd32_t"]))
    assert _rel(y.numpy(), golden["fwd32_y"]) < 1e-5


def test_fwd_plain_rdunet64(golden):
    p = _params(R.param_shapes(64, 3, 3), int(golden["plain64_seed"]))
    with torch.no_grad():
        y = R.rdunet_forward(p, torch.from_numpy(golden["plain64_x"]))
    assert _rel(y.numpy(), golden["plain64_y"]) < 1e-5


def test_train_step_loss_and_grads(golden):
    p = _params(R.param_shapes(16), int(golden["ts_seed"]), prefix="unet.")
    loss, _, grads, total = R.train_step(p, torch.from_numpy(golden["ts_clean"]), torch.from_numpy(golden["ts_noisy"]),
                                         torch.from_numpy(golden["ts_t"]), 20, clip_value=1.0, prefix="unet.")
    assert abs(loss.item() - float(golden["ts_loss"])) <= 1e-5 * abs(float(golden["ts_loss"]))
    names = [str(n) for n in golden["ts_names"]]
    gn = np.array([grads[n].norm().item() for n in names])
    np.testing.assert_allclose(gn, golden["ts_gnorm"], rtol=2e-3, atol=1e-9)
    for n in names:
        idx = golden[f"ts_gidx::{n}"]
        g = grads[n].reshape(-1).numpy()[idx]
        ref = golden[f"ts_gval::{n}"]
        assert np.abs(g - ref).max() <= 2e-3 * np.abs(ref).max() + 1e-9, n


def test_improved_and_direct_sampling(golden):
    T = int(golden["samp_T"])
    p = _params(R.param_shapes(16), int(golden["samp_seed"]))
    fn = lambda x, t: R.rdunet_t_forward(p, x, t)
    noisy = torch.from_numpy(golden["samp_noisy"])
    with torch.no_grad():
        ys = R.improved_sampling(fn, noisy, T)
        yd = R.direct_sampling(fn, noisy)
    assert _rel(ys.numpy(), golden["samp_improved"]) < 1e-5
    assert _rel(yd.numpy(), golden["samp_direct"]) < 1e-5
