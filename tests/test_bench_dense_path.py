"""bench.py's dense-conv-path roofline (the north_star's level-0/1 residual-dense convs,
Sigma algorithmic bytes / Sigma isolated kernel time / 8 TB/s) and its median over
profiling passes (verdict r04 item 2): only block_0_* / block_1_* conv launches count,
the PReLU passes and the other levels do not, and the median pass is reported with the
spread of all passes.  CPU only (fake event pairs)."""
import types

import bench


class _Ev:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def _prof(ms_per_launch):
    recs = []
    for name, phase, nbytes, ms in [("block_0_0.conv_0-2", "fwd", 4e8, 0.09), ("block_0_0.conv_3", "dwgrad", 5e8, 0.14),
                                    ("block_1_0.conv_3", "fwd", 2e8, 0.06), ("block_1_0.conv_3", "prelu", 9e8, 0.5),
                                    ("block_2_0.conv_3", "fwd", 9e8, 0.5), ("up_0.conv", "fwd", 9e8, 0.5)]:
        scale = ms_per_launch if name.startswith(("block_0", "block_1")) and phase != "prelu" else 1.0
        recs.append(((phase, name, "k", 0, nbytes, nbytes * 0.9), _Ev(0.0), _Ev(ms * scale)))
    return types.SimpleNamespace(records=recs)


def test_dense_path_counts_level01_convs_only():
    r = bench.dense_conv_path(_prof(1.0), 16)
    assert r["launches"] == 3
    assert abs(r["bytes_per_step_gb"] - 1.1) < 1e-9
    assert abs(r["kernel_ms_per_step"] - 0.29) < 1e-9
    assert abs(r["frac"] - round(1.1e9 / 0.29e-3 / 1e9 / bench.PEAK_HBM_GBS, 4)) < 1e-9


def test_dense_path_median_of_passes():
    profs = [_prof(1.0), _prof(1.2), _prof(0.9)]
    r = bench.dense_conv_path_median(profs, 32)
    fr = sorted(bench.dense_conv_path(p, 32)["frac"] for p in profs)
    assert r["passes"] == 3 and r["frac"] == fr[1]
    assert r["frac_min"] == fr[0] and r["frac_max"] == fr[2] and r["frac_all"] == fr
