"""Data-parallel gradient sync (vub_image_denoising_amd/ddp.py) with world_size 2
over gloo on the CPU: bucket planning, completion-driven launch order, averaging."""
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vub_image_denoising_amd.ddp import GradSync, plan_buckets


def _fake_flat(seed, sizes):
    g = torch.Generator().manual_seed(seed)
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + 63) // 64 * 64
    params = [torch.zeros(n) for n in sizes]
    gflat = torch.zeros(o)
    for p, off in zip(params, offs):
        gflat[off:off + p.numel()] = torch.randn(p.numel(), generator=g)
    return types.SimpleNamespace(params=params, offsets=offs, numel=o, gflat=gflat,
                                 names=[f"p{i}" for i in range(len(sizes))])


SIZES = [4608, 16, 16, 72000, 32, 32, 16, 300000, 128, 128, 5, 900000, 64]


def test_plan_buckets_cover_everything_once():
    fp = _fake_flat(0, SIZES)
    b = plan_buckets(SIZES, fp.offsets, 100000)
    covered = []
    hi_prev = None
    for lo, hi, first in b:
        hi = fp.numel if hi is None else hi
        if hi_prev is not None:
            assert hi == hi_prev  # contiguous, filled from the end
        covered.append((lo, hi))
        hi_prev = lo
    assert covered[0][1] == fp.numel and covered[-1][0] == 0
    # a parameter larger than the bucket size gets a bucket of its own
    assert any(hi - lo >= 900000 for lo, hi in covered)


def test_plan_buckets_small_tail():
    """The start of the flat buffer (completes last) gets a small bucket of its own."""
    fp = _fake_flat(0, SIZES)
    b0 = plan_buckets(SIZES, fp.offsets, 1000000)
    b = plan_buckets(SIZES, fp.offsets, 1000000, tail_elems=80000)
    assert len(b) == len(b0) + 1
    hi_prev = None
    for lo, hi, first in b:
        hi = fp.numel if hi is None else hi
        assert hi_prev is None or hi == hi_prev
        assert lo == fp.offsets[first]
        hi_prev = lo
    assert b[-1][0] == 0 and 0 < b[-1][1] <= 80000 and b[-1][1] in fp.offsets


def _worker(rank, world, init_file, q, defer=False, bucket_mb=0.4, tail_mb=4.0):
    # file:// rendezvous: no TCP port to race for between parallel test runs
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        fp = _fake_flat(100 + rank, SIZES)
        mine = fp.gflat.clone()
        gs = GradSync(fp, bucket_mb=bucket_mb, overlap=False, tail_mb=tail_mb)
        if tail_mb < 1.0:   # the start bucket split off small (ddp.plan_buckets tail_elems)
            assert len(gs.buckets) == 3 and gs.buckets[-1][0] == 0, gs.buckets
        gs.defer_average = defer
        gs.begin()
        # backward order: parameters complete from the last to the first, in groups of 3
        idx = list(range(len(SIZES)))[::-1]
        for i in range(0, len(idx), 3):
            gs.params_done(idx[i:i + 3])
        assert all(gs._launched), "every bucket launched once its parameters completed"
        gs.finish()
        if defer:   # the sum is left in place and the 1/world factor handed to the caller
            assert gs.take_pending() == 1.0 / world and gs.take_pending() is None
            fp.gflat.mul_(1.0 / world)
        # numpy arrays travel by value; a torch tensor would be shared through a
        # file descriptor whose socket dies with this process (racy FileNotFoundError)
        q.put((rank, mine.numpy(), fp.gflat.clone().numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("defer,bucket_mb,tail_mb", [(False, 0.4, 4.0), (True, 0.4, 4.0), (False, 4.0, 0.3)],
                         ids=["average", "deferred", "small-tail"])
def test_gradsync_world2_gloo_average(tmp_path, defer, bucket_mb, tail_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init_file = str(tmp_path / "rendezvous")
    procs = [ctx.Process(target=_worker, args=(r, 2, init_file, q, defer, bucket_mb, tail_mb)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(2):
        r, mine, synced = q.get(timeout=120)
        res[r] = (torch.from_numpy(mine), torch.from_numpy(synced))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    avg = (res[0][0] + res[1][0]) / 2
    torch.testing.assert_close(res[0][1], avg)
    torch.testing.assert_close(res[1][1], avg)


def test_capture_drain_refuses_unsafe_nccl_groups(monkeypatch):
    """train_graph._drain_collectives (before capturing an RCCL train step): a torch
    build without ProcessGroupNCCL._wait_for_pending_works, or an NCCL group set up
    without TORCH_NCCL_CUDA_EVENT_CACHE=0, raises GraphCaptureUnsafe instead of
    capturing into a possible watchdog abort (bench.py turns it into the eager path)."""
    import torch.distributed as dist
    from vub_image_denoising_amd import train_graph as TG

    class PG:   # an NCCL group of a torch build without the private drain method
        pass

    class PGDrain:
        drained = 0

        def _wait_for_pending_works(self):
            PGDrain.drained += 1

    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_backend", lambda pg=None: "nccl")
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    monkeypatch.setattr(type(dist.group), "WORLD", property(lambda cls: PG()), raising=False)
    with pytest.raises(TG.GraphCaptureUnsafe, match="_wait_for_pending_works"):
        TG._drain_collectives(None)
    monkeypatch.setattr(type(dist.group), "WORLD", property(lambda cls: PGDrain()), raising=False)
    TG._drain_collectives(None)
    assert PGDrain.drained == 1
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")
    with pytest.raises(TG.GraphCaptureUnsafe, match="TORCH_NCCL_CUDA_EVENT_CACHE"):
        TG._drain_collectives(None)


def test_exposure_from_stamps():
    """bench.py's graph-path exposed all-reduce time from GradSync's replayed stamp
    triples: (comm end - backward end) less the back-to-back stamp gap, floored at 0."""
    from vub_image_denoising_amd.ddp import exposure_from_stamps
    khz = 100_000   # 100 MHz clock: 100 ticks per microsecond
    hidden = (1_000_000, 1_000_300, 1_000_600)        # gap 3 us both ways: nothing exposed
    exposed = (2_000_000, 2_050_300, 2_050_600)       # 503 us to the all-reduce end, 3 us gap
    early = (3_000_000, 3_000_100, 3_000_500)         # a slow stamp launch: floored at 0
    st = exposure_from_stamps([hidden, exposed, early], khz)
    assert st["per_step"] == [0.0, 0.5, 0.0]
    assert st["max"] == 0.5 and abs(st["mean"] - 0.5 / 3) < 1e-4
    assert abs(st["raw_mean"] - (0.003 + 0.503 + 0.001) / 3) < 1e-4
    assert exposure_from_stamps([], khz) is None and exposure_from_stamps([hidden], 0) is None
