"""bench.py's multi-GPU launcher (config 3: `python bench.py --gpus N` must run N
ranks, one process per GPU, exactly like `torchrun --nproc-per-node N`).  The
dry-run mode stops every rank before it touches the GPU, so this runs on the CPU."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "RDN_BENCH_LAUNCHED"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], env=e, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def _lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_gpus_n_starts_n_ranks():
    r = _bench("--gpus", "2", "--launch-dry-run")
    assert r.returncode == 0, r.stderr
    ranks = sorted(_lines(r.stdout), key=lambda d: d["rank"])
    assert [d["rank"] for d in ranks] == [0, 1]
    assert [d["local_rank"] for d in ranks] == [0, 1]
    assert all(d["world_size"] == 2 and d["master_addr"] == "127.0.0.1" and d["launched_by"] == "bench.py"
               for d in ranks)
    assert len({d["master_port"] for d in ranks}) == 1


def test_four_ranks():
    r = _bench("--gpus", "4", "--launch-dry-run")
    assert r.returncode == 0, r.stderr
    assert sorted(d["rank"] for d in _lines(r.stdout)) == [0, 1, 2, 3]


def test_single_gpu_runs_in_process():
    r = _bench("--gpus", "1", "--launch-dry-run")
    assert r.returncode == 0, r.stderr
    (d,) = _lines(r.stdout)
    assert d["world_size"] == 1 and d["launched_by"] == "external"


def test_world_size_mismatch_is_refused():
    r = _bench("--gpus", "8", "--launch-dry-run", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_external_launcher_environment_is_used():
    r = _bench("--gpus", "2", "--launch-dry-run", env={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1",
                                                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29555"})
    assert r.returncode == 0, r.stderr
    (d,) = _lines(r.stdout)
    assert d == {"rank": 1, "local_rank": 1, "world_size": 2, "graph": "on", "master_addr": "127.0.0.1",
                 "master_port": "29555", "launched_by": "external"}


def test_graph_capture_failure_restarts_eagerly():
    """A rank whose RCCL-step capture raises exits with EXIT_GRAPH_FAILED; the
    launcher starts the job again from fresh processes with --graph off."""
    r = _bench("--gpus", "2", "--launch-dry-run", env={"RDN_BENCH_DRY_GRAPH_FAIL": "1"})
    assert r.returncode == 0, r.stderr
    ranks = _lines(r.stdout)
    assert sorted(d["rank"] for d in ranks) == [0, 1]
    assert all(d["graph"] == "off" for d in ranks)
    assert "running the job again eagerly" in r.stderr


def test_deadline_kills_a_hung_rank():
    """Every rank hung in a collective must not hang the caller: past --deadline-s the
    launcher kills the ranks still running and exits with EXIT_DEADLINE (124)."""
    t0 = time.monotonic()
    r = _bench("--gpus", "2", "--launch-dry-run", "--deadline-s", "4", env={"RDN_BENCH_DRY_HANG": "1"}, timeout=120)
    assert r.returncode == 124, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 60
    assert "deadline of 4 s passed with rank(s) [1]" in r.stderr
    assert [d["rank"] for d in _lines(r.stdout)] == [0]   # (rank 0 finished normally)


def test_watchdog_ends_a_hung_rank_under_an_external_launcher():
    """Under torchrun the bench's launcher is not there: the rank's own watchdog
    thread ends the process with 124 at the deadline."""
    t0 = time.monotonic()
    r = _bench("--gpus", "2", "--launch-dry-run", "--deadline-s", "3",
               env={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1", "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": "29556", "RDN_BENCH_DRY_HANG": "1"}, timeout=120)
    assert r.returncode == 124, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 60
    assert "deadline of 3 s passed" in r.stderr
