"""bench.py on the GPU: the eager (--graph off) step at world 1, and the multi-rank
launcher end to end -- `--gpus 2` starting two child ranks that train with
ddp.GradSync (gloo, both ranks on the box's one GPU: RCCL needs one GPU per rank,
the 8-GPU RCCL run is the driver's)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = ["--steps", "2", "--warmup", "1", "--batch", "2", "--size", "64", "--no-extra", "--no-inference",
         "--no-cpu-baseline", "--no-traffic"]


def _bench(*argv, timeout=110):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "RDN_BENCH_LAUNCHED"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv, *SHORT], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return line


def test_bench_eager_world1():
    d = _bench("--gpus", "1", "--graph", "off")
    assert d["n_gpus"] == 1 and d["execution"] == "eager launches"
    assert d["value"] > 0 and d["config"]["parallelism"] == "dp1"


def test_bench_launcher_two_ranks_gloo():
    d = _bench("--gpus", "2", "--one-device", "--dist-backend", "gloo", "--graph", "off")
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4
    assert d["config"]["launcher"] == "bench.py child processes" and d["config"]["dist_backend"] == "gloo"
    assert d["value"] > 0 and d["cpu_baseline"] is None
    # the all-reduce time the backward did not hide, per rank (eager pass of the timed steps)
    ex = d["exposed_allreduce_ms"]
    assert len(ex["per_rank"]) == 2 and all(v is not None and v >= 0 for v in ex["per_rank"]), ex
    assert ex["max"] == max(ex["per_rank"])
