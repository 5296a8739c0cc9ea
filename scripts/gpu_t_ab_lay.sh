#!/bin/bash
# GPU tests -> interleaved env A/B (scripts/ab_multi.sh args) -> layer report at default env
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_multi.sh "$@" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --layer-report gpurun_out/layers.json > gpurun_out/bench.json 2> gpurun_out/bench.err
