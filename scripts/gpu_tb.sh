#!/bin/bash
# GPU tests (optionally a subset: $TESTS) -> bench B16 + B32 with per-layer reports
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread $PYARGS > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-traffic --layer-report gpurun_out/b16_layers.json > gpurun_out/b16.json 2> gpurun_out/b16.err
rc=$?; echo "b16 rc=$rc" >> gpurun_out/b16.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 32 --no-cpu-baseline --no-inference --no-traffic --layer-report gpurun_out/b32_layers.json > gpurun_out/b32.json 2> gpurun_out/b32.err
rc=$?; echo "b32 rc=$rc" >> gpurun_out/b32.err; exit $rc
