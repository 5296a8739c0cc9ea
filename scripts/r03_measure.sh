#!/bin/bash
# round-3 measurement: GPU tests -> bench (full JSON line + layer report)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --layer-report gpurun_out/layers.json > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err; exit $rc
