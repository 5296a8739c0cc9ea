#!/bin/bash
# GPU suite, then per-layer A/B of conv3_ws one vs two halo tiles in flight
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 20 --warmup 5"
timeout -k 10 200 $B --layer-report gpurun_out/ab_def.json > gpurun_out/ab_def.out 2>&1 || exit $?
RDN_WS_DEPTH=0 timeout -k 10 200 $B --layer-report gpurun_out/ab_d2.json > gpurun_out/ab_d2.out 2>&1 || exit $?
timeout -k 10 200 $B > gpurun_out/ab_def2.out 2>&1 || exit $?
RDN_WS_DEPTH=0 timeout -k 10 200 $B > gpurun_out/ab_d22.out 2>&1 || exit $?
