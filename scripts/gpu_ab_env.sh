#!/bin/bash
# GPU tests, then interleaved bench A/B of two environment settings
# usage: scripts/gpu_ab_env.sh "A=..." "B=..." [rounds]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab.log
bash scripts/ab_env.sh "$1" "$2" ${3:-2}
