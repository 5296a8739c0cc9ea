#!/bin/bash
# the driver's default bench command, timed, plus stderr
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s" >> gpurun_out/bench.err; exit $rc
