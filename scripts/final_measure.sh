#!/bin/bash
# round-end measurement: GPU tests -> full bench (CPU baseline, PMC traffic, samplers,
# layer report) -> rocprofv3 kernel-trace stats of the train-step bench alone
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --layer-report gpurun_out/layers.json > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof.err; exit $rc
