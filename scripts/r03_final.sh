#!/bin/bash
# round-end measurement: GPU suite (all -m gpu tests), the full bench line (B16 headline,
# B32 / fp32 lines, PMC traffic, CPU baseline, samplers) with its per-layer report, then
# rocprofv3 kernel-trace stats of the B16 train-step bench (OUT dir under gpurun_out)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-final}; mkdir -p gpurun_out/$OUT/prof; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/$OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --layer-report gpurun_out/$OUT/layers.json > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/$OUT/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err
rc=$?; echo "prof rc=$rc" >> gpurun_out/$OUT/prof.err; exit $rc
