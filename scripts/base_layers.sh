#!/bin/bash
# B16 + B32 train-step lines with per-layer reports (OUT=dir under gpurun_out); no tests
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-base}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
for b in 16 32; do
  timeout -k 10 200 python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 --layer-report gpurun_out/$OUT/b${b}.layers.json > gpurun_out/$OUT/b${b}.json 2>gpurun_out/$OUT/b${b}.err || exit $?
done
