#!/bin/bash
# round-2 baseline: B=32 bf16 and B=16 fp32 train-step benches with per-layer reports
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --batch 32 --no-cpu-baseline --no-inference --no-traffic --layer-report gpurun_out/b32_layers.json > gpurun_out/b32.json 2> gpurun_out/b32.err
rc=$?; echo "b32 rc=$rc" >> gpurun_out/b32.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dtype fp32 --no-cpu-baseline --no-inference --no-traffic --steps 10 --warmup 3 > gpurun_out/f32.json 2> gpurun_out/f32.err
rc=$?; echo "f32 rc=$rc" >> gpurun_out/f32.err; exit $rc
