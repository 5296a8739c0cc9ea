#!/bin/bash
# GPU suite under env arm "$1", then interleaved step A/B default vs "$1" (3 rounds) with per-layer tables
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
env $1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/ab6_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ab6_t.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab6.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 --layer-report gpurun_out/ab6_lay_a.json > gpurun_out/ab6_a.json 2>/dev/null || exit 1
  echo "A $(python -c 'import json;print(json.load(open("gpurun_out/ab6_a.json"))["value"])')" >> gpurun_out/ab6.log
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 --layer-report gpurun_out/ab6_lay_b.json > gpurun_out/ab6_b.json 2>/dev/null || exit 1
  echo "B $(python -c 'import json;print(json.load(open("gpurun_out/ab6_b.json"))["value"])')" >> gpurun_out/ab6.log
done
