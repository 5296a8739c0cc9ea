#!/bin/bash
# interleaved step A/B, 3 rounds: default build vs env arm "$1" (e.g. 'RDN_CONV3_WSD=0 RDN_WGLDS=m')
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/ab4.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 > gpurun_out/ab4_a.json 2>/dev/null || exit 1
  echo "A $(python -c 'import json;print(json.load(open("gpurun_out/ab4_a.json"))["value"])')" >> gpurun_out/ab4.log
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 > gpurun_out/ab4_b.json 2>/dev/null || exit 1
  echo "B $(python -c 'import json;print(json.load(open("gpurun_out/ab4_b.json"))["value"])')" >> gpurun_out/ab4.log
done
