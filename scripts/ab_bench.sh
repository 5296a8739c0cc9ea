#!/bin/bash
# interleaved A/B of bench.py: in-tree library vs build/var/$1 (RDN_LIB), N rounds
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=build/var/$1; N=${2:-2}
: > gpurun_out/ab.log
for i in $(seq $N); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --steps 30 > gpurun_out/ab_a.json 2>/dev/null || exit 1
  echo "A $(python -c 'import json;print(json.load(open("gpurun_out/ab_a.json"))["value"])')" >> gpurun_out/ab.log
  RDN_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --steps 30 > gpurun_out/ab_b.json 2>/dev/null || exit 1
  echo "B $(python -c 'import json;print(json.load(open("gpurun_out/ab_b.json"))["value"])')" >> gpurun_out/ab.log
done
