#!/bin/bash
# interleaved A/B of bench.py under two environment settings: ab_env.sh "A=1" "A=2" [rounds]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
EA=$1; EB=$2; N=${3:-2}
echo "--- $EA vs $EB" >> gpurun_out/ab.log
for i in $(seq $N); do
  env $EA timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --steps 30 > gpurun_out/ab_a.json 2>/dev/null || exit 1
  echo "A[$EA] $(python -c 'import json;print(json.load(open("gpurun_out/ab_a.json"))["value"])')" >> gpurun_out/ab.log
  env $EB timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --steps 30 > gpurun_out/ab_b.json 2>/dev/null || exit 1
  echo "B[$EB] $(python -c 'import json;print(json.load(open("gpurun_out/ab_b.json"))["value"])')" >> gpurun_out/ab.log
done
