#!/bin/bash
# interleaved bench.py runs under several environment settings (2 rounds):
# scripts/ab_multi.sh "RDN_X=0" "RDN_X=1" ...   (a setting "-" = default env)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/ab.log
for i in 1 2; do
  for E in "$@"; do
    EE=$E; [ "$E" = "-" ] && EE="RDN_NOP=1"
    env $EE timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --steps 30 > gpurun_out/ab_x.json 2>gpurun_out/ab_x.err || exit 1
    echo "[$E] $(python -c 'import json;print(json.load(open("gpurun_out/ab_x.json"))["value"])')" >> gpurun_out/ab.log
  done
done
