#!/bin/bash
# interleaved step runs over several env arms (3 rounds): bash scripts/gpu_ab7.sh "ARM1" "ARM2" ...  ("-" = default)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/ab7.log
for i in 1 2 3; do
  for arm in "$@"; do
    e=$arm; [ "$e" = "-" ] && e="RDN_DUMMY=1"
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 > gpurun_out/ab7_x.json 2>/dev/null || exit 1
    echo "$arm $(python -c 'import json;print(json.load(open("gpurun_out/ab7_x.json"))["value"])')" >> gpurun_out/ab7.log
  done
done
