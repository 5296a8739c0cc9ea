#!/bin/bash
# interleaved step A/B of environment settings: VARIANTS="A=...;B=..." (each a list of
# VAR=value, space separated), ROUNDS rounds, B16 (and B32 with B32=1); OUT dir under gpurun_out
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-ab}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
IFS=';' read -ra VS <<< "$VARIANTS"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    name=${v%%=*}; envs=${v#*=}
    for b in 16 ${B32:+32}; do
      env $envs timeout -k 10 150 python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 > gpurun_out/$OUT/${name}_b${b}_$r.json 2>/dev/null || exit $?
      python -c "import json;d=json.load(open('gpurun_out/$OUT/${name}_b${b}_$r.json'));print('$name b$b r$r', d['value'], d['ms_per_step'])" >> gpurun_out/$OUT/summary.txt
    done
  done
done
cat gpurun_out/$OUT/summary.txt
