#!/bin/bash
# per-layer isolated times (bench --layer-report) and the B16 step for the in-tree
# library and build/variants/lib_$V.so, interleaved (OUT dir under gpurun_out)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-lab}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
for r in 1 2; do
  for v in base $V; do
    lib=""; [ $v != base ] && lib="RDN_LIB=build/variants/lib_$v.so"
    env $lib timeout -k 10 150 python bench.py --batch 16 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 --layer-report gpurun_out/$OUT/${v}_$r.layers.json > gpurun_out/$OUT/${v}_$r.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('gpurun_out/$OUT/${v}_$r.json'));print('$v r$r', d['value'], d['ms_per_step'])" >> gpurun_out/$OUT/summary.txt
  done
done
cat gpurun_out/$OUT/summary.txt
