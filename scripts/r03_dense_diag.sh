#!/bin/bash
# per-layer report of the fused level-0 launch for the in-tree library and diagnostic builds
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-dd}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
for v in base ${VS}; do
  lib=""; [ $v != base ] && lib="RDN_LIB=build/variants/lib_$v.so"
  env $lib timeout -k 10 150 python bench.py --batch 16 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 5 --warmup 3 --layer-report gpurun_out/$OUT/$v.layers.json > gpurun_out/$OUT/$v.json 2>/dev/null || exit $?
  python -c "import json;pl=json.load(open('gpurun_out/$OUT/$v.layers_per_layer.json'));print('$v', [round(x['us'],1) for x in pl if 'conv_0-2' in x['layer']])" >> gpurun_out/$OUT/summary.txt
done
cat gpurun_out/$OUT/summary.txt
