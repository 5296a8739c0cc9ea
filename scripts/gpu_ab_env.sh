#!/bin/bash
# A/B of env settings on the bench per-layer report: VARS="A=1 A=2 ..." (one setting per run, interleaved twice)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for v in $VARS; do
tag=$(echo $v | tr '=' '_')
env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --batch ${BATCH:-16} --layer-report gpurun_out/ab_${tag}_layers.json > gpurun_out/ab_${tag}.json 2> gpurun_out/ab_${tag}.err || exit 1
echo "$v rep$rep $(python -c "import json;d=json.load(open('gpurun_out/ab_${tag}.json'));print(d['value'], d['roofline']['dense_conv_path_b${BATCH:-16}']['achieved'])")"
done; done
