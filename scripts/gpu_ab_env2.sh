#!/bin/bash
# tests subset, then A/B of env settings (VARS, one per run, interleaved twice)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do for v in $VARS; do
tag=$(echo $v | tr '=,' '__')
env $(echo $v | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --batch ${BATCH:-16} --layer-report gpurun_out/ab_${tag}_layers.json > gpurun_out/ab_${tag}.json 2> gpurun_out/ab_${tag}.err || exit 1
echo "$v rep$rep $(python -c "import json;d=json.load(open('gpurun_out/ab_${tag}.json'));print(d['value'], d['roofline']['dense_conv_path_b${BATCH:-16}']['achieved'])")"
done; done
