#!/bin/bash
# A/B of an env knob ($1) between values $2 and $3: GPU tests first, then wgrad+conv micro-bench and step, per-layer tables
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; A=$2; B=$3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/ab3_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ab3_t.log; [ $rc -eq 0 ] || exit $rc
for v in $A $B; do
  env $VAR=$v KB_CONV=0 timeout -k 10 150 python scripts/kbench.py > gpurun_out/ab3_kb_$v.log 2>&1 || exit 1
done
for i in 1 2; do for v in $A $B; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 30 --layer-report gpurun_out/ab3_lay_$v.json > gpurun_out/ab3_b_$v.$i.json 2>gpurun_out/ab3_b.err || exit 1
done; done
