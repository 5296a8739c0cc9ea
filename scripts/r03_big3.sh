#!/bin/bash
# conv3_big with its dispatch rule: parity tests, per-layer timing vs conv3_halo, step A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/big3; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_big.py -m gpu -x -v -s --timeout 60 --timeout-method thread > gpurun_out/big3/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/big3/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/big_plans.py gpurun_out/big3/plans.json > gpurun_out/big3/plans.log 2>&1 || exit $?
for r in 1 2; do
  for b in 16 32; do
    B="python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5"
    timeout -k 10 150 $B > gpurun_out/big3/big_b${b}_$r.json 2>/dev/null || exit $?
    RDN_BIG=0 timeout -k 10 150 $B > gpurun_out/big3/halo_b${b}_$r.json 2>/dev/null || exit $?
  done
done
