#!/bin/bash
# one measurement round: GPU suite (minus the PSNR experiment), per-layer conv3_big vs conv3_halo, B16 + B32 step with layer reports (OUT=dir under gpurun_out)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-step}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -k "not psnr" -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/$OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/big_plans.py gpurun_out/$OUT/plans.json > gpurun_out/$OUT/plans.log 2>&1 || exit $?
for b in 16 32; do
  timeout -k 10 150 python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 --layer-report gpurun_out/$OUT/b${b}.layers.json > gpurun_out/$OUT/b${b}.json 2>/dev/null || exit $?
done
