#!/bin/bash
# quick GPU check: selected test files (TESTS), then B16 + B32 train-step lines with
# per-layer reports (OUT=dir under gpurun_out).  Each step under its own limit.
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-check}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> gpurun_out/$OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$NO_BENCH" ] && exit 0
for b in ${BATCHES:-16 32}; do
  timeout -k 10 200 python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 --layer-report gpurun_out/$OUT/b${b}.layers.json > gpurun_out/$OUT/b${b}.json 2>gpurun_out/$OUT/b${b}.err || exit $?
done
