#!/bin/bash
# one iteration: new tests first, GPU suite (no PSNR experiment), B16/B32 bench lines
# with layer reports, then a kernel trace of the B16 step (OUT=dir under gpurun_out)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-it}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
if [ -n "$FIRST" ]; then
  timeout -k 10 300 python -u -m pytest $FIRST -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$OUT/first.log 2>&1
  rc=$?; echo "first rc=$rc" >> gpurun_out/$OUT/first.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOSUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -k "not psnr" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1
  rc=$?; echo "tests rc=$rc" >> gpurun_out/$OUT/t.log; [ $rc -eq 0 ] || exit $rc
fi
for b in ${BATCHES:-16 32}; do
  timeout -k 10 150 python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 --layer-report gpurun_out/$OUT/b${b}.layers.json > gpurun_out/$OUT/b${b}.json 2>/dev/null || exit $?
done
if [ -z "$NOTRACE" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/$OUT/trace -o run --output-format csv -- python3 bench.py --batch 16 --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/$OUT/trace.json 2> gpurun_out/$OUT/trace.err || exit $?
fi
