#!/bin/bash
# Round measurement on one GPU box: the GPU suite, the full bench line (with its PMC
# traffic passes, per-layer report) and a rocprofv3 kernel-trace summary of the timed
# train step.  OUT = directory under gpurun_out.  Every step under its own time limit;
# the first failure ends the script.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${OUT:-measure}; mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  RDN_TEST_OUT=$OUT timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
fi
timeout -k 10 600 python -u bench.py --layer-report $OUT/layers.json > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 20 > $OUT/prof.log 2>&1 || exit $?
