#!/bin/bash
# full GPU suite, then rocprofv3 kernel stats of a short bench (train step only)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-x}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 10 --warmup 3 > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
