#!/bin/bash
# rocprofv3 kernel trace (per dispatch, csv) of a short B16 (and B32) bench run, for scripts/timeline.py
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/trace; export TMPDIR=/tmp
for b in ${BATCHES:-16 32}; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/trace/b$b -o run --output-format csv -- python3 bench.py --batch $b --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/trace/b$b.json 2> gpurun_out/trace/b$b.err || exit $?
done
