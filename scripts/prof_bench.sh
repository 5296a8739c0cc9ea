#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run -> gpurun_out/prof
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
