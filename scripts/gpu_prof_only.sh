#!/bin/bash
# rocprofv3 kernel stats of the headline (B16 bf16) train-step bench alone
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof.err; exit $rc
