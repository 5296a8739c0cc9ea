#!/bin/bash
# PMC passes over a short train-step run: per-kernel HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) and SQ wait counters
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PMC_OUT=gpurun_out/pmc bash scripts/pmc.sh python3 bench.py --pmc-child --no-cpu-baseline --no-extra --no-inference --no-traffic --steps 2 --warmup 1
