#!/bin/bash
# batch-32 step A/B of the fused layers' reduce stream (interleaved)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/b32ab; export TMPDIR=/tmp
B="python bench.py --batch 32 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 15 --warmup 4"
for r in 1 2; do
  timeout -k 10 150 $B > gpurun_out/b32ab/main_$r.out 2>&1 || exit $?
  RDN_DW_REDUCE=side timeout -k 10 150 $B > gpurun_out/b32ab/side_$r.out 2>&1 || exit $?
done
