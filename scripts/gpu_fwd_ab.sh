#!/bin/bash
# per-layer A/B of the level-0/1 forward kernels: default vs conv3_wsd everywhere vs conv3_ws two tiles in flight
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 10 --warmup 3"
timeout -k 10 200 $B --layer-report gpurun_out/ab_def.json > gpurun_out/ab_def.out 2>&1 || exit $?
RDN_CONV3_WSD=all timeout -k 10 200 $B --layer-report gpurun_out/ab_wsd.json > gpurun_out/ab_wsd.out 2>&1 || exit $?
RDN_WS_DEPTH=0 timeout -k 10 200 $B --layer-report gpurun_out/ab_d2.json > gpurun_out/ab_d2.out 2>&1 || exit $?
