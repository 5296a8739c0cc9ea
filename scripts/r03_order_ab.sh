#!/bin/bash
# interleaved B16/B32 A/B of the ordering edges (RDN_ORDER_EVERY) and a rocprofv3 trace of each
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-oab}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
OUT=$OUT ROUNDS=2 B32=1 VARIANTS="o0=RDN_ORDER_EVERY=0;o12=RDN_ORDER_EVERY=12;o8=RDN_ORDER_EVERY=8" bash scripts/ab_env.sh || exit $?
for v in 0 12; do
  RDN_ORDER_EVERY=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/prof_o$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/$OUT/prof_o$v.json 2> gpurun_out/$OUT/prof_o$v.err || exit $?
done
