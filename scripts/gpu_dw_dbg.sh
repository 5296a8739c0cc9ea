#!/bin/bash
# where the fused level-0 kernel's time goes: layer report with parts of it switched off
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 0 1 2 3 4 7; do
  RDN_DW_DBG=$m timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --graph off --steps 3 --warmup 2 --layer-report gpurun_out/dbg_$m.json > gpurun_out/dbg_$m.out 2>&1 || exit $?
done
