#!/bin/bash
# PMC counter passes over a short bench run (one pass per counter set, each alone
# beside --kernel-trace; MI355X_MICROARCH.md slot limits), CSVs under gpurun_out/pmcb/pN
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcb; export TMPDIR=/tmp
i=0
while read -r P; do
  [ -z "$P" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmcb/p$i -o run --output-format csv -- python3 bench.py --pmc-child --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 2 --warmup 1 --batch ${BATCH:-16} > gpurun_out/pmcb/p$i.log 2>&1
  rc=$?; echo "pass $i [$P] rc=$rc" >> gpurun_out/pmcb/passes.log
  [ $rc -eq 0 ] || exit $rc
done <<< "$SETS"
