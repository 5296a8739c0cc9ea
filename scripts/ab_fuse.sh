#!/bin/bash
cd "$GRAFT_REPO_ROOT"
run() { echo "=== $1" >> gpurun_out/ab.log; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --layer-report gpurun_out/lay_$RANDOM.json >> gpurun_out/ab.log 2>&1 || exit 1; }
run "wide+fuse" RDN_FUSE_PRELU=1
run "wide nofuse" RDN_FUSE_PRELU=0
run "nowide+fuse" RDN_FUSE_PRELU=1 RDN_LIB=build/var/lib_nowide.so
run "nowide nofuse" RDN_FUSE_PRELU=0 RDN_LIB=build/var/lib_nowide.so
