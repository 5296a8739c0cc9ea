#!/bin/bash
# rocprofv3 kernel traces of the B16 step: graph replay with one slot per layer and with
# a 12-slot ring, and eager launches (the bench's live dominant-kernel timing runs eager)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-pm}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
run() {  # name, env..., bench args
  local name=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 $BARGS > gpurun_out/$OUT/$name.json 2> gpurun_out/$OUT/$name.err
}
BARGS="" run graph_all RDN_WGRAD_SLOTS=0 || exit $?
BARGS="" run graph_s12 RDN_WGRAD_SLOTS=12 || exit $?
BARGS="--graph off" run eager_all RDN_WGRAD_SLOTS=0 || exit $?
