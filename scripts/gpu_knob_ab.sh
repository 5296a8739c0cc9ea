#!/bin/bash
# interleaved step A/B of scheduling knobs after the level-0 fusion
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/knob; export TMPDIR=/tmp
B="python bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5"
for r in 1 2; do
  timeout -k 10 120 $B > gpurun_out/knob/def_$r.out 2>&1 || exit $?
  RDN_DW_REDUCE=main timeout -k 10 120 $B > gpurun_out/knob/redmain_$r.out 2>&1 || exit $?
  RDN_WGLDS_BLOCKS=256 timeout -k 10 120 $B > gpurun_out/knob/glds256_$r.out 2>&1 || exit $?
  RDN_WGLDS_BLOCKS=128 timeout -k 10 120 $B > gpurun_out/knob/glds128_$r.out 2>&1 || exit $?
  RDN_WGRAD_SLOTS=6 timeout -k 10 120 $B > gpurun_out/knob/slots6_$r.out 2>&1 || exit $?
done
