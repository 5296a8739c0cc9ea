#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the conv micro-bench
# launches (scripts/kbench.py), per dispatch, under gpurun_out/pmct/pN
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmct; export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmct/p$i -o run --output-format csv -- python3 scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so > gpurun_out/pmct/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" >> gpurun_out/pmct/p$i.log
  [ $rc -eq 0 ] || exit $rc
done
