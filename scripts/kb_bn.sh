#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for bn in 0 64 128 96 48; do
  echo "=== KB_BN=$bn" >> gpurun_out/kb2.log
  KB_BN=$bn timeout -k 10 200 python scripts/kbench.py build/var/lib_v0.so build/var/lib_lb1.so >> gpurun_out/kb2.log 2>&1 || exit 1
done
