#!/bin/bash
# wgrad rows accumulator budget: parity under each setting, then interleaved bench A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for E in "RDN_WROWS_MAXACC=4096" "RDN_WROWS_MAXACC=4096 RDN_WROWS_BM=128"; do
  env $E timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_network.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wrows.log 2>&1
  rc=$?; echo "[$E] tests rc=$rc" >> gpurun_out/ab_tests.log; tail -3 gpurun_out/t_wrows.log >> gpurun_out/ab_tests.log
  [ $rc -eq 0 ] || exit $rc
done
bash scripts/ab_multi.sh "-" "RDN_WROWS_MAXACC=4096" "RDN_WROWS_MAXACC=4096 RDN_WROWS_BM=128"
