#!/bin/bash
# the test order in which test_gpu_dw failed intermittently (autograd, ddp, dw), three times, then the whole suite
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="tests/test_gpu_autograd.py tests/test_gpu_ddp.py tests/test_gpu_dw.py"
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest $T -q --timeout 120 --timeout-method thread > gpurun_out/fl_$i.log 2>&1; echo "rc=$?" >> gpurun_out/fl_$i.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; echo "tests rc=$?" >> gpurun_out/t.log
