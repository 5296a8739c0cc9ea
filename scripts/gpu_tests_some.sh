#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_planar.py tests/test_gpu_network.py tests/test_gpu_dw.py -q --timeout 120 --timeout-method thread > gpurun_out/ts.log 2>&1
echo "rc=$?" >> gpurun_out/ts.log
