#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -rf > gpurun_out/k.log 2>&1
rc=$?
echo "kernels rc=$rc" >> gpurun_out/k.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_network.py -m gpu -q -rf -s > gpurun_out/n.log 2>&1
rc2=$?
echo "network rc=$rc2" >> gpurun_out/n.log
exit $rc2
