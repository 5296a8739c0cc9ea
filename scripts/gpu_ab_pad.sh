#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_planar.py tests/test_gpu_network.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for pad in 0 2560 0 2560; do
RDN_PLANE_PAD=$pad timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-traffic --layer-report gpurun_out/pad${pad}_layers.json > gpurun_out/pad$pad.json 2> gpurun_out/pad$pad.err || exit 1
echo "pad=$pad $(cut -c1-150 gpurun_out/pad$pad.json)"
done
