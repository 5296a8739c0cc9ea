#!/bin/bash
# GPU tests + kbench A/B of build/var/*.so against the in-tree library + bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/var/*.so > gpurun_out/kb.log 2>&1
rc=$?; echo "kb rc=$rc" >> gpurun_out/kb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-inference --layer-report gpurun_out/layers.json > gpurun_out/bench.json 2> gpurun_out/bench.err
