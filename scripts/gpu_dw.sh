#!/bin/bash
# fused level-0 dgrad+wgrad: its own test, the GPU suite, then the train-step bench with a layer report
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dw_t.log 2>&1
rc=$?; echo "dw tests rc=$rc" >> gpurun_out/dw_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --layer-report gpurun_out/layers.json > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err; exit $rc
