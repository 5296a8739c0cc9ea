#!/bin/bash
# PSNR parity tests (printed numbers) + rocprofv3 kernel-trace stats of the B16 train-step bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_psnr.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/psnr.log 2>&1
rc=$?; echo "psnr rc=$rc" >> gpurun_out/psnr.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof.err; exit $rc
