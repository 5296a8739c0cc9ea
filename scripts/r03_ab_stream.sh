#!/bin/bash
# new config tests, then interleaved A/B of the weight-gradient side stream (B16, B32)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/cfg.log 2>&1
rc=$?; echo "cfg rc=$rc" >> gpurun_out/cfg.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for b in 16 32; do
    B="python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5"
    timeout -k 10 150 $B > gpurun_out/ab/side_b${b}_$r.json 2>/dev/null || exit $?
    RDN_WGRAD_STREAM=0 timeout -k 10 150 $B > gpurun_out/ab/main_b${b}_$r.json 2>/dev/null || exit $?
  done
done
