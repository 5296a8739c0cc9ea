#!/bin/bash
# level-1 wide wgrad channel groups: GPU tests touching wgrad, then interleaved step A/B with layer reports
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/wg; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wg/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/wg/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for b in 16 32; do
    B="python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5"
    timeout -k 10 150 $B --layer-report gpurun_out/wg/wide_b${b}_$r.layers.json > gpurun_out/wg/wide_b${b}_$r.json 2>/dev/null || exit $?
    RDN_WG_WIDE=0 timeout -k 10 150 $B --layer-report gpurun_out/wg/old_b${b}_$r.layers.json > gpurun_out/wg/old_b${b}_$r.json 2>/dev/null || exit $?
  done
done
