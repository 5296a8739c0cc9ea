#!/bin/bash
# conv3_big: parity tests, then interleaved step A/B (RDN_BIG=0 vs default) with per-layer reports
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/big; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_ddp.py tests/test_gpu_graph.py tests/test_gpu_optim.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/big/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/big/t.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for b in 16 32; do
    B="python bench.py --batch $b --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5"
    timeout -k 10 150 $B --layer-report gpurun_out/big/big_b${b}_$r.layers.json > gpurun_out/big/big_b${b}_$r.json 2>/dev/null || exit $?
    RDN_BIG=0 timeout -k 10 150 $B --layer-report gpurun_out/big/halo_b${b}_$r.layers.json > gpurun_out/big/halo_b${b}_$r.json 2>/dev/null || exit $?
  done
done
