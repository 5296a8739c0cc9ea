#!/bin/bash
# quick A/B: kernel micro-bench (both env arms) + step, env var $1 in {1,0}; tests of the touched kernels first
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_planar.py tests/test_gpu_fullsize.py tests/test_gpu_network.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/ab2_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ab2_t.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  env $VAR=$v timeout -k 10 150 python scripts/kbench.py > gpurun_out/ab2_kb_$v.log 2>&1 || exit 1
done
for i in 1 2; do for v in 1 0; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 30 --layer-report gpurun_out/ab2_lay_$v.json > gpurun_out/ab2_b_$v.$i.json 2>gpurun_out/ab2_b.err || exit 1
done; done
