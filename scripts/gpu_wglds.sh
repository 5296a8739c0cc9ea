#!/bin/bash
# glds weight-gradient kernel: parity tests, then kernel micro-bench and step A/B vs the rows kernel
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_planar.py tests/test_gpu_fullsize.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/wg_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/wg_t.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  RDN_WGLDS=$v KB_CONV=0 timeout -k 10 120 python scripts/kbench.py > gpurun_out/wg_kb_$v.log 2>&1 || exit 1
done
for i in 1 2; do for v in 1 0; do
  RDN_WGLDS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 30 > gpurun_out/wg_b_$v.$i.json 2>gpurun_out/wg_b.err || exit 1
done; done
