#!/bin/bash
# conv3_wsd (level-0/1 conv, LDS-DMA halo ring + epilogue waves): full GPU suite, then kernel micro-bench and step A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/wsd_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/wsd_t.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  RDN_CONV3_WSD=$v KB_WGRAD=0 timeout -k 10 120 python scripts/kbench.py > gpurun_out/wsd_kb_$v.log 2>&1 || exit 1
done
for i in 1 2; do for v in 1 0; do
  RDN_CONV3_WSD=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 30 --layer-report gpurun_out/wsd_lay_$v.json > gpurun_out/wsd_b_$v.$i.json 2>gpurun_out/wsd_b.err || exit 1
done; done
