#!/bin/bash
# conv3_glds: GPU suite (default mode), conv micro-bench per mode, interleaved step runs per mode
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/cg_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/cg_t.log; [ $rc -eq 0 ] || exit $rc
for m in 3 1 0; do
  RDN_CONV3_GLDS=$m KB_WGRAD=0 timeout -k 10 150 python scripts/kbench.py > gpurun_out/cg_kb_$m.log 2>&1 || exit 1
done
: > gpurun_out/cg.log
for i in 1 2; do for m in 3 1 0; do
  RDN_CONV3_GLDS=$m timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 --layer-report gpurun_out/cg_lay_$m.json > gpurun_out/cg_b.json 2>/dev/null || exit 1
  echo "$m $(python -c 'import json;print(json.load(open("gpurun_out/cg_b.json"))["value"])')" >> gpurun_out/cg.log
done; done
