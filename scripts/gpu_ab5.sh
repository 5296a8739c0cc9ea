#!/bin/bash
# A/B of the in-tree library against a variant library build/var/$1 (RDN_LIB): GPU tests on the in-tree one,
# conv micro-bench of both in one process, then interleaved step runs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=build/var/$1/librdunet_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/ab5_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ab5_t.log; [ $rc -eq 0 ] || exit $rc
KB_WGRAD=0 timeout -k 10 200 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so $V > gpurun_out/ab5_kb.log 2>&1 || exit 1
: > gpurun_out/ab5.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 --layer-report gpurun_out/ab5_lay_a.json > gpurun_out/ab5_a.json 2>/dev/null || exit 1
  echo "A $(python -c 'import json;print(json.load(open("gpurun_out/ab5_a.json"))["value"])')" >> gpurun_out/ab5.log
  RDN_LIB=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --no-inference --no-extra --steps 40 --layer-report gpurun_out/ab5_lay_b.json > gpurun_out/ab5_b.json 2>/dev/null || exit 1
  echo "B $(python -c 'import json;print(json.load(open("gpurun_out/ab5_b.json"))["value"])')" >> gpurun_out/ab5.log
done
