cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_ws1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_planar.py tests/test_gpu_network.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_ws1/tests.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_ws1/ab VARIANTS="ae=RDN_WS_AE=1;lds=RDN_WS_AE=0" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
for v in 1 0; do RDN_WS_AE=$v timeout -k 10 200 python bench.py --batch 16 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 10 --warmup 3 --layer-report gpurun_out/r05_ws1/ae$v.layers.json > gpurun_out/r05_ws1/ae$v.json 2>/dev/null || exit $?; done
