cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_roll; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_metrics.py tests/test_gpu_big.py tests/test_gpu_gateout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import bench, torch, json; print(json.dumps(bench.metrics_bench(torch.device('cuda'))))" > $O/metrics.json 2>$O/metrics.err || exit $?
OUT=r05_roll/new bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_spill.so OUT=r05_roll/old bash scripts/base_layers.sh || exit $?
OUT=r05_roll/new2 bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_spill.so OUT=r05_roll/old2 bash scripts/base_layers.sh || exit $?
