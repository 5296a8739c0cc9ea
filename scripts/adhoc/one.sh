cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_one; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_network.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
OUT=r05_one/new BATCHES=16 NO_TESTS=1 bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_one0.so OUT=r05_one/old bash scripts/base_layers.sh || exit $?
OUT=r05_one/new2 bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_one0.so OUT=r05_one/old2 bash scripts/base_layers.sh || exit $?
