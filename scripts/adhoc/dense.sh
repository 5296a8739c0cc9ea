cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_dense; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_network.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
OUT=r05_dense/new bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_dlin.so OUT=r05_dense/old bash scripts/base_layers.sh || exit $?
OUT=r05_dense/new2 bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_dlin.so OUT=r05_dense/old2 bash scripts/base_layers.sh || exit $?
