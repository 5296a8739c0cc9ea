cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_spill; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_dw.py tests/test_gpu_gateout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
OUT=r05_spill/new bash scripts/base_layers.sh || exit $?
RDN_LIB=build/variants/lib_spill.so OUT=r05_spill/old bash scripts/base_layers.sh || exit $?
OUT=r05_spill/new2 bash scripts/base_layers.sh || exit $?
