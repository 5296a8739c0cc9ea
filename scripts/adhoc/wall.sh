cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_wall; mkdir -p $O
RDN_LIB=build/variants/lib_wall.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dw.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_wall.so > $O/kb.log 2>&1 || exit $?
DW_BATCH=32 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_wall.so > $O/kb32.log 2>&1 || exit $?
