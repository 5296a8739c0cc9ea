cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_d3; mkdir -p $O
RDN_LIB=build/variants/lib_d3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dw.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_d3.log 2>&1 || exit $?
RDN_LIB=build/variants/lib_fix.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dw.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_fix.log 2>&1 || exit $?
DW_SHAPE="h5" timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_fix.so build/variants/lib_d3.so > $O/kb.log 2>&1 || exit $?
DW_SHAPE="h5" DW_BATCH=32 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_fix.so build/variants/lib_d3.so > $O/kb32.log 2>&1 || exit $?
DW_SHAPE="h5" DW_NOTREE=1 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_d3st.so > $O/st.log 2>&1 || exit $?
