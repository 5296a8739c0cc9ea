cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_h5v; mkdir -p $O
RDN_LIB=build/variants/lib_dpf2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dw.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
DW_SHAPE="h5" timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_dpf2.so build/variants/lib_wp2.so build/variants/lib_wp5.so > $O/kb.log 2>&1 || exit $?
DW_SHAPE="h5" DW_BATCH=32 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_dpf2.so build/variants/lib_wp2.so build/variants/lib_wp5.so > $O/kb32.log 2>&1 || exit $?
