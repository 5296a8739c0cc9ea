cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_wreg; mkdir -p $O
RDN_LIB=build/variants/lib_wreg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dw.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
DW_SHAPE="h5" timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_wreg.so > $O/kb.log 2>&1 || exit $?
DW_SHAPE="h5" DW_BATCH=32 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_wreg.so > $O/kb32.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_wreg/ab VARIANTS="base=RDN_NOP=1;wreg=RDN_LIB=build/variants/lib_wreg.so" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
