cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_deep; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dw.py tests/test_gpu_fullsize.py tests/test_gpu_gateout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
DW_SHAPE=",16>" timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_deep0.so > $O/kb.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_deep/ab VARIANTS="deep=RDN_NOP=1;deep0=RDN_LIB=build/variants/lib_deep0.so" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
