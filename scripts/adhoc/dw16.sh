cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dw16
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw.py tests/test_gpu_gateout.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_dw16/tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_w8.so build/variants/lib_st.so > gpurun_out/r05_dw16/kb.log 2>&1
