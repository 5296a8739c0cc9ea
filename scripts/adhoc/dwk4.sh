cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwk4
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw.py tests/test_gpu_gateout.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_dwk4/tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_dpf.so build/variants/lib_slow.so > gpurun_out/r05_dwk4/ab.log 2>&1
