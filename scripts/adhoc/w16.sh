cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_w16
timeout -k 10 800 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_big.py tests/test_gpu_dense.py tests/test_gpu_dw.py tests/test_gpu_planar.py tests/test_gpu_network.py tests/test_gpu_fullsize.py tests/test_gpu_gateout.py tests/test_gpu_slots.py tests/test_gpu_ddp.py tests/test_gpu_bench.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_w16/tests.log 2>&1 || exit $?
KB_WGRAD=0 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_ws8.so build/variants/lib_big8.so build/variants/lib_base.so > gpurun_out/r05_w16/kb.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_w16/ab VARIANTS="new=RDN_NOP=1;base=RDN_LIB=build/variants/lib_base.so" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
OUT=r05_w16/layers bash scripts/check.sh
