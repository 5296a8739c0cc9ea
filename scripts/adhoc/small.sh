cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_small; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_network.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
KB_WGRAD=0 KB_ONLY=L2 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_small0.so > $O/kb.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_small/ab VARIANTS="small=RDN_NOP=1;big16=RDN_BIG_SMALL=0" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
