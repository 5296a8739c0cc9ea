cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_n80; mkdir -p $O
KB_WGRAD=0 KB_ONLY=L2 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_n80.so > $O/kb.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_n80/ab VARIANTS="base=RDN_NOP=1;n80=RDN_LIB=build/variants/lib_n80.so" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
