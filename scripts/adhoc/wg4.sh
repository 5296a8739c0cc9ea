cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_wg4; mkdir -p $O
KB_CONV=0 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_wg4.so > $O/kb.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_wg4/ab VARIANTS="nw8=RDN_NOP=1;nw4=RDN_LIB=build/variants/lib_wg4.so" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
