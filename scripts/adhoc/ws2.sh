cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_ws2
KB_WGRAD=0 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_pf1.so build/variants/lib_pf2.so build/variants/lib_pf3.so > gpurun_out/r05_ws2/kb.log 2>&1
