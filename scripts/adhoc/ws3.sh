cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_ws3
KB_WGRAD=0 KB_ONLY=L0 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_noload.so build/variants/lib_nomfma.so build/variants/lib_nostore.so > gpurun_out/r05_ws3/kb.log 2>&1
