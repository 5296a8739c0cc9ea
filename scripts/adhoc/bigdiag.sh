cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_bigdiag
V=build/variants
KB_WGRAD=0 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so $V/lib_bnodma.so $V/lib_bnolds.so $V/lib_bnomfma.so $V/lib_bnobar.so $V/lib_bnoepi.so $V/lib_bmfma.so > gpurun_out/r05_bigdiag/kb.log 2>&1
