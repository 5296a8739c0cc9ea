cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwst
timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_stamps.so > gpurun_out/r05_dwst/st.log 2>&1
