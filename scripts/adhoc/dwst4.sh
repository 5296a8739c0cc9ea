cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwst4
DW_SHAPE="h5" DW_NOTREE=1 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_st.so build/variants/lib_st0.so > gpurun_out/r05_dwst4/st.log 2>&1
