cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwst
DW_SHAPE="80,32" timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_st.so build/variants/lib_st_nostore.so build/variants/lib_st_noepi.so build/variants/lib_st_noload.so > gpurun_out/r05_dwst/st2.log 2>&1
