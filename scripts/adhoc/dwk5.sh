cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwk5
DW_SHAPE=${DW_SHAPE:-h5} timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_fastall.so build/variants/lib_nogate.so build/variants/lib_noload.so build/variants/lib_nomfma.so > gpurun_out/r05_dwk5/ab.log 2>&1
