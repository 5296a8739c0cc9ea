cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwk2
DW_SHAPE=h5 timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_dpf.so build/variants/lib_nogate.so build/variants/lib_nogate_dpf.so build/variants/lib_noload.so > gpurun_out/r05_dwk2/diag.log 2>&1 || exit $?
DW_SHAPE=h5 DW_NOTREE= PMC_OUT=gpurun_out/r05_dwk2/pmc bash scripts/pmc.sh python scripts/dw_kbench.py
