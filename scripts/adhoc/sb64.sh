cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_sb64; mkdir -p $O
DW_SHAPE="64,16" timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_sb64.so > $O/kb.log 2>&1 || exit $?
