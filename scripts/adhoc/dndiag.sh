cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_dndiag; mkdir -p $O
V=build/variants
timeout -k 10 300 python scripts/dense_kbench.py $V/lib_dnomfma.so $V/lib_dnolds.so $V/lib_dnostore.so $V/lib_dnox.so $V/lib_dnobar.so $V/lib_dmin.so 16 > $O/kb.log 2>&1 || exit $?
