cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_dwk3
timeout -k 10 300 python scripts/dw_kbench.py build/variants/lib_slow.so build/variants/lib_dpf.so build/variants/lib_slowdpf.so > gpurun_out/r05_dwk3/ab.log 2>&1
