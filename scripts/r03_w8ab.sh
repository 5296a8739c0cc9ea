cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/wg5
timeout -k 10 300 python scripts/wg_kbench.py build/variants/lib_base.so build/variants/lib_w8s.so build/variants/lib_w8.so gpurun_out/wg5/wg.json > gpurun_out/wg5/wg.log 2>&1 || exit $?
OUT=wg5ab ROUNDS=2 B32=1 VARIANTS="base=RDN_LIB=build/variants/lib_base.so;w8s=RDN_LIB=build/variants/lib_w8s.so" bash scripts/ab_env.sh
