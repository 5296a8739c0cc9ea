cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_d3ab; mkdir -p $O
ROUNDS=2 B32=1 OUT=r05_d3ab VARIANTS="base=RDN_NOP=1;d3=RDN_LIB=build/variants/lib_d3.so" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
