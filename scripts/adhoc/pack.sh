cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_pack; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_network.py tests/test_gpu_optim.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python scripts/pack_bench.py > $O/pack.json 2>&1 || exit $?
RDN_PACK_ROWS=0 timeout -k 10 120 python scripts/pack_bench.py >> $O/pack.json 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_pack/ab VARIANTS="rows=RDN_NOP=1;units=RDN_PACK_ROWS=0" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
