cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_hold; mkdir -p $O
RDN_WG_HOLD=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_network.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py tests/test_gpu_ddp.py tests/test_gpu_autograd.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
ROUNDS=2 B32=1 OUT=r05_hold/ab VARIANTS="h0=RDN_WG_HOLD=0;h2=RDN_WG_HOLD=2;h4=RDN_WG_HOLD=4;h8=RDN_WG_HOLD=8" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
