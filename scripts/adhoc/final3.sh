cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_final3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
