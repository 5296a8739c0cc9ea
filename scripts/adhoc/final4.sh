cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r05_final4; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
