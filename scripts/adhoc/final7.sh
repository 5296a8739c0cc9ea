cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r05_final7; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python -u bench.py --batch 32 --no-extra --no-cpu-baseline --no-inference --layer-report $O/layers_b32.json > $O/bench_b32.json 2> $O/bench_b32.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 20 > $O/prof.log 2>&1 || exit $?
