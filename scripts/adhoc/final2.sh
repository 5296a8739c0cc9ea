cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r05_final1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 20 > $O/prof.log 2>&1 || exit $?
