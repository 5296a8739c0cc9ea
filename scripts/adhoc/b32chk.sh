cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r05_b32chk; mkdir -p $O
for i in 1 2; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-inference --no-traffic > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
done
