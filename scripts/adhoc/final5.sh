cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r05_final5; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python bench.py --batch 32 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 > $O/b32_$i.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --batch 16 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 30 --warmup 5 > $O/b16_$i.json 2>/dev/null || exit $?
done
