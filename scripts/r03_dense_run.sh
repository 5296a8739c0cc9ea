OUT=${OUT:-dn}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/$OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ROUNDS=2 B32=1 VARIANTS="off=RDN_DENSE=0;on=RDN_DENSE=1" bash scripts/ab_env.sh
timeout -k 10 150 python bench.py --batch 16 --no-extra --no-cpu-baseline --no-inference --no-traffic --steps 20 --warmup 5 --layer-report gpurun_out/$OUT/b16.layers.json > gpurun_out/$OUT/b16.json 2>/dev/null
