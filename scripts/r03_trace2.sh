cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tr2; export TMPDIR=/tmp
for v in off go; do
  g=0; [ $v = go ] && g=1
  RDN_GATE_OUT=$g RDN_WGRAD_SLOTS=8 timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tr2/$v -o run --output-format csv -- python3 bench.py --batch 16 --no-cpu-baseline --no-inference --no-traffic --no-extra --steps 10 --warmup 3 --layer-report gpurun_out/tr2/$v.layers.json > gpurun_out/tr2/$v.json 2> gpurun_out/tr2/$v.err || exit $?
done
