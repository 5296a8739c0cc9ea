cd $GRAFT_REPO_ROOT; O=gpurun_out/r05_met; mkdir -p $O
for m in 1 4 0; do
RDN_METRICS=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_metrics.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$m.log 2>&1 || exit $?
RDN_METRICS=$m timeout -k 10 120 python -c "import bench, torch, json; print(json.dumps(bench.metrics_bench(torch.device('cuda'))))" > $O/metrics_$m.json 2>$O/metrics_$m.err || exit $?
done
