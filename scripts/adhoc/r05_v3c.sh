cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_v3
timeout -k 10 700 python -u -m pytest tests/test_gpu_forward_graph.py tests/test_gpu_mixed_patch.py tests/test_gpu_synth.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_kernels.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r05_v3/tests2.log 2>&1 || exit $?
KB_WGRAD=0 KB_ONLY=L0 timeout -k 10 300 python scripts/kbench.py vub_image_denoising_amd/librdunet_hip.so build/variants/lib_noload.so build/variants/lib_nomfma.so build/variants/lib_nostore.so > gpurun_out/r05_v3/kb.log 2>&1 || exit $?
timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, '.')
import bench
dev = torch.device('cuda', 0)
print(json.dumps({'rdunet128': bench.rdunet128_forward(dev), 'config1': bench.config1_forward(dev)}))
" > gpurun_out/r05_v3/infer.json 2> gpurun_out/r05_v3/infer.err
